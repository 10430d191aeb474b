#!/bin/bash
# Shared step runner of the tools/gpu_*.sh scripts: every GPU step under its own time limit,
# output to $D/<name>.out/.err, the script stops at the first failing step (no retries).
export TMPDIR=/tmp
step() {  # step <name> <seconds> <command...>
  local name=$1 t=$2
  shift 2
  timeout -k 10 "$t" "$@" > "$D/$name.out" 2> "$D/$name.err"
  local rc=$?
  echo "$name rc=$rc" | tee -a "$D/steps.log"
  if [ $rc -ne 0 ]; then exit $rc; fi
}
# like step, but a test failure (exit status 1) is logged and the script goes on; any other
# non-zero status (time limit, abort, fault) still ends it
try_step() {  # try_step <name> <seconds> <command...>
  local name=$1 t=$2
  shift 2
  timeout -k 10 "$t" "$@" > "$D/$name.out" 2> "$D/$name.err"
  local rc=$?
  echo "$name rc=$rc" | tee -a "$D/steps.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
}
