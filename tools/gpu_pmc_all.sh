#!/bin/bash
# HBM traffic PMC passes (FETCH_SIZE and WRITE_SIZE in separate runs, MI355X_MICROARCH.md HBM
# section) for the dominant kernel of every SIR bench workload; folded into
# profiles/pmc_traffic*.json by tools/pmc_summary.py afterwards (on the build host).
# The resident SV kernel runs its default plain launch (a cooperative launch crashes rocprofv3
# at process exit: tools/coop_min.hip reproduces that without this engine).
D=gpurun_out/pmc_r2
mkdir -p $D
export TMPDIR=/tmp
run() {  # run <name> <counter> <bench args...>
  local name=$1 ctr=$2
  shift 2
  timeout -s KILL 120 rocprofv3 --pmc $ctr --output-format csv -d $D/${name}_$ctr -o $name -- \
    python3 bench.py --no-cpu-baseline --no-ref "$@" > $D/${name}_$ctr.log 2>&1
  local rc=$?
  echo "$name $ctr rc=$rc" | tee -a $D/steps.log
  if [ $rc -ne 0 ]; then exit $rc; fi
}
sq() {  # sq <name> "<counters>" <bench args...>: SQ instruction / wait counters (rocpd database)
  local name=$1 ctrs=$2
  shift 2
  timeout -s KILL 150 rocprofv3 --pmc $ctrs -d $D/$name -o $name -- python3 bench.py --no-cpu-baseline "$@" \
    > $D/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc" | tee -a $D/steps.log
  if [ $rc -ne 0 ]; then exit $rc; fi
}
for c in FETCH_SIZE WRITE_SIZE; do
  run sv $c --steps 200 --warmup 20
  run sv64 $c --workload sv64 --steps 20 --warmup 2
  run l96 $c --workload l96 --steps 50 --warmup 5
  run mat $c --workload mat --steps 20 --warmup 2
done
ISSUE="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES"
WAIT="SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS"
sq sv_issue "$ISSUE" --steps 200 --warmup 20
sq sv_wait "$WAIT" --steps 200 --warmup 20
sq ledh_issue "$ISSUE" --workload ledh --steps 50 --warmup 5
sq ledh_wait "$WAIT" --workload ledh --steps 50 --warmup 5
sq ledhmat_issue "$ISSUE" --workload ledh_mat --steps 6 --warmup 1
sq ledhmat_wait "$WAIT" --workload ledh_mat --steps 6 --warmup 1
echo done >> $D/steps.log
