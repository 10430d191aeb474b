#!/bin/bash
# Round-2 first GPU pass: full GPU suite (incl. the resident-kernel-vs-oracle and RCCL tests),
# smoke, the driver-config SV bench (cooperative and plain launch), the spawn path, and
# rocprofv3 kernel statistics at the driver's --steps 20 and at T = 1000.
# A step that exits 1 (test / assertion failure) lets the pass go on; any other non-zero
# status (fault, abort, time limit) ends it.
D=gpurun_out/r2a
mkdir -p $D
export TMPDIR=/tmp
step() {  # step <name> <timeout> <cmd...>
  local name=$1 t=$2
  shift 2
  timeout -k 10 $t "$@" > $D/$name.out 2> $D/$name.err
  local rc=$?
  echo "$name rc=$rc" | tee -a $D/steps.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
}
step gpu_tests 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread
step smoke 200 python -u -c "import __graft_entry__ as g; g.smoke()"
step bench_sv_k20 300 python -u bench.py --steps 20 --warmup 5
step bench_sv_k20_plain 300 env PF_COOP=0 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-ref
step bench_spawn1 300 python -u bench.py --gpus 1 --spawn --steps 20 --warmup 5 --no-cpu-baseline
step bench_gpus2_refuse 120 bash -c 'python -u bench.py --gpus 2 --steps 20 --warmup 5; echo exit=$?'
step bench_sv_fp64 300 python -u bench.py --steps 20 --warmup 5 --precision fp64 --no-cpu-baseline
step prof_k20 300 rocprofv3 --kernel-trace --stats -d $D/prof_k20 -o sv -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-ref
step prof_k1000 300 rocprofv3 --kernel-trace --stats -d $D/prof_k1000 -o sv -- python3 bench.py --steps 1000 --warmup 100 --no-cpu-baseline --no-ref
echo done >> $D/steps.log
