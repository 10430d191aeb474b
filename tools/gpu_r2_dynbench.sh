#!/bin/bash
# Runtime-shape kernel measurements: L96 d=40 on the compiled vs the runtime path (A/B),
# L96 d=1000 (runtime path only), rocprofv3 kernel statistics of the latter two.
D=gpurun_out/r2dynb
mkdir -p $D
export TMPDIR=/tmp
step() {
  local name=$1 t=$2
  shift 2
  timeout -k 10 $t "$@" > $D/$name.out 2> $D/$name.err
  local rc=$?
  echo "$name rc=$rc" | tee -a $D/steps.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ] && [ $rc -ne 2 ]; then exit $rc; fi
}
step l96_auto 300 python -u bench.py --workload l96 --steps 100 --warmup 10 --no-cpu-baseline --no-ref
step l96_rt 300 python -u bench.py --workload l96 --steps 100 --warmup 10 --no-cpu-baseline --no-ref --kernel-path runtime
step l96_1000 600 python -u bench.py --workload l96_1000
step prof_l96_rt 300 rocprofv3 --kernel-trace --stats -d $D/prof_l96_rt -o run -- python3 bench.py --workload l96 --steps 100 --warmup 10 --no-cpu-baseline --no-ref --kernel-path runtime
step prof_l96_1000 300 rocprofv3 --kernel-trace --stats -d $D/prof_l96_1000 -o run -- python3 bench.py --workload l96_1000 --no-cpu-baseline --no-ref
echo done >> $D/steps.log
