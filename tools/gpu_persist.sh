#!/bin/bash
# The persistent fp64 kernel: its bitwise tests against the launch-per-step loop, the fp64 parity
# tests that now run through it, and the fp64 bench line.   tools/gpu_persist.sh OUTDIR [bench]
D=${1:-gpurun_out/persist}
mkdir -p "$D"; . "$(dirname "$0")/gpu_lib.sh"
PYT="python -u -m pytest -x -v --timeout 200 --timeout-method thread"
try_step persist 420 $PYT tests/test_gpu_persist.py
try_step fp64_tests 400 $PYT tests/test_gpu_teacher_forced.py tests/test_gpu_parity.py -k fp64
if [ "$2" = bench ]; then
  step bench_fp64 200 python -u bench.py --precision fp64 --steps 20 --warmup 5 --no-cpu-baseline
  step prof_fp64 200 rocprofv3 --kernel-trace --stats -d "$D/prof_fp64" -o run -- python3 bench.py --precision fp64 --steps 20 --warmup 5 --no-cpu-baseline --no-ref
fi
echo done >> "$D/steps.log"
