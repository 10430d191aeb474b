#!/bin/bash
# Round-4: the grid-order event recorded lazily (only when a grid comes on another stream): wall
# anatomy (markers vs dispatch-stamped timing events), the tests that exercise the order (resident
# launch, two handles, fused LEDH), and driver bench lines with either timing mode.
D=${1:-gpurun_out/r4s}
mkdir -p "$D"; . "$(dirname "$0")/gpu_lib.sh"
step wall 300 python -u tools/diag_wall.py
try_step order_tests 900 python -u -m pytest -x -v --timeout 280 --timeout-method thread tests/test_gpu_resident_launch.py tests/test_gpu_resident_oracle.py tests/test_gpu_ledh.py
for rep in 1 2 3; do
  step "bench_$rep" 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-ref
  PF_EXT_EVENTS=0 step "bench_markers_$rep" 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-ref
done
echo done >> "$D/steps.log"
