#!/bin/bash
# Round-4: wall-time anatomy of the driver's K = 20 job with the resident launch stamping its own
# timing events (hipExtLaunchKernel) vs marker packets, with and without the grid-order event;
# then the resident tests and the driver's bench command.
D=${1:-gpurun_out/r4r}
mkdir -p "$D"; . "$(dirname "$0")/gpu_lib.sh"
step wall 300 python -u tools/diag_wall.py
PF_NO_ORDER=1 step wall_noorder 300 python -u tools/diag_wall.py
try_step res_tests 600 python -u -m pytest -x -v --timeout 280 --timeout-method thread tests/test_gpu_resident_launch.py tests/test_gpu_resident_oracle.py
for rep in 1 2 3; do
  step "bench_$rep" 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-ref
  PF_EXT_EVENTS=0 step "bench_markers_$rep" 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-ref
done
step bench_full 400 python -u bench.py --gpus 1 --steps 20 --warmup 5
echo done >> "$D/steps.log"
