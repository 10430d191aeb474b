#!/bin/bash
# Round-4: dot products over the acoustic Jacobian skip its exact-zero velocity columns (compile time)
# the LEDH / EDH / replay tests, then same-box LEDH-MAT (k_flow_wave) and config-5 LEDH lines
# against the previous library (build/libpf_hip_prev.so).
D=${1:-gpurun_out/r4y}
mkdir -p "$D"; . "$(dirname "$0")/gpu_lib.sh"
try_step flow_tests 900 python -u -m pytest -x -v --timeout 280 --timeout-method thread tests/test_gpu_ledh.py tests/test_gpu_edh.py tests/test_gpu_flow_run_replay.py
for rep in 1 2; do
  step "ledh_mat_new_$rep" 300 python -u bench.py --workload ledh_mat --no-cpu-baseline --no-ref
  PF_LIB=build/libpf_hip_prev.so step "ledh_mat_old_$rep" 300 python -u bench.py --workload ledh_mat --no-cpu-baseline --no-ref
done
step ledh_new 300 python -u bench.py --workload ledh --no-cpu-baseline --no-ref
PF_LIB=build/libpf_hip_prev.so step ledh_old 300 python -u bench.py --workload ledh --no-cpu-baseline --no-ref
echo done >> "$D/steps.log"
