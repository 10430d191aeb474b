#!/bin/bash
# Round-4: a fresh record of the nonlinear-h LEDH path (the MAT notebook's joint run, k_flow_wave):
# bench line and rocprofv3 kernel statistics.
D=${1:-gpurun_out/r4u}
mkdir -p "$D"; . "$(dirname "$0")/gpu_lib.sh"
step bench_ledh_mat 600 python -u bench.py --workload ledh_mat
step prof_ledh_mat 600 rocprofv3 --kernel-trace --stats -d "$D/prof_ledh_mat" -o run -- python3 bench.py --workload ledh_mat --no-cpu-baseline --no-ref
echo done >> "$D/steps.log"
