#!/bin/bash
# Round-4 closing pass, part B: the other configurations' bench lines (with their CPU legs) and the
# rocprofv3 kernel statistics of the sv64 line.   tools/gpu_r4_finalB.sh OUTDIR
D=${1:-gpurun_out/r4_finalB}
mkdir -p "$D"; . "$(dirname "$0")/gpu_lib.sh"
step bench_sv64 300 python -u bench.py --workload sv64
step bench_l96 300 python -u bench.py --workload l96
step bench_mat 300 python -u bench.py --workload mat
step bench_ledh 300 python -u bench.py --workload ledh
step bench_edh 300 python -u bench.py --workload edh
step prof_sv64 300 rocprofv3 --kernel-trace --stats -d "$D/prof_sv64" -o run -- python3 bench.py --workload sv64 --no-cpu-baseline --no-ref
echo done >> "$D/steps.log"
