#!/bin/bash
# Round-4 closing pass, part C: every bench line again after the PMC refresh (the lines read
# profiles/pmc_*.json for roofline.traffic / valu).   tools/gpu_r4_finalC.sh OUTDIR
D=${1:-gpurun_out/r4_finalC}
mkdir -p "$D"; . "$(dirname "$0")/gpu_lib.sh"
step bench_default 300 python -u bench.py --gpus 1 --steps 20 --warmup 5
step bench_k1000 300 python -u bench.py --steps 1000 --warmup 100 --no-cpu-baseline
step bench_fp64 300 python -u bench.py --precision fp64 --steps 20 --warmup 5 --no-cpu-baseline
step bench_sv64 300 python -u bench.py --workload sv64
step bench_l96 300 python -u bench.py --workload l96 --no-cpu-baseline
step bench_mat 300 python -u bench.py --workload mat --no-cpu-baseline
step bench_ledh 300 python -u bench.py --workload ledh --no-cpu-baseline
echo done >> "$D/steps.log"
