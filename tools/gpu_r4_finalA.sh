#!/bin/bash
# Round-4 closing pass, part A: the GPU suite + smoke, the headline bench lines and the rocprofv3
# kernel statistics of the default line.   tools/gpu_r4_finalA.sh OUTDIR
D=${1:-gpurun_out/r4_finalA}
mkdir -p "$D"; . "$(dirname "$0")/gpu_lib.sh"
PF_EVIDENCE_DIR=$D/evidence try_step tests 1000 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread
step smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()"
step bench_default 300 python -u bench.py --gpus 1 --steps 20 --warmup 5
step bench_k1000 300 python -u bench.py --steps 1000 --warmup 100 --no-cpu-baseline
step bench_fp64 300 python -u bench.py --precision fp64 --steps 20 --warmup 5 --no-cpu-baseline
step prof_default 300 rocprofv3 --kernel-trace --stats -d "$D/prof_default" -o run -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-ref
echo done >> "$D/steps.log"
