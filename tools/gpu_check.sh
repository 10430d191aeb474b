#!/bin/bash
# Closing check of a tree on the GPU box (what the driver runs at round end, plus a profile):
#   tools/gpu_check.sh OUTDIR [extra bench presets of tools/gpu_bench.sh ...]
# GPU suite (evidence JSON under OUTDIR/evidence), smoke, the driver's bench command, its
# rocprofv3 kernel-trace summary, the no-flag bench, then any extra bench presets.
D=${1:-gpurun_out/check}; shift
mkdir -p "$D"; . "$(dirname "$0")/gpu_lib.sh"
PF_EVIDENCE_DIR=$D/evidence try_step suite 1000 python -u -m pytest tests -m gpu -v -s --timeout 300 --timeout-method thread
step smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()"
step bench_default 300 python -u bench.py --gpus 1 --steps 20 --warmup 5
step prof_default 300 rocprofv3 --kernel-trace --stats -d "$D/prof_default" -o run -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-ref
step bench_noflags 600 python -u bench.py
[ $# -gt 0 ] && bash "$(dirname "$0")/gpu_bench.sh" "$D/extra" "$@"
echo done >> "$D/steps.log"
