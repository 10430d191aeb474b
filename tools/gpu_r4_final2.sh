#!/bin/bash
# Round-4 closing pass after the timing / grid-order change: GPU suite, smoke, the driver's bench
# command, the no-flag bench, and the rocprofv3 kernel statistics of the driver's command.
D=${1:-gpurun_out/r4_final2}
mkdir -p "$D"; . "$(dirname "$0")/gpu_lib.sh"
try_step suite 1000 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread
step smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()"
step bench_default 300 python -u bench.py --gpus 1 --steps 20 --warmup 5
step prof_default 300 rocprofv3 --kernel-trace --stats -d "$D/prof_default" -o run -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-ref
step bench_noflags 600 python -u bench.py
echo done >> "$D/steps.log"
