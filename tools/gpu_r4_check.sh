#!/bin/bash
# Round-4 last check of the committed tree: GPU suite, smoke, the driver's bench command.
D=${1:-gpurun_out/r4_check}
mkdir -p "$D"; . "$(dirname "$0")/gpu_lib.sh"
try_step suite 1000 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread
step smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()"
step bench_default 300 python -u bench.py --gpus 1 --steps 20 --warmup 5
step bench_noflags 600 python -u bench.py
echo done >> "$D/steps.log"
