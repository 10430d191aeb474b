#!/bin/bash
# Round-4: k_step_stream vs k_step bitwise (tests/test_gpu_stream.py), then the whole GPU suite and smoke
# on the closing tree.   tools/gpu_r4o.sh OUTDIR
D=${1:-gpurun_out/r4o}
mkdir -p "$D"; . "$(dirname "$0")/gpu_lib.sh"
try_step stream_tests 600 python -u -m pytest tests/test_gpu_stream.py -v --timeout 280 --timeout-method thread
PF_EVIDENCE_DIR=$D/evidence try_step suite 1000 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread
step smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()"
echo done >> "$D/steps.log"
