#!/bin/bash
# GPU test suite + smoke.   tools/gpu_suite.sh OUTDIR [pytest selection...]
D=${1:-gpurun_out/suite}; shift
mkdir -p "$D"; . "$(dirname "$0")/gpu_lib.sh"
sel=${*:-tests}
step tests 1000 python -u -m pytest $sel -m gpu -v -s --timeout 300 --timeout-method thread
step smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()"
echo done >> "$D/steps.log"
