#!/bin/bash
# Round-4: the resident launch tests with the interleaved full-grid two-handle case.
D=${1:-gpurun_out/r4t}
mkdir -p "$D"; . "$(dirname "$0")/gpu_lib.sh"
try_step res_launch 600 python -u -m pytest -x -v --timeout 280 --timeout-method thread tests/test_gpu_resident_launch.py
echo done >> "$D/steps.log"
