#!/bin/bash
# Resident SV kernel: parity tests on the in-tree library, then the variant sweep.
set -e
mkdir -p gpurun_out/r8sv
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_resident.py tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread > gpurun_out/r8sv/tests.log 2>&1 || { tail -30 gpurun_out/r8sv/tests.log; exit 1; }
tail -3 gpurun_out/r8sv/tests.log
bash tools/gpu_sv_variants.sh "$@"
