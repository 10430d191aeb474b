#!/bin/bash
# Second-chunk prefetch in the scalar k_step: parity (fp64 replay vs the reference at two-pass
# tiles) + sv64 A/B.
set -e
mkdir -p gpurun_out/pre1
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pre1/tests.log 2>&1 || { tail -30 gpurun_out/pre1/tests.log; exit 1; }
tail -1 gpurun_out/pre1/tests.log
bash tools/gpu_sv64_var.sh pre1 nopre1 pre1 nopre1
