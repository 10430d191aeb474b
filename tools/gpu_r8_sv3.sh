#!/bin/bash
# Resident SV kernel: resident parity tests on the in-tree library, variant sweep, phase stamps.
set -e
mkdir -p gpurun_out/r8sv
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_resident.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r8sv/tests3.log 2>&1 || { tail -30 gpurun_out/r8sv/tests3.log; exit 1; }
tail -1 gpurun_out/r8sv/tests3.log
bash tools/gpu_sv_variants.sh "$@"
PF_LIB=build/libpf_hip_stamps.so timeout -k 10 200 python -u tools/diag_resident_stamps.py > gpurun_out/r8sv/stamps3.log 2>&1
head -16 gpurun_out/r8sv/stamps3.log
