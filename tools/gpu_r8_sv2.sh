#!/bin/bash
# Resident SV kernel: variant sweep + phase stamps of the current code.
set -e
mkdir -p gpurun_out/r8sv
export TMPDIR=/tmp
bash tools/gpu_sv_variants.sh "$@"
PF_LIB=build/libpf_hip_stamps.so timeout -k 10 200 python -u tools/diag_resident_stamps.py > gpurun_out/r8sv/stamps_resident.log 2>&1
cat gpurun_out/r8sv/stamps_resident.log | head -16
