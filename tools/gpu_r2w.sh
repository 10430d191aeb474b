#!/bin/bash
# A/B of the scalar step on the 64 x 1e6 SV run: base (HEAD~ lib), DPP record merge, DPP + 5 waves/SIMD.
D=gpurun_out/r2w
mkdir -p $D
step() { echo "$1 rc=$2" >> $D/steps.log; }
for v in base w5; do
PF_LIB=build/libpf_hip_$v.so timeout -k 10 300 python -u tools/diag_sv64.py 64 1000000 20 > $D/sv64_$v.log 2>&1
rc=$?; step sv64_$v $rc; [ $rc -ne 0 ] && exit $rc
done
timeout -k 10 300 python -u tools/diag_sv64.py 64 1000000 20 > $D/sv64_dpp.log 2>&1
rc=$?; step sv64_dpp $rc; [ $rc -ne 0 ] && exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $D/gpu_tests.log 2>&1
rc=$?; step tests $rc
