#!/bin/bash
# L96 lane-group step at 5 waves per SIMD (96 VGPRs + 41 spilled, MAXG 1280): parity, then tile A/B
D=gpurun_out/r2wpe5
mkdir -p $D
PF_LIB=build/libpf_hip_wpe5.so timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu -k "l96 or L96 or grp" tests > $D/tests.log 2>&1
rc=$?; echo "tests rc=$rc" >> $D/steps.log; [ $rc = 0 ] || exit 1
for r in 1 2; do
  timeout -k 10 200 python -u bench.py --workload l96 --no-cpu-baseline --no-ref > $D/l96_main_$r.json 2>/dev/null
  rc=$?; echo "main $r rc=$rc" >> $D/steps.log; [ $rc = 0 ] || exit 1
  PF_LIB=build/libpf_hip_wpe5.so timeout -k 10 200 python -u bench.py --workload l96 --no-cpu-baseline --no-ref > $D/l96_wpe5_$r.json 2>/dev/null
  rc=$?; echo "wpe5 $r rc=$rc" >> $D/steps.log; [ $rc = 0 ] || exit 1
  PF_CHUNKS_PER_THREAD=3 PF_LIB=build/libpf_hip_wpe5.so timeout -k 10 200 python -u bench.py --workload l96 --no-cpu-baseline --no-ref > $D/l96_wpe5t96_$r.json 2>/dev/null
  rc=$?; echo "wpe5t96 $r rc=$rc" >> $D/steps.log; [ $rc = 0 ] || exit 1
  PF_CHUNKS_PER_THREAD=2 PF_LIB=build/libpf_hip_wpe5.so timeout -k 10 200 python -u bench.py --workload l96 --no-cpu-baseline --no-ref > $D/l96_wpe5t64_$r.json 2>/dev/null
  rc=$?; echo "wpe5t64 $r rc=$rc" >> $D/steps.log; [ $rc = 0 ] || exit 1
done
