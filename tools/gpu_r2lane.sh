#!/bin/bash
# group-step lane exchanges on DPP / permlane: device self-check, GPU suite, L96 / MAT A/B vs HEAD
D=gpurun_out/r2lane
mkdir -p $D
timeout -k 10 60 ./build/lane_check > $D/lane_check.log 2>&1
rc=$?; echo "lane_check rc=$rc" >> $D/steps.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $D/gpu_tests.log 2>&1
rc=$?; echo "tests rc=$rc" >> $D/steps.log; [ $rc -ne 0 ] && exit $rc
for r in 1 2; do for v in prev main; do
  lib=particle_filters_amd/libpf_hip.so; [ $v != main ] && lib=build/libpf_hip_$v.so
  PF_LIB=$lib timeout -k 10 200 python -u bench.py --workload l96 --steps 100 --warmup 10 --no-cpu-baseline --no-ref > $D/l96_${v}_$r.json 2>/dev/null
  PF_LIB=$lib timeout -k 10 200 python -u bench.py --workload mat --steps 50 --warmup 5 --no-cpu-baseline --no-ref > $D/mat_${v}_$r.json 2>/dev/null
  echo "$v $r rc=$?" >> $D/steps.log
done; done
