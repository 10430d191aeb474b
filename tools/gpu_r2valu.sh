#!/bin/bash
# VALU cuts (raw v_log in the fp32 Box-Muller, chunk-max accumulation in k_step): GPU suite, then
# A/B against the previous library (sv64, SV K=20 / K=1000, L96, MAT)
D=gpurun_out/r2valu
mkdir -p $D
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $D/gpu_tests.log 2>&1
rc=$?; echo "tests rc=$rc" >> $D/steps.log; [ $rc -ne 0 ] && exit $rc
for v in prev new prev2 new2; do
  lib=particle_filters_amd/libpf_hip.so; [ ${v#prev} != $v ] && lib=build/libpf_hip_prev.so
  PF_LIB=$lib timeout -k 10 200 python -u bench.py --workload sv64 --steps 50 --warmup 3 --no-cpu-baseline --no-ref > $D/sv64_$v.json 2>/dev/null
  PF_LIB=$lib timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-ref > $D/k20_$v.json 2>/dev/null
  PF_LIB=$lib timeout -k 10 200 python -u bench.py --steps 1000 --warmup 100 --no-cpu-baseline --no-ref > $D/k1000_$v.json 2>/dev/null
  PF_LIB=$lib timeout -k 10 200 python -u bench.py --workload l96 --steps 100 --warmup 10 --no-cpu-baseline --no-ref > $D/l96_$v.json 2>/dev/null
  PF_LIB=$lib timeout -k 10 200 python -u bench.py --workload mat --steps 50 --warmup 5 --no-cpu-baseline --no-ref > $D/mat_$v.json 2>/dev/null
  echo "$v rc=$?" >> $D/steps.log
done
