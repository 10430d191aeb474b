#!/bin/bash
# raw-v_log Box-Muller + chunk-max accumulation (main) vs raw log only (noadd4) vs the previous
# library: the N=1e6 fp32-vs-reference replay test for both, the full suite on main, sv64 / SV A/B
D=gpurun_out/r2valu2
mkdir -p $D
T=tests/test_gpu_parity.py::test_replay_fp32_bench_config_vs_reference
for v in main noadd4 prev; do
  lib=particle_filters_amd/libpf_hip.so; [ $v != main ] && lib=build/libpf_hip_$v.so
  PF_LIB=$lib timeout -k 10 300 python -u -m pytest $T -s -q --timeout 250 --timeout-method thread > $D/replay_$v.log 2>&1
  echo "replay_$v rc=$?" >> $D/steps.log
done
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $D/gpu_tests.log 2>&1
echo "tests rc=$?" >> $D/steps.log
for r in 1 2; do for v in prev noadd4 main; do
  lib=particle_filters_amd/libpf_hip.so; [ $v != main ] && lib=build/libpf_hip_$v.so
  PF_LIB=$lib timeout -k 10 200 python -u bench.py --workload sv64 --steps 50 --warmup 3 --no-cpu-baseline --no-ref > $D/sv64_${v}_$r.json 2>/dev/null
  PF_LIB=$lib timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-ref > $D/k20_${v}_$r.json 2>/dev/null
  PF_LIB=$lib timeout -k 10 200 python -u bench.py --steps 1000 --warmup 100 --no-cpu-baseline --no-ref > $D/k1000_${v}_$r.json 2>/dev/null
  echo "$v $r rc=$?" >> $D/steps.log
done; done
