#!/bin/bash
# resident loop top: snapshot frame / step in registers (main) vs in LDS (prev)
D=gpurun_out/r2sf
mkdir -p $D
timeout -k 10 300 python -u -m pytest tests/test_gpu_resident.py tests/test_gpu_resident_oracle.py tests/test_gpu_resident_launch.py -x -q --timeout 250 --timeout-method thread > $D/tests.log 2>&1
echo "tests rc=$?" >> $D/steps.log
for r in 1 2 3; do for v in prev main; do
  lib=particle_filters_amd/libpf_hip.so; [ $v != main ] && lib=build/libpf_hip_$v.so
  PF_LIB=$lib timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-ref > $D/k20_${v}_$r.json 2>/dev/null
  PF_LIB=$lib timeout -k 10 200 python -u bench.py --steps 1000 --warmup 100 --no-cpu-baseline --no-ref > $D/k1000_${v}_$r.json 2>/dev/null
  echo "$v $r rc=$?" >> $D/steps.log
done; done
