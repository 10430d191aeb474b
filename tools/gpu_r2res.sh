#!/bin/bash
# resident kernel flag variants: granule replicas, publishing wave, priorities (K=20 / K=1000)
D=gpurun_out/r2res
mkdir -p $D
for r in 1 2; do for v in main rc4 rc2 young pubw4 sticky; do
  lib=particle_filters_amd/libpf_hip.so; [ $v != main ] && lib=build/libpf_hip_$v.so
  PF_LIB=$lib timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-ref > $D/k20_${v}_$r.json 2>/dev/null
  PF_LIB=$lib timeout -k 10 200 python -u bench.py --steps 1000 --warmup 100 --no-cpu-baseline --no-ref > $D/k1000_${v}_$r.json 2>/dev/null
  echo "$v $r rc=$?" >> $D/steps.log
done; done
