#!/bin/bash
# sv64 (64 x 1e6 SV, launch-per-step k_step) bench per variant library.
mkdir -p gpurun_out/sv64v
export TMPDIR=/tmp
for v in "$@"; do
  lib=build/libpf_hip_$v.so; [ "$v" = "default" ] && lib=particle_filters_amd/libpf_hip.so
  PF_LIB=$lib timeout -k 10 150 python -u bench.py --workload sv64 --no-cpu-baseline --steps 50 --warmup 5 \
    > gpurun_out/sv64v/$v.json 2> gpurun_out/sv64v/$v.err || { echo "variant $v failed: $?"; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/sv64v/$v.json'));print('$v', round(d['ms_per_step']*1e3,1),'us/step frac',round(d['roofline']['frac'],3),'value %.3g'%d['value'],'rmse',round(d['rmse'],5))"
done
