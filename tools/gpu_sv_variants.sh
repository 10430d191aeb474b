#!/bin/bash
# Resident SV kernel variant sweep: bench line (no CPU leg) per variant library.
mkdir -p gpurun_out/sv_var
export TMPDIR=/tmp
for v in "$@"; do
  PF_LIB=build/libpf_hip_$v.so timeout -k 10 120 python -u bench.py --no-cpu-baseline --steps 1000 --warmup 100 \
    > gpurun_out/sv_var/$v.json 2> gpurun_out/sv_var/$v.err || { echo "variant $v failed: $?"; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/sv_var/$v.json'));print('$v', round(d['ms_per_step']*1e3,3),'us/step frac',round(d['roofline']['frac'],3),'rmse',d['rmse'],'rr',d['resample_rate'],d['roofline'].get('kernel'))"
done
