#!/bin/bash
# Large-state (k_step_grp) tile-size sweep: chunks per thread -> particles per workgroup.
#   tools/gpu_grp_sweep.sh l96 "1 4 8 12 16"
mkdir -p gpurun_out/grp
export TMPDIR=/tmp
w=$1
for c in $2; do
  PF_CHUNKS_PER_THREAD=$c timeout -k 10 150 python -u bench.py --workload $w --no-cpu-baseline \
    > gpurun_out/grp/${w}_c$c.json 2> gpurun_out/grp/${w}_c$c.err || { echo "$w chunks $c failed: $?"; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/grp/${w}_c$c.json'));print('$w chunks $c', round(d['ms_per_step']*1e3,1),'us/step frac',round(d['roofline']['frac'],3),'value %.3g'%d['value'],'rmse',round(d['rmse'],5),'rr',d['resample_rate'],d['config']['geometry'])"
done
