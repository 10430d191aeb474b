#!/bin/bash
# sv64 (64 x N=1e6 SV filters, launch-per-step k_step) over tile sizes (chunks per thread).
mkdir -p gpurun_out/sv64
export TMPDIR=/tmp
for c in "$@"; do
  PF_CHUNKS_PER_THREAD=$c timeout -k 10 150 python -u bench.py --workload sv64 --no-cpu-baseline --steps 50 --warmup 5 \
    > gpurun_out/sv64/c$c.json 2> gpurun_out/sv64/c$c.err || { echo "chunks $c failed: $?"; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/sv64/c$c.json'));print('chunks $c', round(d['ms_per_step']*1e3,1),'us/step frac',round(d['roofline']['frac'],3),'value %.3g'%d['value'],'rmse',round(d['rmse'],5),d['config']['geometry'])"
done
