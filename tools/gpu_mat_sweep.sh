#!/bin/bash
# MAT (config 4, 8 replicates x 1e5 per GPU) over tile sizes (PF_CHUNKS_PER_THREAD x 64 particles).
mkdir -p gpurun_out/matsw
export TMPDIR=/tmp
for c in "$@"; do
  PF_CHUNKS_PER_THREAD=$c timeout -k 10 200 python -u bench.py --workload mat --no-cpu-baseline --steps 60 --warmup 5 \
    > gpurun_out/matsw/c$c.json 2> gpurun_out/matsw/c$c.err || { echo "chunks $c failed: $?"; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/matsw/c$c.json'));print('chunks $c', round(d['ms_per_step']*1e3,1),'us/step value %.3g'%d['value'],'rmse',round(d['rmse'],4),d['config']['geometry'])"
done
