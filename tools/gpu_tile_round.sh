#!/bin/bash
# Tile rounded to whole chunk-loop passes (default) vs the old geometry (PF_TILE_ROUND=0).
mkdir -p gpurun_out/tr
export TMPDIR=/tmp
for w in l96 mat sv64; do
  for r in 1 0 1 0; do
    PF_TILE_ROUND=$r timeout -k 10 200 python -u bench.py --workload $w --no-cpu-baseline --steps 50 --warmup 5 > gpurun_out/tr/${w}_$r.json 2> gpurun_out/tr/${w}_$r.err || { echo "$w $r failed"; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/tr/${w}_$r.json'));print('$w round=$r', round(d['ms_per_step']*1e3,1),'us/step value %.3g'%d['value'],'rmse',round(d['rmse'],5),d['config']['geometry'])"
  done
done
