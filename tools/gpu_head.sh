#!/bin/bash
# k_head (per-replicate heads) round: parity tests + many-replicate benches.
set -e
mkdir -p gpurun_out/head
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread -k "heads or global_cdf or run_equals" > gpurun_out/head/tests.log 2>&1
tail -2 gpurun_out/head/tests.log
for w in $1; do
  for f in 0 1; do
    PF_HEAD=$f timeout -k 10 150 python -u bench.py --workload $w --no-cpu-baseline > gpurun_out/head/${w}_h$f.json 2> gpurun_out/head/${w}_h$f.err
    python -c "import json;d=json.load(open('gpurun_out/head/${w}_h$f.json'));print('$w head=$f', round(d['ms_per_step']*1e3,1),'us/step frac',round(d['roofline']['frac'],3),'value %.3g'%d['value'],'rmse',round(d['rmse'],5))"
  done
done
