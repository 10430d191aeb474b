#!/bin/bash
# Full GPU suite + smoke + the L96/MAT bench lines after the many-replicate tile rounding.
set -e
D=gpurun_out/r8c
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > $D/gpu_tests.log 2>&1 || { tail -30 $D/gpu_tests.log; exit 1; }
tail -1 $D/gpu_tests.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $D/smoke.log 2>&1
tail -1 $D/smoke.log
for w in mat l96 sv; do
  timeout -k 10 300 python -u bench.py --workload $w > $D/bench_$w.json 2> $D/bench_$w.err
  python -c "import json;d=json.load(open('$D/bench_$w.json'));print('$w', round(d['ms_per_step']*1e3,1),'us/step value %.3g'%d['value'],'frac',round(d['roofline']['frac'],3),d['config']['geometry'])"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $D/prof_mat -o mat -- python3 bench.py --workload mat --no-cpu-baseline > $D/prof_mat.log 2>&1
