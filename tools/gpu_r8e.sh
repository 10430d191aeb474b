#!/bin/bash
# Round-8 closing pass: full GPU suite, smoke, sv / sv64 bench lines, sv64 kernel stats.
set -e
D=gpurun_out/r8e
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > $D/gpu_tests.log 2>&1 || { tail -30 $D/gpu_tests.log; exit 1; }
tail -1 $D/gpu_tests.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $D/smoke.log 2>&1
tail -1 $D/smoke.log
for w in sv sv64; do
  timeout -k 10 300 python -u bench.py --workload $w > $D/bench_$w.json 2> $D/bench_$w.err
  python -c "import json;d=json.load(open('$D/bench_$w.json'));print('$w', round(d['ms_per_step']*1e3,1),'us/step value %.3g'%d['value'],'frac',round(d['roofline']['frac'],3),d['config']['geometry'])"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $D/prof_sv64 -o sv64 -- python3 bench.py --workload sv64 --no-cpu-baseline --steps 50 --warmup 5 > $D/prof_sv64.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $D/prof_sv -o sv -- python3 bench.py --no-cpu-baseline > $D/prof_sv.log 2>&1
