#!/bin/bash
# rounds-aware tile rule: GPU suite, MAT 8 x 1e5 and 64 x 1e5 lines
D=gpurun_out/r2mattile2
mkdir -p $D
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $D/gpu_tests.log 2>&1
rc=$?; echo "tests rc=$rc" >> $D/steps.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py --workload mat > $D/bench_mat.json 2> $D/bench_mat.err
echo "mat rc=$?" >> $D/steps.log
timeout -k 10 300 python -u bench.py --workload mat --replicates-total 64 --steps 40 --warmup 4 --no-cpu-baseline --no-ref > $D/bench_mat64.json 2>/dev/null
echo "mat64 rc=$?" >> $D/steps.log
