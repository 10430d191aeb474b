#!/bin/bash
# fp64 one-replicate geometry rule: suite, then default (2 chunks) vs PF_CHUNKS_PER_THREAD=1
D=gpurun_out/r2fp64b
mkdir -p $D
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $D/gpu_tests.log 2>&1
rc=$?; echo "tests rc=$rc" >> $D/steps.log; [ $rc -ne 0 ] && exit $rc
for r in 1 2 3; do
  timeout -k 10 200 python -u bench.py --precision fp64 --steps 20 --warmup 5 --no-cpu-baseline --no-ref > $D/k20_new_$r.json 2>/dev/null
  PF_CHUNKS_PER_THREAD=1 timeout -k 10 200 python -u bench.py --precision fp64 --steps 20 --warmup 5 --no-cpu-baseline --no-ref > $D/k20_old_$r.json 2>/dev/null
  timeout -k 10 200 python -u bench.py --precision fp64 --steps 200 --warmup 5 --no-cpu-baseline --no-ref > $D/k200_new_$r.json 2>/dev/null
  PF_CHUNKS_PER_THREAD=1 timeout -k 10 200 python -u bench.py --precision fp64 --steps 200 --warmup 5 --no-cpu-baseline --no-ref > $D/k200_old_$r.json 2>/dev/null
  echo "run $r rc=$?" >> $D/steps.log
done
