#!/bin/bash
# MAT 8 x 1e5 tile sweep (64-particle chunk passes per tile) at the lane-local kernel
D=gpurun_out/r2mattile
mkdir -p $D
for r in 1 2; do for c in 4 5 6 7 8; do
  PF_CHUNKS_PER_THREAD=$c timeout -k 10 200 python -u bench.py --workload mat --steps 50 --warmup 5 --no-cpu-baseline --no-ref > $D/mat_c${c}_$r.json 2>/dev/null
  echo "c$c $r rc=$?" >> $D/steps.log
done; done
for c in 4 7; do
  PF_CHUNKS_PER_THREAD=$c timeout -k 10 300 python -u bench.py --workload mat --replicates-total 64 --steps 20 --warmup 2 --no-cpu-baseline --no-ref > $D/mat64_c${c}.json 2>/dev/null
  echo "mat64 c$c rc=$?" >> $D/steps.log
done
