#!/bin/bash
# The driver's default bench line, three times (single-shot wall-time spread), plus the spawn path.
D=gpurun_out/r2b3
mkdir -p $D
for i in 1 2 3; do
  timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $D/default_$i.json 2> $D/default_$i.err || exit $?
done
timeout -k 10 300 python -u bench.py --gpus 1 --spawn --steps 20 --warmup 5 --no-cpu-baseline --no-ref > $D/spawn.json 2> $D/spawn.err
