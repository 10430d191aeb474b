#!/bin/bash
# L96 config-3 bench line with its rmse_vs_ref leg (NumPy oracle on the engine's Philox draws)
D=gpurun_out/r2l96ref
mkdir -p $D
timeout -k 10 900 python -u bench.py --workload l96 > $D/bench_l96.json 2> $D/bench_l96.err
echo "l96 rc=$?" >> $D/steps.log
