#!/bin/bash
# VALU / SALU / LDS instruction counts of the large-state step kernel (k_step_grp) on the
# L96 (config 3) and MAT (config 4) bench workloads.
set -e
mkdir -p gpurun_out/valu
export TMPDIR=/tmp
for w in l96 mat; do
  timeout -s KILL 150 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES -d gpurun_out/valu/$w -o $w -- python3 bench.py --workload $w --no-cpu-baseline --steps 20 --warmup 2 > gpurun_out/valu/$w.log 2>&1
done
ls -R gpurun_out/valu | head
