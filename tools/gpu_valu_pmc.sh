#!/bin/bash
# VALU / SALU / LDS instruction counts of the SV resident kernel (bench default) and of the
# sv64 streaming k_step: the instruction-issue floor reported beside the HBM roofline.
set -e
mkdir -p gpurun_out/valu
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES -d gpurun_out/valu/sv -o sv -- python3 bench.py --no-cpu-baseline --steps 1000 --warmup 10 > gpurun_out/valu/sv.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES -d gpurun_out/valu/sv64 -o sv64 -- python3 bench.py --workload sv64 --no-cpu-baseline --steps 10 --warmup 2 > gpurun_out/valu/sv64.log 2>&1
ls -R gpurun_out/valu | head
