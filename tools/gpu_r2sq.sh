#!/bin/bash
# SQ wait / issue counters of the 64 x 1e6 scalar step (k_step) and the L96 step (k_step_grp)
D=gpurun_out/r2sq
mkdir -p $D
export TMPDIR=/tmp
C="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT"
timeout -s KILL 150 rocprofv3 --pmc $C -d $D/sv64 -o sv64 -- python3 bench.py --no-cpu-baseline --no-ref --workload sv64 --steps 20 --warmup 2 > $D/sv64.log 2>&1
echo "sv64 rc=$?" >> $D/steps.log
timeout -s KILL 150 rocprofv3 --pmc $C -d $D/l96 -o l96 -- python3 bench.py --no-cpu-baseline --no-ref --workload l96 --steps 50 --warmup 5 > $D/l96.log 2>&1
echo "l96 rc=$?" >> $D/steps.log
