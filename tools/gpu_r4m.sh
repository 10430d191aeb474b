#!/bin/bash
# Round-4: k_step_stream at 4 vs 3 waves per SIMD vs k_step (same box), and its issue counters.
D=${1:-gpurun_out/r4m}
mkdir -p "$D"; . "$(dirname "$0")/gpu_lib.sh"
for rep in 1 2; do
  step "sv64_stream_$rep" 180 python -u bench.py --workload sv64 --steps 30 --warmup 5 --no-cpu-baseline --no-ref
  PF_LIB=build/libpf_hip_stream3.so step "sv64_stream3_$rep" 180 python -u bench.py --workload sv64 --steps 30 --warmup 5 --no-cpu-baseline --no-ref
  PF_STREAM=0 step "sv64_nostream_$rep" 180 python -u bench.py --workload sv64 --steps 30 --warmup 5 --no-cpu-baseline --no-ref
done
step diag_sv64 180 python -u tools/diag_sv64.py
step sv64_issue 150 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES -d "$D/sv64_issue" -o sv64 -- \
  python3 bench.py --no-cpu-baseline --no-ref --workload sv64 --steps 20 --warmup 3
try_step sv64_stall 150 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SMEM SQ_WAVE_CYCLES -d "$D/sv64_stall" -o sv64 -- \
  python3 bench.py --no-cpu-baseline --no-ref --workload sv64 --steps 20 --warmup 3
echo done >> "$D/steps.log"
