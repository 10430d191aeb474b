#!/bin/bash
# Round-4: k_step_stream at 5 waves per SIMD (96 VGPRs, a few spills in the loop) vs 4, same box.
D=${1:-gpurun_out/r4n}
mkdir -p "$D"; . "$(dirname "$0")/gpu_lib.sh"
for rep in 1 2 3; do
  step "sv64_stream_$rep" 180 python -u bench.py --workload sv64 --steps 30 --warmup 5 --no-cpu-baseline --no-ref
  PF_LIB=build/libpf_hip_stream5.so step "sv64_stream5_$rep" 180 python -u bench.py --workload sv64 --steps 30 --warmup 5 --no-cpu-baseline --no-ref
done
echo done >> "$D/steps.log"
