#!/bin/bash
# fp32 sharding W=1 vs W=2 per step, across step-kernel variants.   tools/gpu_r4i.sh OUTDIR
D=${1:-gpurun_out/r4i}
mkdir -p "$D"; . "$(dirname "$0")/gpu_lib.sh"
for lib in particle_filters_amd/libpf_hip.so build/libpf_hip_head.so build/libpf_hip_nomlds.so build/libpf_hip_nofast.so; do
  PF_LIB=$lib step "shards_$(basename $lib .so)" 120 python -u tools/diag_shards.py
done
echo done >> "$D/steps.log"
