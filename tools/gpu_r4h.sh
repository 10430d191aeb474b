#!/bin/bash
# Round-4: source-driven systematic ancestors (lower-bound marks), gather-fast block, split
# gather / non-gather chunk loops.  Full GPU suite, same-box sv64 A/B against the previous step
# kernel, resample overhead and the stamps of a fused gather launch.   tools/gpu_r4h.sh OUTDIR
D=${1:-gpurun_out/r4h}
mkdir -p "$D"; . "$(dirname "$0")/gpu_lib.sh"
B=particle_filters_amd/libpf_hip.so
PF_EVIDENCE_DIR=$D/evidence try_step suite 900 python -u -m pytest tests -m gpu -x -q --timeout 280 --timeout-method thread
for rep in 1 2; do
  for lib in $B build/libpf_hip_head.so; do
    PF_LIB=$lib step "sv64_$(basename $lib .so)_$rep" 180 python -u bench.py --workload sv64 --steps 30 --warmup 5 --no-cpu-baseline --no-ref
  done
done
step diag_sv64 180 python -u tools/diag_sv64.py
PF_LIB=build/libpf_hip_stamps.so step diag_sv64_stamps 240 python -u tools/diag_sv64.py
echo done >> "$D/steps.log"
