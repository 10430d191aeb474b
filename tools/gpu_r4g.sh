#!/bin/bash
# Round-4: source-driven systematic ancestors + gather-fast block in k_step.  Full GPU suite, sv64
# lines, resample overhead and the stamps of a fused gather launch.   tools/gpu_r4g.sh OUTDIR
D=${1:-gpurun_out/r4g}
mkdir -p "$D"; . "$(dirname "$0")/gpu_lib.sh"
PF_EVIDENCE_DIR=$D/evidence try_step suite 900 python -u -m pytest tests -m gpu -x -q --timeout 280 --timeout-method thread
for rep in 1 2; do
  step "sv64_$rep" 180 python -u bench.py --workload sv64 --steps 30 --warmup 5 --no-cpu-baseline --no-ref
done
step diag_sv64 180 python -u tools/diag_sv64.py
PF_LIB=build/libpf_hip_stamps.so step diag_sv64_stamps 240 python -u tools/diag_sv64.py
echo done >> "$D/steps.log"
