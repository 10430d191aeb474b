#!/bin/bash
# Round-4 check of the fp32 scalar step changes + resident phase stamps.   tools/gpu_r4e.sh OUTDIR
D=${1:-gpurun_out/r4e}
mkdir -p "$D"; . "$(dirname "$0")/gpu_lib.sh"
T="-q --timeout 280 --timeout-method thread"
PF_EVIDENCE_DIR=$D/evidence try_step tests 900 python -u -m pytest tests/test_gpu_teacher_forced.py tests/test_gpu_checkpoint.py tests/test_gpu_parity.py tests/test_gpu_resident_trace.py tests/test_gpu_resident.py $T
for rep in 1 2; do
  step "sv64_$rep" 180 python -u bench.py --workload sv64 --steps 30 --warmup 5 --no-cpu-baseline --no-ref
  step "k20_$rep" 120 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-ref
done
PF_LIB=build/libpf_hip_stamps.so step stamps_T1000 120 python -u tools/diag_resident_stamps.py 1000000 1000
PF_LIB=build/libpf_hip_stamps.so step stamps_T20 120 python -u tools/diag_resident_stamps.py 1000000 20
echo done >> "$D/steps.log"
