#!/bin/bash
# Round-4 sv64 diagnosis: resample overhead (thresh 0.5 vs 0), per-phase stamps, A/B of the generic
# loop's max-first stash, and issue/stall counters of the step kernel.   tools/gpu_r4f.sh OUTDIR
D=${1:-gpurun_out/r4f}
mkdir -p "$D"; . "$(dirname "$0")/gpu_lib.sh"
B=particle_filters_amd/libpf_hip.so
step diag_sv64 180 python -u tools/diag_sv64.py
PF_LIB=build/libpf_hip_stamps.so step diag_sv64_stamps 180 python -u tools/diag_sv64.py
for rep in 1 2; do
  for lib in $B build/libpf_hip_nostash.so; do
    PF_LIB=$lib step "sv64_$(basename $lib .so)_$rep" 180 python -u bench.py --workload sv64 --steps 30 --warmup 5 --no-cpu-baseline --no-ref
  done
done
step sv64_issue 150 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES -d "$D/sv64_issue" -o sv64 -- \
  python3 bench.py --no-cpu-baseline --no-ref --workload sv64 --steps 20 --warmup 3
try_step sv64_stall 150 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SMEM SQ_WAVE_CYCLES -d "$D/sv64_stall" -o sv64 -- \
  python3 bench.py --no-cpu-baseline --no-ref --workload sv64 --steps 20 --warmup 3
echo done >> "$D/steps.log"
