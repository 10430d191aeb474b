#!/bin/bash
# A/B of the fp64 line: launch-per-step (PF_PERSIST=0), k_persist, and variant libraries.
#   tools/gpu_persist_ab.sh OUTDIR [variant...]   (variant: build/libpf_hip_<name>.so)
D=${1:-gpurun_out/persist_ab}; shift
mkdir -p "$D"; . "$(dirname "$0")/gpu_lib.sh"
B="python -u bench.py --precision fp64 --steps 20 --warmup 5 --no-cpu-baseline --no-ref"
try_step persist 420 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_persist.py
for i in 1 2; do
  PF_PERSIST=0 step "kstep_$i" 120 $B
  step "persist_$i" 120 $B
  for v in "$@"; do PF_LIB=build/libpf_hip_$v.so step "${v}_$i" 120 $B; done
done
echo done >> "$D/steps.log"
