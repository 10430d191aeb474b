#!/bin/bash
# Round-4 measurement call: correctness of the experiment libraries, then same-box A/B
# (build/libpf_hip_<name>.so from tools/build_sv_variants.sh / build_inst_variant.sh).
#   tools/gpu_probe.sh OUTDIR
D=${1:-gpurun_out/probe}
mkdir -p "$D"; . "$(dirname "$0")/gpu_lib.sh"
B=particle_filters_amd/libpf_hip.so
T="-x -q --timeout 280 --timeout-method thread"
PF_EVIDENCE_DIR=$D/ev_base try_step tests_base 600 python -u -m pytest tests/test_gpu_teacher_forced.py::test_step_sv64 tests/test_gpu_teacher_forced.py::test_step_grp_l96_config3 tests/test_gpu_teacher_forced.py::test_step_grp_mat_config4 tests/test_gpu_cov.py $T
PF_LIB=build/libpf_hip_ldspub.so PF_EVIDENCE_DIR=$D/ev_ldspub try_step trace_ldspub 300 python -u -m pytest tests/test_gpu_resident_trace.py $T
PF_LIB=build/libpf_hip_mlds.so PF_EVIDENCE_DIR=$D/ev_mlds try_step tf_mlds 300 python -u -m pytest tests/test_gpu_teacher_forced.py::test_step_sv64 $T
for rep in 1 2; do
  for lib in $B build/libpf_hip_ldspub.so; do
    PF_LIB=$lib step "k1000_$(basename $lib .so)_$rep" 120 python -u bench.py --steps 1000 --warmup 100 --no-cpu-baseline --no-ref
    PF_LIB=$lib step "k20_$(basename $lib .so)_$rep" 120 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-ref
  done
  for lib in build/libpf_hip_nofast.so $B build/libpf_hip_mlds.so; do
    PF_LIB=$lib step "sv64_$(basename $lib .so)_$rep" 180 python -u bench.py --workload sv64 --steps 30 --warmup 5 --no-cpu-baseline --no-ref
  done
done
for ov in 0 1; do
  for wl in l96 mat; do
    PF_COV_OVERLAP=$ov step "${wl}_ov${ov}" 240 python -u bench.py --workload $wl --no-cpu-baseline --no-ref
  done
done
for lib in $B build/libpf_hip_ledhold.so; do
  PF_LIB=$lib step "ledh_$(basename $lib .so)" 180 python -u bench.py --workload ledh --steps 100 --warmup 10 --no-cpu-baseline --no-ref
done
echo done >> "$D/steps.log"
