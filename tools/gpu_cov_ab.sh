#!/bin/bash
# Overlapped device-loop covariance (pf_engine.hip cov_ovl): GPU tests that check every step's
# covariance, then same-box A/B of the L96 / MAT lines with PF_COV_OVERLAP=0 (serial) vs 1.
#   tools/gpu_cov_ab.sh OUTDIR
D=${1:-gpurun_out/covab}
mkdir -p "$D"; . "$(dirname "$0")/gpu_lib.sh"
PF_EVIDENCE_DIR=$D/evidence step cov_tests 600 python -u -m pytest tests/test_gpu_cov.py tests/test_gpu_teacher_forced.py::test_step_grp_l96_config3 tests/test_gpu_teacher_forced.py::test_step_grp_mat_config4 tests/test_gpu_distributed.py -x -q --timeout 500 --timeout-method thread
for rep in 1 2; do
  for ov in 0 1; do
    for wl in l96 mat; do
      PF_COV_OVERLAP=$ov step "${wl}_ov${ov}_$rep" 240 python -u bench.py --workload $wl --no-cpu-baseline --no-ref
    done
  done
done
echo done >> "$D/steps.log"
