#!/bin/bash
# Round-4: persistent pipelined fused step (k_step_stream) for the many-replicate fp32 scalar
# launches.  Step-kernel tests with it on, then same-box sv64 lines: stream on / off / 3 waves.
D=${1:-gpurun_out/r4l}
mkdir -p "$D"; . "$(dirname "$0")/gpu_lib.sh"
B=particle_filters_amd/libpf_hip.so
PF_EVIDENCE_DIR=$D/evidence try_step tests 900 python -u -m pytest tests/test_gpu_teacher_forced.py::test_step_sv64 tests/test_gpu_parity.py tests/test_gpu_checkpoint.py tests/test_gpu_distributed.py tests/test_gpu_sharded.py -x -q --timeout 280 --timeout-method thread
for rep in 1 2; do
  step "sv64_stream_$rep" 180 python -u bench.py --workload sv64 --steps 30 --warmup 5 --no-cpu-baseline --no-ref
  PF_STREAM=0 step "sv64_nostream_$rep" 180 python -u bench.py --workload sv64 --steps 30 --warmup 5 --no-cpu-baseline --no-ref
  PF_LIB=build/libpf_hip_stream3.so step "sv64_stream3_$rep" 180 python -u bench.py --workload sv64 --steps 30 --warmup 5 --no-cpu-baseline --no-ref
done
step diag_sv64 180 python -u tools/diag_sv64.py
PF_STREAM=0 step diag_sv64_nostream 180 python -u tools/diag_sv64.py
echo done >> "$D/steps.log"
