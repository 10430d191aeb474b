#!/bin/bash
# Round-4: the gather pass of k_step_stream with the next tile's prefix and the next source tile's
# log-weights in flight (AHEAD=1 / 0) vs the committed kernel: stream tests, then same-box sv64 lines.
D=${1:-gpurun_out/r4p}
mkdir -p "$D"; . "$(dirname "$0")/gpu_lib.sh"
B=particle_filters_amd/libpf_hip.so
try_step stream_tests 600 python -u -m pytest tests/test_gpu_stream.py tests/test_gpu_teacher_forced.py::test_step_sv64 -q --timeout 280 --timeout-method thread
for rep in 1 2 3; do
  for lib in $B build/libpf_hip_ahead0.so build/libpf_hip_head.so; do
    PF_LIB=$lib step "sv64_$(basename $lib .so)_$rep" 180 python -u bench.py --workload sv64 --steps 40 --warmup 5 --no-cpu-baseline --no-ref
  done
done
echo done >> "$D/steps.log"
