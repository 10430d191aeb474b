set -e
mkdir -p gpurun_out/r7
timeout -k 10 300 python -u -m pytest tests/test_gpu_ledh.py tests/test_gpu_edh.py tests/test_gpu_diag.py -x -v --timeout 120 --timeout-method thread > gpurun_out/r7/fused_tests.log 2>&1
timeout -k 10 300 python -u bench.py --workload ledh --no-cpu-baseline > gpurun_out/r7/bench_ledh_fused.json 2> gpurun_out/r7/bench_ledh_fused.err
PF_LIB=build/libpf_hip_stamps.so timeout -k 10 200 python tools/diag_stamps_ledh.py 10000 > gpurun_out/r7/stamps_ledh.log 2>&1
