set -e
mkdir -p gpurun_out/r7
timeout -k 10 300 python -u -m pytest tests/test_gpu_ledh.py tests/test_gpu_edh.py -x -v --timeout 120 --timeout-method thread > gpurun_out/r7/fused_tests.log 2>&1
timeout -k 10 300 python -u bench.py --workload ledh --no-cpu-baseline > gpurun_out/r7/bench_ledh_fused.json 2> gpurun_out/r7/bench_ledh_fused.err
timeout -k 10 300 python -u bench.py --workload edh --no-cpu-baseline > gpurun_out/r7/bench_edh_fused.json 2> gpurun_out/r7/bench_edh_fused.err
export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/r7/prof_ledh_fused -o ledh -- python3 bench.py --workload ledh --no-cpu-baseline > gpurun_out/r7/prof_ledh_fused.log 2>&1
