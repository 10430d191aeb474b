set -e
mkdir -p gpurun_out/r7
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_sharded.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r7/parity2.log 2>&1
timeout -k 10 300 python -u bench.py --workload l96 --no-cpu-baseline > gpurun_out/r7/bench_l96_stage.json 2> gpurun_out/r7/bench_l96_stage.err
timeout -k 10 300 python -u bench.py --workload mat --no-cpu-baseline > gpurun_out/r7/bench_mat_stage.json 2> gpurun_out/r7/bench_mat_stage.err
PF_LIB=build/libpf_hip_stamps.so timeout -k 10 200 python tools/diag_stamps_grp.py l96 > gpurun_out/r7/stamps_l96.log 2>&1
