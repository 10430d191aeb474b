set -e
mkdir -p gpurun_out/r7
timeout -k 10 300 python -u bench.py --workload l96 --no-cpu-baseline > gpurun_out/r7/bench_l96_qdiag.json 2>/dev/null
PF_LIB=build/libpf_hip_noqdiag.so timeout -k 10 300 python -u bench.py --workload l96 --no-cpu-baseline > gpurun_out/r7/bench_l96_noqdiag.json 2>/dev/null
