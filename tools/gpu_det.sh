set -e
mkdir -p gpurun_out/r7/det
timeout -k 10 200 python -u bench.py --workload mat --no-cpu-baseline --steps 60 --warmup 5 > gpurun_out/r7/det/mat_new.json 2>/dev/null
PF_LIB=build/libpf_hip_prev.so timeout -k 10 200 python -u bench.py --workload mat --no-cpu-baseline --steps 60 --warmup 5 > gpurun_out/r7/det/mat_prev.json 2>/dev/null
timeout -k 10 200 python -u bench.py --workload l96 --no-cpu-baseline --steps 60 --warmup 5 > gpurun_out/r7/det/l96_new.json 2>/dev/null
PF_LIB=build/libpf_hip_prev.so timeout -k 10 200 python -u bench.py --workload l96 --no-cpu-baseline --steps 60 --warmup 5 > gpurun_out/r7/det/l96_prev.json 2>/dev/null
