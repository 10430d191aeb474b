set -e
mkdir -p gpurun_out/r7
timeout -k 10 300 python -u bench.py --workload edh > gpurun_out/r7/bench_edh.json 2> gpurun_out/r7/bench_edh.err
timeout -k 10 300 python -u bench.py --workload ledh > gpurun_out/r7/bench_ledh.json 2> gpurun_out/r7/bench_ledh.err
timeout -k 10 300 python -u bench.py --workload l96 > gpurun_out/r7/bench_l96.json 2> gpurun_out/r7/bench_l96.err
timeout -k 10 300 python -u bench.py --workload mat > gpurun_out/r7/bench_mat.json 2> gpurun_out/r7/bench_mat.err
export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/r7/prof_edh -o edh -- python3 bench.py --workload edh --no-cpu-baseline > gpurun_out/r7/prof_edh.log 2>&1
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/r7/prof_l96 -o l96 -- python3 bench.py --workload l96 --no-cpu-baseline > gpurun_out/r7/prof_l96.log 2>&1
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/r7/prof_mat -o mat -- python3 bench.py --workload mat --no-cpu-baseline > gpurun_out/r7/prof_mat.log 2>&1
