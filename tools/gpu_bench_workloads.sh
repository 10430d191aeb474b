set -e
mkdir -p gpurun_out/r2
timeout -k 10 200 python -u bench.py > gpurun_out/r2/bench_sv.json 2> gpurun_out/r2/bench_sv.err
timeout -k 10 200 python -u bench.py --workload l96 > gpurun_out/r2/bench_l96.json 2> gpurun_out/r2/bench_l96.err
timeout -k 10 200 python -u bench.py --workload mat > gpurun_out/r2/bench_mat.json 2> gpurun_out/r2/bench_mat.err
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/r2/prof_l96 -o l96 -- python3 bench.py --workload l96 --no-cpu-baseline > gpurun_out/r2/prof_l96.log 2>&1
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/r2/prof_mat -o mat -- python3 bench.py --workload mat --no-cpu-baseline > gpurun_out/r2/prof_mat.log 2>&1
