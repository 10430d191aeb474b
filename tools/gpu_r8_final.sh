# Round-8 measurement pass: GPU tests, smoke, the default bench line (config 2) and the
# workload benches, rocprofv3 kernel stats of each (summaries copied into profiles/r01/r7).
set -e
mkdir -p gpurun_out/r8
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/r8/gpu_tests.log 2>&1
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r8/smoke.log 2>&1
timeout -k 10 300 python -u bench.py > gpurun_out/r8/bench_sv.json 2> gpurun_out/r8/bench_sv.err
for w in l96 mat ledh edh; do
  timeout -k 10 300 python -u bench.py --workload $w > gpurun_out/r8/bench_$w.json 2> gpurun_out/r8/bench_$w.err
done
for w in sv l96 mat ledh edh; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r8/prof_$w -o $w -- python3 bench.py --workload $w --no-cpu-baseline > gpurun_out/r8/prof_$w.log 2>&1
done
