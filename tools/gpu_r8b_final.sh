# Round-8 final measurement pass: GPU tests, smoke, bench lines of every workload, rocprofv3
# kernel stats, and the SV resident kernel's HBM traffic PMC passes (FETCH_SIZE / WRITE_SIZE).
set -e
D=gpurun_out/r8b
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > $D/gpu_tests.log 2>&1
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $D/smoke.log 2>&1
timeout -k 10 300 python -u bench.py > $D/bench_sv.json 2> $D/bench_sv.err
for w in l96 mat ledh edh sv64; do
  timeout -k 10 300 python -u bench.py --workload $w > $D/bench_$w.json 2> $D/bench_$w.err
done
for w in sv l96 mat ledh edh; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $D/prof_$w -o $w -- python3 bench.py --workload $w --no-cpu-baseline > $D/prof_$w.log 2>&1
done
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $D/pmc_fetch -o fetch -- python3 bench.py --no-cpu-baseline --steps 200 --warmup 200 > $D/pmc_fetch.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $D/pmc_write -o write -- python3 bench.py --no-cpu-baseline --steps 200 --warmup 200 > $D/pmc_write.log 2>&1
find $D -name "*.csv" | head
