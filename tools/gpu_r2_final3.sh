#!/bin/bash
# Round-2 closing pass, session 3 (after the rounds-aware MAT tile): GPU suite, smoke, every
# bench line, kernel statistics of the default / MAT lines, and the MAT step's PMC passes
# (its geometry changed: FETCH_SIZE, WRITE_SIZE, SQ issue counters in separate runs).
D=gpurun_out/r2final3
mkdir -p $D
export TMPDIR=/tmp
step() {
  local name=$1 t=$2
  shift 2
  timeout -k 10 $t "$@" > $D/$name.out 2> $D/$name.err
  local rc=$?
  echo "$name rc=$rc" | tee -a $D/steps.log
  if [ $rc -ne 0 ]; then exit $rc; fi
}
step tests 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread
step smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()"
step bench_default 300 python -u bench.py --gpus 1 --steps 20 --warmup 5
step bench_k1000 300 python -u bench.py --steps 1000 --warmup 100 --no-cpu-baseline
step bench_fp64 300 python -u bench.py --precision fp64 --steps 20 --warmup 5 --no-cpu-baseline
step bench_sv64 300 python -u bench.py --workload sv64
step bench_l96 300 python -u bench.py --workload l96
step bench_mat 300 python -u bench.py --workload mat
step bench_mat64 300 python -u bench.py --workload mat --replicates-total 64 --steps 40 --warmup 4 --no-cpu-baseline --no-ref
step bench_ledh 300 python -u bench.py --workload ledh
step bench_edh 300 python -u bench.py --workload edh
step prof_default 300 rocprofv3 --kernel-trace --stats -d $D/prof_default -o run -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-ref
step prof_mat 300 rocprofv3 --kernel-trace --stats -d $D/prof_mat -o run -- python3 bench.py --workload mat --no-cpu-baseline --no-ref
for c in FETCH_SIZE WRITE_SIZE; do
  step pmc_mat_$c 120 rocprofv3 --pmc $c --output-format csv -d $D/pmc_mat_$c -o mat -- python3 bench.py --no-cpu-baseline --no-ref --workload mat --steps 20 --warmup 2
done
ISSUE="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES"
step valu_mat 150 rocprofv3 --pmc $ISSUE -d $D/valu_mat -o mat -- python3 bench.py --no-cpu-baseline --no-ref --workload mat --steps 20 --warmup 2
echo done >> $D/steps.log
