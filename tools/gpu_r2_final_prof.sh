#!/bin/bash
# Round-2 closing pass, part 2: rocprofv3 kernel statistics of the bench lines, and the PMC
# passes of the kernels that changed this session (MAT / L96 k_step_grp, sv64 k_step):
# FETCH_SIZE and WRITE_SIZE in separate runs, SQ issue counters in a third.  -> gpurun_out/r2fprof
D=gpurun_out/r2fprof
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
step prof_default 300 rocprofv3 --kernel-trace --stats -d $D/prof_default -o run -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-ref
step prof_k1000 300 rocprofv3 --kernel-trace --stats -d $D/prof_k1000 -o run -- python3 bench.py --steps 1000 --warmup 100 --no-cpu-baseline --no-ref
step prof_sv64 300 rocprofv3 --kernel-trace --stats -d $D/prof_sv64 -o run -- python3 bench.py --workload sv64 --no-cpu-baseline --no-ref
step prof_l96 300 rocprofv3 --kernel-trace --stats -d $D/prof_l96 -o run -- python3 bench.py --workload l96 --no-cpu-baseline --no-ref
step prof_mat 300 rocprofv3 --kernel-trace --stats -d $D/prof_mat -o run -- python3 bench.py --workload mat --no-cpu-baseline --no-ref
step prof_ledh 300 rocprofv3 --kernel-trace --stats -d $D/prof_ledh -o run -- python3 bench.py --workload ledh --no-cpu-baseline --no-ref
for c in FETCH_SIZE WRITE_SIZE; do
  step pmc_mat_$c 120 rocprofv3 --pmc $c --output-format csv -d $D/pmc_mat_$c -o mat -- python3 bench.py --no-cpu-baseline --no-ref --workload mat --steps 20 --warmup 2
  step pmc_l96_$c 120 rocprofv3 --pmc $c --output-format csv -d $D/pmc_l96_$c -o l96 -- python3 bench.py --no-cpu-baseline --no-ref --workload l96 --steps 50 --warmup 5
  step pmc_sv64_$c 120 rocprofv3 --pmc $c --output-format csv -d $D/pmc_sv64_$c -o sv64 -- python3 bench.py --no-cpu-baseline --no-ref --workload sv64 --steps 20 --warmup 2
done
ISSUE="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES"
step valu_mat 150 rocprofv3 --pmc $ISSUE -d $D/valu_mat -o mat -- python3 bench.py --no-cpu-baseline --no-ref --workload mat --steps 20 --warmup 2
step valu_l96 150 rocprofv3 --pmc $ISSUE -d $D/valu_l96 -o l96 -- python3 bench.py --no-cpu-baseline --no-ref --workload l96 --steps 50 --warmup 5
echo done >> $D/steps.log
