#!/bin/bash
# Bench lines (+ rocprofv3 kernel statistics of each).   tools/gpu_bench.sh OUTDIR LINE...
# LINE names: default k1000 fp64 sv64 l96 mat mat64 ledh edh ledh_mat l96_1000 spawn
# "prof_<LINE>" runs the same line under rocprofv3 --kernel-trace --stats (no CPU / oracle legs).
D=${1:-gpurun_out/bench}; shift
mkdir -p "$D"; . "$(dirname "$0")/gpu_lib.sh"
args() {
  case $1 in
    default) echo "--gpus 1 --steps 20 --warmup 5" ;;
    k1000) echo "--steps 1000 --warmup 100 --no-cpu-baseline" ;;
    fp64) echo "--precision fp64 --steps 20 --warmup 5 --no-cpu-baseline" ;;
    mat64) echo "--workload mat --replicates-total 64 --steps 40 --warmup 4 --no-cpu-baseline --no-ref" ;;
    spawn) echo "--gpus 1 --spawn --steps 20 --warmup 5 --no-cpu-baseline --no-ref" ;;
    *) echo "--workload $1" ;;
  esac
}
for l in "$@"; do
  case $l in
    prof_*) b=${l#prof_}
      step "$l" 300 rocprofv3 --kernel-trace --stats -d "$D/$l" -o run -- python3 bench.py $(args "$b") --no-cpu-baseline --no-ref ;;
    *) step "bench_$l" 300 python -u bench.py $(args "$l") ;;
  esac
done
echo done >> "$D/steps.log"
