#!/bin/bash
# Every bench line's PMC passes at HEAD (FETCH_SIZE, WRITE_SIZE, SQ issue counters; separate runs,
# no trace domains - MI355X_MICROARCH.md HBM section), plus rocprofv3 kernel statistics of each
# line.  Fold on the build host with tools/pmc_fold.py.   tools/gpu_pmc_all.sh OUTDIR [workload...]
D=${1:-gpurun_out/pmc}
mkdir -p "$D"; . "$(dirname "$0")/gpu_lib.sh"
ISSUE="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES"
run_pmc() {  # name "bench args"
  local name=$1 bargs=$2
  for c in FETCH_SIZE WRITE_SIZE; do
    step "${name}_$c" 150 rocprofv3 --pmc $c --output-format csv -d "$D/${name}_$c" -o "$name" -- \
      python3 bench.py --no-cpu-baseline --no-ref $bargs
  done
  step "${name}_issue" 150 rocprofv3 --pmc $ISSUE -d "$D/${name}_issue" -o "$name" -- \
    python3 bench.py --no-cpu-baseline --no-ref $bargs
  step "${name}_stats" 150 rocprofv3 --kernel-trace --stats -d "$D/${name}_stats" -o "$name" -- \
    python3 bench.py --no-cpu-baseline --no-ref $bargs
}
shift
for w in ${@:-sv sv64 sv_fp64 l96 mat ledh}; do
  case $w in
    sv) run_pmc sv "--steps 20 --warmup 5" ;;
    sv64) run_pmc sv64 "--workload sv64 --steps 20 --warmup 3" ;;
    sv_fp64) run_pmc sv_fp64 "--precision fp64 --steps 20 --warmup 5" ;;
    l96) run_pmc l96 "--workload l96 --steps 50 --warmup 5" ;;
    mat) run_pmc mat "--workload mat --steps 40 --warmup 4" ;;
    ledh) run_pmc ledh "--workload ledh --steps 50 --warmup 5" ;;
    ledh_mat) run_pmc ledh_mat "--workload ledh_mat --steps 10 --warmup 2" ;;
  esac
done
echo done >> "$D/steps.log"
