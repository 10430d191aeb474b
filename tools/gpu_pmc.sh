#!/bin/bash
# PMC passes for one bench line (MI355X_MICROARCH.md HBM section: FETCH_SIZE and WRITE_SIZE in
# separate runs; SQ issue / wait counters in their own runs; no trace domains with --pmc).
#   tools/gpu_pmc.sh OUTDIR NAME "BENCH ARGS" [traffic] [issue] [wait]
# Fold the results with tools/pmc_summary.py / tools/pmc_valu.py on the build host.
D=${1:-gpurun_out/pmc}; name=$2; bargs=$3; shift 3
mkdir -p "$D"; . "$(dirname "$0")/gpu_lib.sh"
ISSUE="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES"
WAIT="SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS"
for what in "${@:-traffic issue}"; do
  for w in $what; do
    case $w in
      traffic) for c in FETCH_SIZE WRITE_SIZE; do
          step "${name}_$c" 120 rocprofv3 --pmc $c --output-format csv -d "$D/${name}_$c" -o "$name" -- \
            python3 bench.py --no-cpu-baseline --no-ref $bargs
        done ;;
      issue) step "${name}_issue" 150 rocprofv3 --pmc $ISSUE -d "$D/${name}_issue" -o "$name" -- \
          python3 bench.py --no-cpu-baseline --no-ref $bargs ;;
      wait) step "${name}_wait" 150 rocprofv3 --pmc $WAIT -d "$D/${name}_wait" -o "$name" -- \
          python3 bench.py --no-cpu-baseline --no-ref $bargs ;;
    esac
  done
done
echo done >> "$D/steps.log"
