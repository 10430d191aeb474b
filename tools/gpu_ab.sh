#!/bin/bash
# Same-box A/B of two engine libraries on one bench line, alternating.
#   tools/gpu_ab.sh OUTDIR "BENCH ARGS" LIB_A LIB_B [REPS]
# Each run: PF_LIB=<lib> python bench.py <args> --no-cpu-baseline --no-ref, under its own time limit.
set -o pipefail
out=$1; args=$2; a=$3; b=$4; reps=${5:-3}
mkdir -p "$out"
for i in $(seq 1 "$reps"); do
  for tag in A B; do
    lib=$a; [ "$tag" = B ] && lib=$b
    PF_LIB=$lib timeout -k 10 120 python bench.py $args --no-cpu-baseline --no-ref > "$out/${tag}_$i.json" 2> "$out/${tag}_$i.err" || exit $?
    python -c "import json,sys; d=json.load(open('$out/${tag}_$i.json')); print('$tag', $i, d['value'], d['ms_per_step'], d.get('roofline',{}).get('frac'))" | tee -a "$out/summary.txt"
  done
done
