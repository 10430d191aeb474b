#!/bin/bash
# Same-box A/B/n of engine libraries on one bench line, alternating.
#   tools/gpu_abn.sh OUTDIR "BENCH ARGS" REPS LIB_1 [LIB_2 ...]   (LIB "main" = the in-tree library)
# Each run: PF_LIB=<lib> python bench.py <args> --no-cpu-baseline --no-ref, under its own time limit.
set -o pipefail
out=$1; args=$2; reps=$3; shift 3
mkdir -p "$out"
for i in $(seq 1 "$reps"); do
  for lib in "$@"; do
    tag=$(basename "$lib" .so)
    if [ "$lib" = main ]; then unset PF_LIB; else export PF_LIB=$lib; fi
    timeout -k 10 120 python bench.py $args --no-cpu-baseline --no-ref > "$out/${tag}_$i.json" 2> "$out/${tag}_$i.err" || exit $?
    python -c "import json; d=json.load(open('$out/${tag}_$i.json')); r=d['roofline']; print('$tag', $i, '%.4g' % d['value'], '%.3f' % (d['ms_per_step']*1e3), 'us/step', '%.4f' % r['frac'], '%.1f us/launch' % r['avg_launch_us'])" | tee -a "$out/summary.txt"
  done
done
