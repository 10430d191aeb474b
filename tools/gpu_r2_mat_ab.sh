#!/bin/bash
# MAT step A/B: 3 vs 4 waves per SIMD (PF_GRP_WPE_SMALL), tile 256 vs 320.
D=gpurun_out/r2mat
mkdir -p $D
run() {
  local name=$1 lib=$2
  shift 2
  local envs=()
  while [ "$1" != "--" ]; do envs+=("$1"); shift; done
  shift
  if [ "$lib" != "-" ]; then envs+=("PF_LIB=$lib"); fi
  env "${envs[@]}" timeout -k 10 300 python -u bench.py "$@" --no-cpu-baseline --no-ref > $D/$name.out 2> $D/$name.err
  local rc=$?
  echo "$name rc=$rc" >> $D/steps.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
}
for rep in 1 2; do
run mat_base_$rep - -- --workload mat --steps 50 --warmup 5
run mat_w4_$rep build/libpf_hip_mw4.so -- --workload mat --steps 50 --warmup 5
run mat_t320_$rep - PF_CHUNKS_PER_THREAD=5 -- --workload mat --steps 50 --warmup 5
run mat_w4t320_$rep build/libpf_hip_mw4.so PF_CHUNKS_PER_THREAD=5 -- --workload mat --steps 50 --warmup 5
done
echo done >> $D/steps.log
