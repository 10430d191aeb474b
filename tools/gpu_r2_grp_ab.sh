#!/bin/bash
# Large-state step A/B: L96 geometry / occupancy variants, MAT fp32 reciprocal (bench lines).
D=gpurun_out/r2grp
mkdir -p $D
run() {  # run <name> <lib or -> <env...> -- bench args
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
run l96_base_$rep - -- --workload l96 --steps 100 --warmup 10
run l96_t128_$rep - PF_CHUNKS_PER_THREAD=4 -- --workload l96 --steps 100 --warmup 10
run l96_w8t64_$rep build/libpf_hip_w8g2k.so PF_CHUNKS_PER_THREAD=2 -- --workload l96 --steps 100 --warmup 10
run l96_w6t64_$rep build/libpf_hip_w6g2k.so PF_CHUNKS_PER_THREAD=2 -- --workload l96 --steps 100 --warmup 10
run l96_w8t49_$rep build/libpf_hip_w8g2k.so -- --workload l96 --steps 100 --warmup 10
run mat_base_$rep - -- --workload mat --steps 50 --warmup 5
run mat_rcp_$rep build/libpf_hip_rcp.so -- --workload mat --steps 50 --warmup 5
done
echo done >> $D/steps.log
