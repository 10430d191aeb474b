#!/bin/bash
# Round-2 pass n: PMC passes (traffic for every SIR workload, SQ counters for SV and LEDH), L96
# per-phase stamps, the spawn launcher with the single-collective gather.
D=gpurun_out/r2n
mkdir -p $D
export TMPDIR=/tmp
step() {  # step <name> <timeout> <cmd...>; exit status 0/1 go on, anything else ends the pass
  local name=$1 t=$2
  shift 2
  timeout -k 10 $t "$@" > $D/$name.out 2> $D/$name.err
  local rc=$?
  echo "$name rc=$rc" | tee -a $D/steps.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
}
step bench_spawn 300 python -u bench.py --gpus 1 --spawn --steps 20 --warmup 5 --no-cpu-baseline --no-ref
step bench_spawn_mat 300 python -u bench.py --gpus 1 --spawn --workload mat --no-cpu-baseline --no-ref
step stamps_l96 200 env PF_LIB=build/libpf_hip_l96st.so python -u tools/diag_stamps_grp.py l96
step t_dist 300 python -u -m pytest tests/test_gpu_distributed.py tests/test_gpu_resident_launch.py -v --timeout 200 --timeout-method thread
bash tools/gpu_pmc_all.sh
echo done >> $D/steps.log
