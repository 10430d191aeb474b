#!/bin/bash
# Round-2 pass c: new parity tests (resident vs oracle, exact SV, host-replay shards, RCCL) and
# the record-ring replica A/B (1 / 4 / 8 replicas, plain launch) at --steps 20 and 1000.
D=gpurun_out/r2c
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
step t_new 700 python -u -m pytest tests/test_gpu_resident_oracle.py tests/test_gpu_sv_exact.py tests/test_gpu_sharded.py tests/test_gpu_distributed.py tests/test_gpu_api_edges.py tests/test_gpu_resident.py -v -s --timeout 300 --timeout-method thread
for k in 20 1000; do
  w=$((k / 10 > 5 ? k / 10 : 5))
  for v in rc1 rc4; do
    step b_${v}_k$k 300 env PF_COOP=0 PF_LIB=build/libpf_hip_$v.so python -u bench.py --steps $k --warmup $w --no-cpu-baseline --no-ref
  done
  step b_rc8_k$k 300 env PF_COOP=0 python -u bench.py --steps $k --warmup $w --no-cpu-baseline --no-ref
done
step coop_min_coop_destroy 60 rocprofv3 --kernel-trace --stats -d $D/cm1 -o cm -- ./build/coop_min 1 1 10
echo done >> $D/steps.log
