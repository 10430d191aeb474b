#!/bin/bash
# Round-2 pass b: resident kernel vs oracle after the fp64 tile mass; record-ring replicas A/B
# (8 replicas vs 1, build/libpf_hip_rc1.so); cooperative vs plain launch; the minimal
# cooperative-launch program under rocprofv3 (does the exit crash need torch / the engine?).
D=gpurun_out/r2b
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
step t_resident_oracle 400 python -u -m pytest tests/test_gpu_resident_oracle.py -v -s --timeout 300 --timeout-method thread
for k in 20 1000; do
  w=$((k / 10 > 5 ? k / 10 : 5))
  step b_rc8_coop_k$k 300 python -u bench.py --steps $k --warmup $w --no-cpu-baseline --no-ref
  step b_rc8_plain_k$k 300 env PF_COOP=0 python -u bench.py --steps $k --warmup $w --no-cpu-baseline --no-ref
  step b_rc1_coop_k$k 300 env PF_LIB=build/libpf_hip_rc1.so python -u bench.py --steps $k --warmup $w --no-cpu-baseline --no-ref
  step b_rc1_plain_k$k 300 env PF_COOP=0 PF_LIB=build/libpf_hip_rc1.so python -u bench.py --steps $k --warmup $w --no-cpu-baseline --no-ref
done
step coop_min_plain 60 rocprofv3 --kernel-trace --stats -d $D/cm0 -o cm -- ./build/coop_min 0 1 10
step coop_min_coop_nodestroy 60 rocprofv3 --kernel-trace --stats -d $D/cm2 -o cm -- ./build/coop_min 1 0 10
step coop_min_coop 60 rocprofv3 --kernel-trace --stats -d $D/cm1 -o cm -- ./build/coop_min 1 1 10
echo done >> $D/steps.log
