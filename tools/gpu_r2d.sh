#!/bin/bash
# Round-2 pass d: the reworked resident-vs-oracle / exact-SV / sharded tests; resident kernel
# phase stamps for a verifying wave (thread 0) and the publishing wave (thread 448) at T = 20
# and 1000; verification / rollback ablations at --steps 20 and 1000 (plain launch).
D=gpurun_out/r2d
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
step t_gpu 1200 python -u -m pytest tests -m gpu -v -s --timeout 300 --timeout-method thread
for v in st0 st7; do
  for T in 20 1000; do
    step stamps_${v}_T$T 200 env PF_COOP=0 PF_LIB=build/libpf_hip_$v.so python -u tools/diag_resident_stamps.py 1000000 $T
  done
done
for k in 20 1000; do
  w=$((k / 10 > 5 ? k / 10 : 5))
  for v in abl1 abl2; do
    step b_${v}_k$k 300 env PF_COOP=0 PF_LIB=build/libpf_hip_$v.so python -u bench.py --steps $k --warmup $w --no-cpu-baseline --no-ref
  done
done
for lc in 0 1; do
  step b_l96_lcum$lc 300 env PF_LCUM=$lc python -u bench.py --workload l96 --steps 100 --warmup 10 --no-cpu-baseline --no-ref
done
for c in 0 1; do
  for T in 20 1000; do
    step launch_coop${c}_T$T 200 env PF_COOP=$c python -u tools/diag_launch_overhead.py $T 20
  done
done
step b_ledh_mat 600 python -u bench.py --workload ledh_mat
echo done >> $D/steps.log
