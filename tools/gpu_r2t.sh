#!/bin/bash
# Round-2 pass t: sticky priority for the publishing wave vs default.
D=gpurun_out/r2t
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
for rep in 1 2; do
  for T in 1000 20; do
    step ab_new_T${T}_$rep 200 python -u tools/diag_launch_overhead.py $T 20
    step ab_sticky_T${T}_$rep 200 env PF_LIB=build/libpf_hip_sticky.so python -u tools/diag_launch_overhead.py $T 20
  done
done
for v in st0 st7; do
  step stamps_${v}_T1000 200 env PF_LIB=build/libpf_hip_$v.so python -u tools/diag_resident_stamps.py 1000000 1000
  step stamps_${v}_T20 200 env PF_LIB=build/libpf_hip_$v.so python -u tools/diag_resident_stamps.py 1000000 20
done
echo done >> $D/steps.log
