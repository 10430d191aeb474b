#!/bin/bash
# Round-2 pass i: plain launch with the in-kernel co-residency check (default) vs cooperative;
# same-box A/B against the previous kernel; launch tests; bench K=20 at two warm-ups; rocprof.
D=gpurun_out/r2j
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
step t_launch 600 python -u -m pytest tests/test_gpu_resident_launch.py -v -s --timeout 300 --timeout-method thread
for rep in 1 2; do
  for T in 1000 20; do
    step ab_prev_T${T}_$rep 200 env PF_COOP=0 PF_LIB=build/libpf_hip_prev.so python -u tools/diag_launch_overhead.py $T 20
    step ab_new_T${T}_$rep 200 python -u tools/diag_launch_overhead.py $T 20
    step ab_coop_T${T}_$rep 200 env PF_COOP=1 python -u tools/diag_launch_overhead.py $T 20
  done
done
for v in st0 st7; do
  step stamps_${v}_T1000 200 env PF_LIB=build/libpf_hip_$v.so python -u tools/diag_resident_stamps.py 1000000 1000
done
step b_sv_k20 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline
step b_sv_k20_w200 300 python -u bench.py --steps 20 --warmup 200 --no-cpu-baseline --no-ref
step b_sv_k1000 300 python -u bench.py --steps 1000 --warmup 100 --no-cpu-baseline --no-ref

step t_res 900 python -u -m pytest tests/test_gpu_resident.py tests/test_gpu_resident_oracle.py tests/test_gpu_sv_exact.py -v -s --timeout 300 --timeout-method thread
echo done >> $D/steps.log
