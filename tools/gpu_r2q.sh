#!/bin/bash
# Round-2 pass o: resident entry header (no records' prologue after a resident run).
D=gpurun_out/r2q
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
step t_res 900 python -u -m pytest tests/test_gpu_resident_launch.py tests/test_gpu_resident.py tests/test_gpu_resident_oracle.py tests/test_gpu_sv_exact.py tests/test_gpu_api_edges.py tests/test_gpu_parity.py -v --timeout 300 --timeout-method thread
for T in 1000 20; do
  step ab_new_T$T 200 python -u tools/diag_launch_overhead.py $T 20
  step ab_nohdr_T$T 200 env PF_RES_HDR=0 python -u tools/diag_launch_overhead.py $T 20
done
step alt_T20 200 python -u tools/diag_alternate.py 20 12
for v in st0 st7; do
  step stamps_${v}_T1000 200 env PF_LIB=build/libpf_hip_$v.so python -u tools/diag_resident_stamps.py 1000000 1000
done
step b_sv_k20 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline
echo done >> $D/steps.log
