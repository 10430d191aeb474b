#!/bin/bash
# Round-2 pass f: k_resident with per-iteration granule registers (208 VGPRs) and the branch-free
# publish; 1024-thread variant (4 waves / SIMD); resident tests; SV bench and stamps.
D=gpurun_out/r2f
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
step t_res 900 python -u -m pytest tests/test_gpu_resident.py tests/test_gpu_resident_oracle.py tests/test_gpu_sv_exact.py -v -s --timeout 300 --timeout-method thread
step b_sv_k20 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline
step b_sv_k1000 300 python -u bench.py --steps 1000 --warmup 100 --no-cpu-baseline --no-ref
step b_rbs1024_k1000 300 env PF_LIB=build/libpf_hip_rbs1024.so python -u bench.py --steps 1000 --warmup 100 --no-cpu-baseline --no-ref
step b_rbs1024_k20 300 env PF_LIB=build/libpf_hip_rbs1024.so python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-ref
for v in st0 st7; do
  step stamps_${v}_T1000 200 env PF_COOP=0 PF_LIB=build/libpf_hip_$v.so python -u tools/diag_resident_stamps.py 1000000 1000
done
step launch_coop0_T20 200 env PF_COOP=0 python -u tools/diag_launch_overhead.py 20 20
step launch_coop1_T20 200 env PF_COOP=1 python -u tools/diag_launch_overhead.py 20 20
echo done >> $D/steps.log
