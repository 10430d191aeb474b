#!/bin/bash
# Round-2 pass e: GPU suite after the transposed publish / quad combine of k_resident; SV bench
# at the driver's configuration (cooperative and plain launch) and T = 1000; phase stamps;
# L96 / MAT / LEDH-MAT bench lines.
D=gpurun_out/r2e
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
step b_sv_k20 300 python -u bench.py --steps 20 --warmup 5
step b_sv_k20_plain 300 env PF_COOP=0 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-ref
step b_sv_k1000 300 python -u bench.py --steps 1000 --warmup 100 --no-cpu-baseline
for v in st0 st7; do
  step stamps_${v}_T1000 200 env PF_COOP=0 PF_LIB=build/libpf_hip_$v.so python -u tools/diag_resident_stamps.py 1000000 1000
done
step launch_coop0_T20 200 env PF_COOP=0 python -u tools/diag_launch_overhead.py 20 20
step launch_coop1_T20 200 env PF_COOP=1 python -u tools/diag_launch_overhead.py 20 20
step b_l96 300 python -u bench.py --workload l96
step b_mat 300 python -u bench.py --workload mat
step b_ledh_mat 900 python -u bench.py --workload ledh_mat
echo done >> $D/steps.log
