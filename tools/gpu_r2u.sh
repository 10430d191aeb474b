#!/bin/bash
# Round-2 pass u: L96 / MAT step kernels - output-field skip (new lib) vs heads on/off.
D=gpurun_out/r2u
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
  step l96_new_$rep 300 python -u bench.py --workload l96 --steps 200 --warmup 10 --no-cpu-baseline --no-ref
  step l96_head_$rep 300 env PF_HEAD=1 python -u bench.py --workload l96 --steps 200 --warmup 10 --no-cpu-baseline --no-ref
  step l96_prev_$rep 300 env PF_LIB=build/libpf_hip_prev.so python -u bench.py --workload l96 --steps 200 --warmup 10 --no-cpu-baseline --no-ref
  step mat_new_$rep 300 python -u bench.py --workload mat --steps 40 --warmup 4 --no-cpu-baseline --no-ref
  step mat_prev_$rep 300 env PF_LIB=build/libpf_hip_prev.so python -u bench.py --workload mat --steps 40 --warmup 4 --no-cpu-baseline --no-ref
done
step t_grp 600 python -u -m pytest tests/test_gpu_grp.py tests/test_gpu_parity.py -v --timeout 300 --timeout-method thread
echo done >> $D/steps.log
