#!/bin/bash
# fp64 SV N=1e6 launch-per-step: tile / head knobs A/B (bench lines, K=20 and K=200)
D=gpurun_out/r2fp64
mkdir -p $D
b() {  # b <name> <env...>
  local name=$1; shift
  env "$@" timeout -k 10 200 python -u bench.py --precision fp64 --steps 200 --warmup 5 --no-cpu-baseline --no-ref > $D/$name.json 2> $D/$name.err
  echo "$name rc=$?" >> $D/steps.log
}
b base PF_X=0
b head PF_HEAD=1
b ch2 PF_CHUNKS_PER_THREAD=2
b ch4 PF_CHUNKS_PER_THREAD=4
b ch8 PF_CHUNKS_PER_THREAD=8
b head_ch2 PF_HEAD=1 PF_CHUNKS_PER_THREAD=2
b head_ch4 PF_HEAD=1 PF_CHUNKS_PER_THREAD=4
env PF_RESIDENT=0 timeout -k 10 200 python -u bench.py --steps 200 --warmup 5 --no-cpu-baseline --no-ref > $D/fp32_step.json 2> $D/fp32_step.err
echo "fp32_step rc=$?" >> $D/steps.log
env PF_RESIDENT=0 PF_CHUNKS_PER_THREAD=4 timeout -k 10 200 python -u bench.py --steps 200 --warmup 5 --no-cpu-baseline --no-ref > $D/fp32_step_ch4.json 2> $D/fp32_step_ch4.err
echo "fp32_step_ch4 rc=$?" >> $D/steps.log
