#!/bin/bash
# L96: 5 waves/SIMD (96 VGPRs) with 96-particle tiles (3 whole passes, 1042 tiles) vs the default.
D=gpurun_out/r2l96w5
mkdir -p $D
for rep in 1 2; do
  timeout -k 10 300 python -u bench.py --workload l96 --steps 100 --warmup 10 --no-cpu-baseline --no-ref > $D/base_$rep.out 2>&1 || exit $?
  PF_LIB=build/libpf_hip_w5g2k.so PF_CHUNKS_PER_THREAD=3 timeout -k 10 300 python -u bench.py --workload l96 --steps 100 --warmup 10 --no-cpu-baseline --no-ref > $D/w5t96_$rep.out 2>&1 || exit $?
  PF_LIB=build/libpf_hip_w5g2k.so timeout -k 10 300 python -u bench.py --workload l96 --steps 100 --warmup 10 --no-cpu-baseline --no-ref > $D/w5t49_$rep.out 2>&1 || exit $?
done
