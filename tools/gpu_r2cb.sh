#!/bin/bash
# rollback slot counts by floor + fraction: resident tests, phase stamps (new / old fill), bench A/B at K = 20 / 1000
D=gpurun_out/r2cb
mkdir -p $D
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_resident.py tests/test_gpu_resident_launch.py tests/test_gpu_parity.py tests/test_gpu_resident_oracle.py > $D/tests.log 2>&1
rc=$?; echo "tests rc=$rc" >> $D/steps.log; [ $rc = 0 ] || exit 1
for v in stamps stampscb0; do
  PF_LIB=build/libpf_hip_$v.so timeout -k 10 120 python -u tools/diag_resident_stamps.py 1000000 1000 > $D/stamps_$v.log 2>&1
  rc=$?; echo "$v rc=$rc" >> $D/steps.log; [ $rc = 0 ] || exit 1
done
for r in 1 2 3; do for v in main cb0; do
  lib=particle_filters_amd/libpf_hip.so; [ $v != main ] && lib=build/libpf_hip_$v.so
  PF_LIB=$lib timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-ref > $D/k20_${v}_$r.json 2>/dev/null
  PF_LIB=$lib timeout -k 10 200 python -u bench.py --steps 1000 --warmup 100 --no-cpu-baseline --no-ref > $D/k1000_${v}_$r.json 2>/dev/null
  rc=$?; echo "$v $r rc=$rc" >> $D/steps.log; [ $rc = 0 ] || exit 1
done; done
