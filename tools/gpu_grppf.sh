#!/bin/bash
# Large-state step with software-pipelined state loads (PF_GRP_PF): parity on the variant
# library (L96/MAT cases of the GPU parity suite) + L96 / MAT bench A/B.
set -e
mkdir -p gpurun_out/grppf
export TMPDIR=/tmp
PF_LIB=build/libpf_hip_grppf.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/grppf/tests.log 2>&1 || { tail -30 gpurun_out/grppf/tests.log; exit 1; }
tail -1 gpurun_out/grppf/tests.log
for w in l96 mat; do
  for v in grppf default grppf default; do
    lib=build/libpf_hip_$v.so; [ "$v" = "default" ] && lib=particle_filters_amd/libpf_hip.so
    PF_LIB=$lib timeout -k 10 200 python -u bench.py --workload $w --no-cpu-baseline > gpurun_out/grppf/${w}_$v.json 2> gpurun_out/grppf/${w}_$v.err || { echo "$w $v failed"; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/grppf/${w}_$v.json'));print('$w $v', round(d['ms_per_step']*1e3,1),'us/step value %.3g'%d['value'],'rmse',round(d['rmse'],4))"
  done
done
