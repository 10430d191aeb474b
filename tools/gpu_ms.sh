#!/bin/bash
# Multi-step fused LEDH launch check: the LEDH / EDH / flow-replay GPU tests on a variant library,
# then an A/B of LEDH config 5 against the in-tree library and with one step per launch.
#   tools/gpu_ms.sh OUTDIR LIB
set -o pipefail
D=$1; LIB=$2
mkdir -p "$D"
source tools/gpu_lib.sh
PF_LIB=$LIB step tests 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_ledh.py tests/test_gpu_edh.py tests/test_gpu_flow_run_replay.py
bash tools/gpu_ab.sh "$D/ab" "--workload ledh" particle_filters_amd/libpf_hip.so "$LIB" 3 || exit $?
PF_LEDH_FSTEPS=1 PF_LIB=$LIB step ledh_fs1 120 python bench.py --workload ledh --no-cpu-baseline --no-ref
PF_LIB=$LIB step edh_ms 120 python bench.py --workload edh --no-cpu-baseline --no-ref
