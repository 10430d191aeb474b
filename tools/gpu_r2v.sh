#!/bin/bash
# Round 2 (session 3): GPU suite after the lane-local MAT transition and the L96 c_k staging,
# MAT / L96 / sv64 bench lines, and where the 64 x 1e6 SV step spends its time.
D=gpurun_out/r2v
mkdir -p $D
step() { echo "$1 rc=$2" >> $D/steps.log; }
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $D/gpu_tests.log 2>&1
rc=$?; step tests $rc; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py --workload mat --no-cpu-baseline --no-ref > $D/bench_mat.json 2> $D/bench_mat.err
rc=$?; step mat $rc; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py --workload l96 --no-cpu-baseline --no-ref > $D/bench_l96.json 2> $D/bench_l96.err
rc=$?; step l96 $rc; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u tools/diag_sv64.py 64 1000000 20 > $D/sv64_diag.log 2>&1
rc=$?; step sv64diag $rc; [ $rc -ne 0 ] && exit $rc
PF_LIB=build/libpf_hip_stamps.so timeout -k 10 300 python -u tools/diag_sv64.py 64 1000000 10 > $D/sv64_stamps.log 2>&1
rc=$?; step sv64stamps $rc; [ $rc -ne 0 ] && exit $rc
for v in w5 w6; do
PF_LIB=build/libpf_hip_$v.so timeout -k 10 300 python -u tools/diag_sv64.py 64 1000000 20 > $D/sv64_$v.log 2>&1
rc=$?; step sv64_$v $rc; [ $rc -ne 0 ] && exit $rc
done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $D/prof_mat -o mat -- python3 bench.py --workload mat --steps 50 --warmup 5 --no-cpu-baseline --no-ref > $D/prof_mat.out 2>&1
rc=$?; step prof_mat $rc
