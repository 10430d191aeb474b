# Covariance kernel timings: the cov tests, then bench lines under rocprof with PF_COV_DIAG ablations
# (1 no staging loads, 2 no MFMA loop, 4 no output) at PF_COV_CPB chunks per workgroup.
# usage: bash tools/gpu_covdiag.sh OUT "DIAGS" "CPBS" WORKLOADS...
D=gpurun_out/$1; DIAGS=$2; CPBS=$3; shift 3; mkdir -p $D
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_cov.py > $D/test.log 2>&1 || exit 1
for w in "$@"; do for c in $CPBS; do for v in $DIAGS; do
  PF_COV_CPB=$c PF_COV_DIAG=$v timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $D/${w}_c${c}_p$v -o run -- python3 bench.py --workload $w --steps 50 --warmup 5 --no-cpu-baseline --no-ref > $D/${w}_c${c}_p$v.log 2>&1 || exit 1
done; done; done
