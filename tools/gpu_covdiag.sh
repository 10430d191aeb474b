# Covariance kernel timings: the cov tests, then bench lines under rocprof with PF_COV_DIAG ablations.
# usage: bash tools/gpu_covdiag.sh OUT "DIAGS" WORKLOADS...
D=gpurun_out/$1; DIAGS=$2; shift 2; mkdir -p $D
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_cov.py > $D/test.log 2>&1 || exit 1
for w in "$@"; do for v in $DIAGS; do
  PF_COV_DIAG=$v timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $D/${w}_p$v -o run -- python3 bench.py --workload $w --steps 50 --warmup 5 --no-cpu-baseline --no-ref > $D/${w}_p$v.log 2>&1 || exit 1
done; done
