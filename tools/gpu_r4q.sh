#!/bin/bash
# Round-4: where the L96 covariance launch (k_cov_part, ~16.5 us) spends its time - rocprof kernel
# statistics of the L96 bench line under PF_COV_DIAG ablations (1 rows not used, 2 no MFMA loop,
# 4 no output, 32 return at entry).
D=${1:-gpurun_out/r4q}
mkdir -p "$D"; . "$(dirname "$0")/gpu_lib.sh"
for v in 0 32 4 2 6 7; do
  PF_COV_DIAG=$v step "l96_p$v" 150 rocprofv3 --kernel-trace --stats -d "$D/l96_p$v" -o run -- python3 bench.py --workload l96 --steps 50 --warmup 5 --no-cpu-baseline --no-ref
done
echo done >> "$D/steps.log"
