#!/bin/bash
# sv64 (SURVEY 8d roofline run: 64 x 1e6 SV filters): probe with/without resampling,
# kernel stats, and HBM traffic PMC passes of k_step.
set -e
mkdir -p gpurun_out/sv64p
export TMPDIR=/tmp
timeout -k 10 200 python -u tools/sv64_probe.py 64 1000000 40 > gpurun_out/sv64p/probe.log 2>&1
cat gpurun_out/sv64p/probe.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/sv64p/prof -o sv64 -- python3 bench.py --workload sv64 --no-cpu-baseline --steps 50 --warmup 5 > gpurun_out/sv64p/prof.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/sv64p/pmc_fetch -o f -- python3 bench.py --workload sv64 --no-cpu-baseline --steps 10 --warmup 2 > gpurun_out/sv64p/pmc_fetch.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/sv64p/pmc_write -o w -- python3 bench.py --workload sv64 --no-cpu-baseline --steps 10 --warmup 2 > gpurun_out/sv64p/pmc_write.log 2>&1
ls -R gpurun_out/sv64p | head -30
