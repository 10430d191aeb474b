#!/bin/bash
# Full -m gpu suite + smoke.
D=gpurun_out/r2suite
mkdir -p $D
timeout -k 10 1500 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $D/gpu_tests.log 2>&1
rc=$?
echo "tests rc=$rc" >> $D/steps.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $D/smoke.log 2>&1
echo "smoke rc=$?" >> $D/steps.log
timeout -k 10 300 python -u bench.py --workload mat --replicates-total 16 --steps 20 --warmup 2 --no-cpu-baseline --no-ref > $D/mat_strong16.json 2> $D/mat_strong16.err
echo "mat_strong rc=$?" >> $D/steps.log
