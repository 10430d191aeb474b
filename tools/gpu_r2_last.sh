#!/bin/bash
# last check of the shipped library (rebuilt after the reverted experiments): GPU suite, smoke, default bench line
D=gpurun_out/r2last
mkdir -p $D
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $D/tests.log 2>&1
rc=$?; echo "tests rc=$rc" >> $D/steps.log; [ $rc = 0 ] || exit 1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $D/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc" >> $D/steps.log; [ $rc = 0 ] || exit 1
timeout -k 10 300 python -u bench.py > $D/bench_default.json 2> $D/bench_default.err
rc=$?; echo "bench rc=$rc" >> $D/steps.log
