#!/bin/bash
# shipped library after the slot-count change: GPU suite, smoke, driver-window bench line and its
# rocprofv3 kernel statistics (K = 20 and K = 1000)
D=gpurun_out/r2last2
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $D/tests.log 2>&1
rc=$?; echo "tests rc=$rc" >> $D/steps.log; [ $rc = 0 ] || exit 1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $D/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc" >> $D/steps.log; [ $rc = 0 ] || exit 1
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $D/bench_k20.json 2> $D/bench_k20.err
rc=$?; echo "bench rc=$rc" >> $D/steps.log; [ $rc = 0 ] || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $D/prof_k20 -o run -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-ref > $D/prof_k20.out 2>&1
rc=$?; echo "prof_k20 rc=$rc" >> $D/steps.log; [ $rc = 0 ] || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $D/prof_k1000 -o run -- python3 bench.py --steps 1000 --warmup 100 --no-cpu-baseline --no-ref > $D/prof_k1000.out 2>&1
rc=$?; echo "prof_k1000 rc=$rc" >> $D/steps.log
