#!/bin/bash
# Runtime-shape kernels: their GPU tests, then the parity file they share helpers with.
D=gpurun_out/r2dyn
mkdir -p $D
timeout -k 10 600 python -u -m pytest tests/test_gpu_runtime_shapes.py -x -v --timeout 240 --timeout-method thread > $D/dyn_tests.log 2>&1
rc=$?
echo "dyn rc=$rc" | tee -a $D/steps.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 240 --timeout-method thread > $D/parity.log 2>&1
echo "parity rc=$?" | tee -a $D/steps.log
