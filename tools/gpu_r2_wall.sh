#!/bin/bash
# Host-side wall anatomy of the K=20 SV job (tools/diag_wall.py), with and without the grid-order event.
D=gpurun_out/r2wall
mkdir -p $D
timeout -k 10 300 python -u tools/diag_wall.py > $D/order_on.log 2>&1 || exit $?
PF_NO_ORDER=1 timeout -k 10 300 python -u tools/diag_wall.py > $D/order_off.log 2>&1
