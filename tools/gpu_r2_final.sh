#!/bin/bash
# Round-2 closing pass, part 1: full -m gpu suite, smoke, every bench line (the driver's default
# command first), the spawn launcher.  -> gpurun_out/r2final
D=gpurun_out/r2final
mkdir -p $D
export TMPDIR=/tmp
step() {  # step <name> <timeout> <cmd...>; exit status 0/1/2 go on, anything else ends the pass
  local name=$1 t=$2
  shift 2
  timeout -k 10 $t "$@" > $D/$name.out 2> $D/$name.err
  local rc=$?
  echo "$name rc=$rc" | tee -a $D/steps.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ] && [ $rc -ne 2 ]; then exit $rc; fi
}
step tests 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread
step smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()"
step bench_default 300 python -u bench.py --gpus 1 --steps 20 --warmup 5
step bench_k1000 300 python -u bench.py --steps 1000 --warmup 100 --no-cpu-baseline
step bench_fp64 300 python -u bench.py --precision fp64 --steps 20 --warmup 5 --no-cpu-baseline
step bench_spawn 300 python -u bench.py --gpus 1 --spawn --steps 20 --warmup 5 --no-cpu-baseline --no-ref
step bench_sv64 300 python -u bench.py --workload sv64
step bench_l96 300 python -u bench.py --workload l96
step bench_mat 300 python -u bench.py --workload mat
step bench_mat64 300 python -u bench.py --workload mat --replicates-total 64 --steps 40 --warmup 4 --no-cpu-baseline --no-ref
step bench_ledh 300 python -u bench.py --workload ledh
step bench_edh 300 python -u bench.py --workload edh
echo done >> $D/steps.log
