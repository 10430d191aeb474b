set -e
mkdir -p gpurun_out/r7/scal
export TMPDIR=/tmp
for n in 1000 4000 10000 16000; do
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/r7/scal/n$n -o n$n -- python3 tools/ledh_scaling.py $n > gpurun_out/r7/scal/n$n.log 2>&1
done
