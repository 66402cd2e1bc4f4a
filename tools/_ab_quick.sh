#!/bin/bash
# Interleaved A/B of the working tree's library against tools/mb/base (the previous HEAD), after the sort/sweep parity tests.
export TMPDIR=/tmp
O=${1:-gpurun_out/abq}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > $O/parity.log 2>&1 || exit 1
for rep in 1 2 3; do
  for v in new base; do
    if [ $v = new ]; then L=repkiller_amd/librepkiller_amd.so; else L=tools/mb/base/librepkiller_amd.so; fi
    RK_LIB=$L timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu > $O/bench_${v}_$rep.json 2> $O/bench_${v}_$rep.err || exit 2
  done
done
