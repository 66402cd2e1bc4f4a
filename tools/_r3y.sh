#!/bin/bash
# Round 3: group-sort final insertion pass -- rank loop to the longest leaf (variant) vs 16 unrolled reads; per-phase cycles.
export TMPDIR=/tmp
O=gpurun_out/r3y
mkdir -p $O
RK_LIB=tools/mb/gsv1/librepkiller_amd.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q -k "sort" --timeout 300 --timeout-method thread > $O/parity_v1.log 2>&1 || exit 1
for rep in 1 2; do
  for v in def gsv1; do
    if [ $v = def ]; then L=repkiller_amd/librepkiller_amd.so; else L=tools/mb/$v/librepkiller_amd.so; fi
    RK_LIB=$L timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu > $O/bench_${v}_$rep.json 2> $O/bench_${v}_$rep.err || exit 2
  done
done
for v in gsprof gsprof1; do
  RK_LIB=tools/mb/$v/librepkiller_amd.so timeout -k 10 300 python3 bench.py --gpus 1 --steps 2 --warmup 1 --no-cpu > $O/$v.json 2> $O/$v.err || exit 3
done
