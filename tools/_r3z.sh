#!/bin/bash
# Round 3: group-sort final pass with branch-free rank terms (variant) vs default.
export TMPDIR=/tmp
O=gpurun_out/r3z
mkdir -p $O
RK_LIB=tools/mb/gsv2/librepkiller_amd.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q -k "sort" --timeout 300 --timeout-method thread > $O/parity_v2.log 2>&1 || exit 1
for rep in 1 2 3; do
  for v in def gsv2; do
    if [ $v = def ]; then L=repkiller_amd/librepkiller_amd.so; else L=tools/mb/$v/librepkiller_amd.so; fi
    RK_LIB=$L timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu > $O/bench_${v}_$rep.json 2> $O/bench_${v}_$rep.err || exit 2
  done
done
