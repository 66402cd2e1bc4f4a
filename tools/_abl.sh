#!/bin/bash
# Timing-only ablation (results deliberately wrong, no parity claimed): the group sort's final insertion pass removed.
export TMPDIR=/tmp
O=gpurun_out/abl
mkdir -p $O
for rep in 1 2; do
  for v in def ablf; do
    if [ $v = def ]; then L=repkiller_amd/librepkiller_amd.so; else L=tools/mb/$v/librepkiller_amd.so; fi
    RK_LIB=$L timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu > $O/bench_${v}_$rep.json 2> $O/bench_${v}_$rep.err || exit 2
  done
done
