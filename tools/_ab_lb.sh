#!/bin/bash
# Look-back batch 4 / 6 / 8 (default) / 12 and no sleep between polls: record passes per step, interleaved.
export TMPDIR=/tmp
O=gpurun_out/ablb
mkdir -p $O
for rep in 1 2; do
  for v in def lb4 lb6 lb12 sl0; do
    if [ $v = def ]; then L=repkiller_amd/librepkiller_amd.so; else L=tools/mb/$v/librepkiller_amd.so; fi
    RK_LIB=$L timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu > $O/bench_${v}_$rep.json 2> $O/bench_${v}_$rep.err || exit 2
  done
done
