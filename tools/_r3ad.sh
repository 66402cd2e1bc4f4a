#!/bin/bash
# Round 3: the Y window sweep kernel at 7 waves per SIMD (no VGPR spills) vs 8 (44 B of scratch per lane).
export TMPDIR=/tmp
O=gpurun_out/r3ad
mkdir -p $O
for rep in 1 2 3; do
  for v in def w7; do
    if [ $v = def ]; then L=repkiller_amd/librepkiller_amd.so; else L=tools/mb/$v/librepkiller_amd.so; fi
    RK_LIB=$L timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu > $O/bench_${v}_$rep.json 2> $O/bench_${v}_$rep.err || exit 2
  done
done
