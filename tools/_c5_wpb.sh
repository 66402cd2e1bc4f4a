#!/bin/bash
export TMPDIR=/tmp
O=gpurun_out/c5
mkdir -p $O
for v in def wpb4; do
  if [ $v = def ]; then E="RK_GS_WPB=1"; else E="RK_GS_WPB=4"; fi
  env $E timeout -k 10 600 python3 bench.py --gpus 1 --config cfg5 --steps 3 --warmup 1 --no-cpu > $O/bench_$v.json 2> $O/bench_$v.err || exit 1
done
