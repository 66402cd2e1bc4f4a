#!/bin/bash
# Round 3: look-back batch A/B (RK_LB_BATCH 4 / 8 / 16 builds), interleaved, plus FETCH_SIZE of each.
export TMPDIR=/tmp
O=gpurun_out/r3k
mkdir -p $O
for rep in 1 2; do
  for v in lb4 lb8 def; do
    if [ $v = def ]; then L=repkiller_amd/librepkiller_amd.so; else L=tools/mb/$v/librepkiller_amd.so; fi
    RK_LIB=$L timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu > $O/bench_${v}_$rep.json 2> $O/bench_${v}_$rep.err || exit 1
  done
done
for v in lb4 def; do
  if [ $v = def ]; then L=repkiller_amd/librepkiller_amd.so; else L=tools/mb/$v/librepkiller_amd.so; fi
  RK_LIB=$L timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/f_$v -o p -- python3 bench.py --no-cpu --steps 3 --warmup 1 > $O/f_$v.log 2>&1 || exit 2
done
