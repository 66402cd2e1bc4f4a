#!/bin/bash
# Round 3: group-sort regression hunt (HEAD's rk_groupsort vs WPB 1/4) + look-back batch 8, interleaved.
export TMPDIR=/tmp
O=gpurun_out/r3n
mkdir -p $O
for rep in 1 2; do
  for v in def w1 hg; do
    case $v in
      def) E="RK_LIB=repkiller_amd/librepkiller_amd.so";;
      w1) E="RK_GS_WPB=1 RK_LIB=repkiller_amd/librepkiller_amd.so";;
      *) E="RK_LIB=tools/mb/$v/librepkiller_amd.so";;
    esac
    env $E timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu > $O/bench_${v}_$rep.json 2> $O/bench_${v}_$rep.err || exit 4
  done
done
