#!/bin/bash
# Round 3: heap pops with typed LDS accesses (parity + killer timings), group-sort A/B (HEAD's rk_groupsort vs WPB 1/4).
export TMPDIR=/tmp
O=gpurun_out/r3n
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k "sort" > $O/parity.log 2>&1 || exit 1
timeout -k 10 300 python3 tools/heap_killer_check.py 10000 100000 > $O/heap_killer.log 2>&1 || exit 2
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
