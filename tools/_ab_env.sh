#!/bin/bash
# A/B of environment switches: the record-pipeline parity suite under the
# last one, then interleaved benches of each, then a per-tile trace of each.
# usage: tools/_ab_env.sh OUTDIR REPS "VAR=a" "VAR=b" ...
export TMPDIR=/tmp
O=$1; REPS=$2; shift 2
mkdir -p $O
LAST=${@: -1}
env $LAST timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > $O/parity.log 2>&1 || exit 1
for rep in $(seq 1 $REPS); do
  i=0
  for E in "$@"; do
    i=$((i+1))
    env $E timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu > $O/bench_${i}_$rep.json 2> $O/bench_${i}_$rep.err || exit 2
  done
done
i=0
for E in "$@"; do
  i=$((i+1))
  env $E RK_NW_VERBOSE=1 RK_NW_TRACE=$O/trace_$i.bin timeout -k 10 300 python3 bench.py --no-cpu --steps 2 --warmup 1 > $O/bt_$i.json 2> $O/bt_$i.err || exit 3
  python3 tools/nw_trace.py $O/trace_$i.bin > $O/trace_$i.txt 2>&1
  rm -f $O/trace_$i.bin
done
