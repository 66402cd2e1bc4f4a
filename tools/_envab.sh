#!/bin/bash
# A/B of environment settings on the default bench (interleaved, two rounds).
# usage: tools/_envab.sh OUTDIR "VAR=a" "VAR=b" ...
export TMPDIR=/tmp
O=${1:-gpurun_out/envab}; shift
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || exit 1
for rep in 1 2; do
  i=0
  for e in "$@"; do
    i=$((i+1))
    env $e timeout -k 10 200 python bench.py --no-cpu --steps 10 --warmup 3 > $O/b$i.$rep.json 2> $O/b$i.$rep.err || exit 2
  done
done
