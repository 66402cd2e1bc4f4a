#!/bin/bash
# Parity (GPU suite + the full-size configs), then an A/B of environment
# settings on the default bench, three interleaved rounds.
# usage: tools/_ab3r.sh OUTDIR "VAR=a" "VAR=b" ...
export TMPDIR=/tmp
O=${1:-gpurun_out/ab3r}; shift
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_large_configs.py -m gpu -x -q --timeout 400 --timeout-method thread > $O/large.log 2>&1 || exit 1
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread --deselect tests/test_large_configs.py > $O/tests.log 2>&1 || exit 2
for rep in 1 2 3; do
  i=0
  for e in "$@"; do
    i=$((i+1))
    env $e timeout -k 10 200 python bench.py --no-cpu --steps 10 --warmup 3 > $O/b$i.$rep.json 2> $O/b$i.$rep.err || exit 3
  done
done
