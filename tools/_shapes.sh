#!/bin/bash
# record-pass tile shapes: parity (record pipeline tests) with the candidate
# shape, then the default bench per shape.  usage: tools/_shapes.sh OUTDIR SHAPES...
export TMPDIR=/tmp
O=${1:-gpurun_out/shapes}; shift
mkdir -p $O
for s in "$@"; do
  RK_NW_SHAPE=$s timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k record --timeout 120 --timeout-method thread > $O/t$s.log 2>&1 || exit 1
done
for rep in 1 2; do
  for s in "$@"; do
    RK_NW_SHAPE=$s timeout -k 10 200 python bench.py --no-cpu --steps 10 --warmup 3 > $O/b$s.$rep.json 2> $O/b$s.$rep.err || exit 2
  done
done
