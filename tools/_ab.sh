#!/bin/bash
# A/B of environment variants: tools/_ab.sh OUTDIR "ENV1" "ENV2" ... (each twice, interleaved)
export TMPDIR=/tmp
OUT=$1; shift
mkdir -p $OUT
for rep in 1 2; do
  i=0
  for V in "$@"; do
    i=$((i+1))
    env $V timeout -k 10 200 python bench.py --steps 10 --warmup 3 --no-cpu > $OUT/b$i.$rep.json 2> $OUT/b$i.$rep.err || exit 1
  done
done
