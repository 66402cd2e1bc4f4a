#!/bin/bash
# GPU parity file, then one bench per environment variant:
#   tools/_ab1.sh OUTDIR "ENV1" "ENV2" ...
export TMPDIR=/tmp
OUT=$1; shift
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/parity.log 2>&1 || exit 1
i=0
for V in "$@"; do
  i=$((i+1))
  env $V timeout -k 10 200 python bench.py --steps 10 --warmup 3 --no-cpu > $OUT/b$i.json 2> $OUT/b$i.err || exit 2
done
