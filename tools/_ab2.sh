#!/bin/bash
# one-stream traced benches per variant, then the parity file, then 2-stream benches
#   tools/_ab2.sh OUTDIR "ENV1" "ENV2" ...
export TMPDIR=/tmp
OUT=$1; shift
mkdir -p $OUT
i=0
for V in "$@"; do
  i=$((i+1))
  env RK_ONE_STREAM=1 RK_NW_TRACE=$OUT/t$i.bin $V timeout -k 10 200 python bench.py --steps 2 --warmup 1 --no-cpu > $OUT/s$i.json 2> $OUT/s$i.err || exit 1
done
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/parity.log 2>&1 || exit 2
i=0
for V in "$@"; do
  i=$((i+1))
  env $V timeout -k 10 200 python bench.py --steps 10 --warmup 3 --no-cpu > $OUT/b$i.json 2> $OUT/b$i.err || exit 3
done
