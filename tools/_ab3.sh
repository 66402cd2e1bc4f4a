#!/bin/bash
# GPU parity (record parity file + host IO tests), then one-stream and two-stream benches
#   tools/_ab3.sh OUTDIR "ENV1" ...
export TMPDIR=/tmp
OUT=$1; shift
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_host_io.py -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/parity.log 2>&1 || exit 1
i=0
for V in "$@"; do
  i=$((i+1))
  env RK_ONE_STREAM=1 $V timeout -k 10 200 python bench.py --steps 5 --warmup 2 --no-cpu > $OUT/s$i.json 2> $OUT/s$i.err || exit 2
  env $V timeout -k 10 200 python bench.py --steps 10 --warmup 3 --no-cpu > $OUT/b$i.json 2> $OUT/b$i.err || exit 3
done
