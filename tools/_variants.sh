#!/bin/bash
# usage: tools/_variants.sh OUTDIR FILE "EXTRA1" "EXTRA2" ... (rebuilds FILE per variant, benches each)
set -e
OUT=$1; FILE=$2; shift 2
mkdir -p $OUT
i=0
for V in "$@"; do
  i=$((i+1))
  touch repkiller_amd/csrc/$FILE
  make -C repkiller_amd/csrc -j16 EXTRA="$V" > $OUT/build$i.log 2>&1
  echo "$V" > $OUT/v$i.txt
  timeout -k 10 200 python bench.py --steps 10 --warmup 3 --no-cpu > $OUT/b$i.json 2> $OUT/b$i.err
done
