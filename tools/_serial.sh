#!/bin/bash
# Per-kernel times with every kernel on one stream (RK_ONE_STREAM=1), cfg5 and cfg3.
export TMPDIR=/tmp
O=gpurun_out/serial
mkdir -p $O
RK_ONE_STREAM=1 timeout -k 10 400 python bench.py --config cfg5 --no-cpu --steps 2 --warmup 1 > $O/cfg5.json 2> $O/cfg5.err || exit 1
RK_ONE_STREAM=1 timeout -k 10 300 python bench.py --no-cpu > $O/cfg3.json 2> $O/cfg3.err || exit 2
