#!/bin/bash
# Round 3: per-phase shader cycles of the first window sweep and of the LDS group-sort tiers (measurement builds).
export TMPDIR=/tmp
O=gpurun_out/r3x
mkdir -p $O
RK_LIB=tools/mb/sprof/librepkiller_amd.so timeout -k 10 300 python3 bench.py --gpus 1 --steps 2 --warmup 1 --no-cpu > $O/sprof.json 2> $O/sprof.err || exit 1
