#!/bin/bash
# trace of the record passes (block entry included), the sharded parity tests
# and world-1 Y-schedule A/B, then the driver's bench command (CPU leg included)
export TMPDIR=/tmp
O=gpurun_out/r4d
mkdir -p $O
RK_NW_TRACE=$O/trace.bin timeout -k 10 300 python3 bench.py --no-cpu --steps 2 --warmup 1 > $O/bt.json 2> $O/bt.err || exit 1
python3 tools/nw_trace.py $O/trace.bin > $O/trace.txt 2>&1; rm -f $O/trace.bin
bash tools/_shard_ab.sh $O/shab || exit 2
timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || exit 3
