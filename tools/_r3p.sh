#!/bin/bash
# Round 3: where the sharded driver's world-1 time goes (kernel trace), HEAD single-device line.
export TMPDIR=/tmp
O=gpurun_out/r3p
mkdir -p $O
timeout -k 10 300 python3 bench.py --mode sharded --steps 10 --warmup 3 --no-cpu > $O/bench_sh.json 2> $O/bench_sh.err || exit 1
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_sh -o p -- python3 bench.py --mode sharded --steps 10 --warmup 3 --no-cpu > $O/prof_sh.log 2>&1 || exit 2
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu > $O/bench.json 2> $O/bench.err || exit 3
