#!/bin/bash
# Round 3: the sharded driver on the record pipeline -- multi-rank parity, world-1 timing (record vs generic), cfg4 over 4/8 ranks.
export TMPDIR=/tmp
O=gpurun_out/r3c
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_sharded.py -x -v --timeout 300 --timeout-method thread > $O/sharded_tests.log 2>&1 || exit 1
timeout -k 10 300 python3 bench.py --mode sharded --steps 10 --warmup 3 --no-cpu > $O/bench_sh_nw.json 2> $O/bench_sh_nw.err || exit 2
RK_SHARD_GENERIC=1 timeout -k 10 300 python3 bench.py --mode sharded --steps 10 --warmup 3 --no-cpu > $O/bench_sh_gen.json 2> $O/bench_sh_gen.err || exit 3
timeout -k 10 600 python -u -m pytest tests/test_large_configs.py -x -v -k "sharded or cfg5q" --timeout 500 --timeout-method thread > $O/large_tests.log 2>&1 || exit 4
