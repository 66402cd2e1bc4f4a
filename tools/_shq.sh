#!/bin/bash
# Sharded driver check: multi-rank parity (host and local comms), cfg4 over 4/8 ranks, world-1 bench.
export TMPDIR=/tmp
O=${1:-gpurun_out/shq}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_sharded.py -x -q --timeout 300 --timeout-method thread > $O/sharded_tests.log 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest tests/test_large_configs.py -x -q -k "sharded" --timeout 500 --timeout-method thread > $O/large_tests.log 2>&1 || exit 2
timeout -k 10 300 python3 bench.py --mode sharded --steps 20 --warmup 5 --no-cpu > $O/bench_sh.json 2> $O/bench_sh.err || exit 3
