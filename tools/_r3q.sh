#!/bin/bash
# Round 3: sharded driver with fewer host round trips -- multi-rank parity, world-1 timing + trace.
export TMPDIR=/tmp
O=gpurun_out/r3s
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_sharded.py -x -q --timeout 300 --timeout-method thread > $O/sharded_tests.log 2>&1 || exit 1
timeout -k 10 300 python3 bench.py --mode sharded --steps 20 --warmup 5 --no-cpu > $O/bench_sh.json 2> $O/bench_sh.err || exit 2
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_sh -o p -- python3 bench.py --mode sharded --steps 10 --warmup 3 --no-cpu > $O/prof_sh.log 2>&1 || exit 3
timeout -k 10 600 python -u -m pytest tests/test_large_configs.py -x -q -k "cfg4_sharded" --timeout 500 --timeout-method thread > $O/large_tests.log 2>&1 || exit 4
