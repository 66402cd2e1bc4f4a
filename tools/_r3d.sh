#!/bin/bash
# Round 3: sharded record driver after the partition / roots / shortcut changes -- parity, world-1 timing, cfg4 over 4/8 ranks; FETCH_SIZE calibration.
export TMPDIR=/tmp
O=gpurun_out/r3d
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_sharded.py -x -v --timeout 300 --timeout-method thread > $O/sharded_tests.log 2>&1 || exit 1
timeout -k 10 300 python3 bench.py --mode sharded --steps 10 --warmup 3 --no-cpu > $O/bench_sh_nw.json 2> $O/bench_sh_nw.err || exit 2
timeout -k 10 600 python -u -m pytest tests/test_large_configs.py -x -v -k "sharded" --timeout 500 --timeout-method thread > $O/large_tests.log 2>&1 || exit 3
bash tools/_r3cal.sh || exit 4
