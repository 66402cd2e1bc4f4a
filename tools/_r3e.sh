#!/bin/bash
# Round 3: local Y parents written in place -- sharded parity, world-1 timing, the N=2 bench rehearsal on one GPU.
export TMPDIR=/tmp
O=gpurun_out/r3e
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_sharded.py -x -v --timeout 300 --timeout-method thread > $O/sharded_tests.log 2>&1 || exit 1
timeout -k 10 300 python3 bench.py --mode sharded --steps 10 --warmup 3 --no-cpu > $O/bench_sh_nw.json 2> $O/bench_sh_nw.err || exit 2
bash tools/_rehearse.sh $O/reh || exit 3
