#!/bin/bash
# Round 3: the prefetching Y tail pass -- parity suite, bench, rocprof stats.
export TMPDIR=/tmp
O=gpurun_out/r3f
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > $O/parity.log 2>&1 || exit 1
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu > $O/bench.json 2> $O/bench.err || exit 2
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o p -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu > $O/prof.log 2>&1 || exit 3
