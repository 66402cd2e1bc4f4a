#!/bin/bash
# Round 3: the driver's bench command on HEAD, the Y-serial A/B, its rocprof summary, then the GPU suite.
export TMPDIR=/tmp
O=gpurun_out/r3b
mkdir -p $O
timeout -k 10 400 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || exit 1
RK_Y_SERIAL=1 timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu > $O/bench_yser.json 2> $O/bench_yser.err || exit 2
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o p -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu > $O/prof.log 2>&1 || exit 3
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || exit 4
