#!/bin/bash
# Round 3: late-Y schedule A/B against the overlapped one, parity suite, heap kernel timing under rocprof.
export TMPDIR=/tmp
O=gpurun_out/r3h
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > $O/parity.log 2>&1 || exit 1
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu > $O/bench.json 2> $O/bench.err || exit 2
RK_Y_OVERLAP=1 timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu > $O/bench_overlap.json 2> $O/bench_overlap.err || exit 3
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o p -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu > $O/prof.log 2>&1 || exit 4
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/hprof -o p -- python3 tools/heap_killer_check.py 10000 100000 > $O/hprof.log 2>&1 || exit 5
