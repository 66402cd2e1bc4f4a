#!/bin/bash
# Round 3: uniform X-hit words in the late Y first pass, heap with a wavefront fence, cfg5q sharded over 8 ranks.
export TMPDIR=/tmp
O=gpurun_out/r3i
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > $O/parity.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/hprof -o p -- python3 tools/heap_killer_check.py 10000 100000 > $O/hprof.log 2>&1 || exit 2
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu > $O/bench.json 2> $O/bench.err || exit 3
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o p -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu > $O/prof.log 2>&1 || exit 4
timeout -k 10 900 python -u -m pytest tests/test_large_configs.py -x -v -k "cfg5q or cfg3" --timeout 800 --timeout-method thread > $O/large.log 2>&1 || exit 5
