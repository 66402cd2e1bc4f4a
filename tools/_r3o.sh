#!/bin/bash
# Round 3: heap pops, unconditional round loads (parity + killer timings).
export TMPDIR=/tmp
O=gpurun_out/r3o
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k "sort" > $O/parity.log 2>&1 || exit 1
timeout -k 10 300 python3 tools/heap_killer_check.py 10000 100000 > $O/heap_killer.log 2>&1 || exit 2
