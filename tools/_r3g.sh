#!/bin/bash
# Round 3: block heapsort (parity + killer timings), sharded driver with local parents, sweep phase profile.
export TMPDIR=/tmp
O=gpurun_out/r3g
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > $O/parity.log 2>&1 || exit 1
timeout -k 10 300 python3 tools/heap_killer_check.py 1000 10000 100000 > $O/heap_killer.log 2>&1 || exit 2
timeout -k 10 600 python -u -m pytest tests/test_sharded.py -x -q --timeout 300 --timeout-method thread > $O/sharded_tests.log 2>&1 || exit 3
timeout -k 10 300 python3 bench.py --mode sharded --steps 10 --warmup 3 --no-cpu > $O/bench_sh_nw.json 2> $O/bench_sh_nw.err || exit 4
RK_LIB=tools/mb/prof/librepkiller_amd.so RK_BENCH_NOPROF=1 timeout -k 10 300 python3 bench.py --steps 3 --warmup 1 --no-cpu > $O/bench_sweepprof.json 2> $O/bench_sweepprof.err || exit 5
