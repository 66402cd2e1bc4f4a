#!/bin/bash
# GPU suite, then BASELINE cfg5 (1B fragments) on one GPU: checks + bench line.
export TMPDIR=/tmp
O=gpurun_out/c5
mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || exit 1
timeout -k 10 600 python -u tools/cfg5_check.py --out $O/cfg5_check.json > $O/cfg5_check.log 2>&1 || exit 2
timeout -k 10 400 python bench.py --config cfg5 --no-cpu --steps 3 --warmup 1 > $O/bench_cfg5.json 2> $O/bench_cfg5.err || exit 3
timeout -k 10 300 python bench.py --no-cpu > $O/bench_cfg3.json 2> $O/bench_cfg3.err || exit 4
