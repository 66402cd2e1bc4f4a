#!/bin/bash
# GPU suite in two steps (the full-size configs first, with per-test
# durations), then the default bench.  usage: tools/_suite.sh OUTDIR
export TMPDIR=/tmp
O=${1:-gpurun_out/suite}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_large_configs.py -m gpu -x -v --durations=0 --timeout 400 --timeout-method thread > $O/large.log 2>&1 || exit 1
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --durations=15 --timeout 300 --timeout-method thread --deselect tests/test_large_configs.py > $O/gpu_tests.log 2>&1 || exit 2
timeout -k 10 300 python bench.py --no-cpu > $O/bench.json 2> $O/bench.err || exit 3
