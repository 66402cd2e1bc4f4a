#!/bin/bash
# GPU suite, then the default bench (no CPU leg) twice.
export TMPDIR=/tmp
O=gpurun_out/q
mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --no-cpu > $O/b1.json 2> $O/b1.err || exit 2
timeout -k 10 300 python bench.py --no-cpu > $O/b2.json 2> $O/b2.err || exit 3
