#!/bin/bash
# Sharded path on a one-GPU box: multi-rank parity tests, then the world-1 bench.
export TMPDIR=/tmp
O=gpurun_out/sp
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_sharded.py -x -v --timeout 250 --timeout-method thread > $O/tests.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --mode sharded --no-cpu --steps 5 --warmup 2 > $O/p1_rccl.json 2> $O/p1_rccl.err || exit 2
