#!/bin/bash
# the full-size configs (cfg3 reference hash, cfg4 oracle digest, cfg5) and the cfg5 bench
export TMPDIR=/tmp
O=${1:-gpurun_out/large}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_large_configs.py -m gpu -x -v --durations=0 --timeout 400 --timeout-method thread > $O/large.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --config cfg5 --no-cpu --steps 3 --warmup 1 > $O/cfg5.json 2> $O/cfg5.err || exit 2
