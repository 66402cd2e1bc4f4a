#!/bin/bash
# Reciprocal-based deviations in the long-run walk: parity (suite, deviation boundaries, cfg5q digest), cfg5 A/B.
export TMPDIR=/tmp
O=gpurun_out/rcp
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > $O/parity.log 2>&1 || exit 1
timeout -k 10 900 python -u -m pytest tests/test_large_configs.py -x -q -k "cfg5q_oracle or cfg3" --timeout 600 --timeout-method thread > $O/large.log 2>&1 || exit 2
for v in new base; do
  if [ $v = new ]; then L=repkiller_amd/librepkiller_amd.so; else L=tools/mb/base/librepkiller_amd.so; fi
  RK_LIB=$L timeout -k 10 600 python3 bench.py --gpus 1 --config cfg5 --steps 3 --warmup 1 --no-cpu > $O/bench5_$v.json 2> $O/bench5_$v.err || exit 3
done
