#!/bin/bash
# Round 3: lane-parallel winner deviations in the window sweep -- parity (suite + large digests), A/B against the serial loop, sweep profile.
export TMPDIR=/tmp
O=gpurun_out/r3w
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > $O/parity.log 2>&1 || exit 1
timeout -k 10 900 python -u -m pytest tests/test_large_configs.py -x -q -k "cfg3 or cfg4_oracle or cfg5q_oracle" --timeout 600 --timeout-method thread > $O/large.log 2>&1 || exit 2
for rep in 1 2; do
  for v in new base; do
    if [ $v = new ]; then L=repkiller_amd/librepkiller_amd.so; else L=tools/mb/base/librepkiller_amd.so; fi
    RK_LIB=$L timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu > $O/bench_${v}_$rep.json 2> $O/bench_${v}_$rep.err || exit 3
  done
done
