#!/bin/bash
# Round 3: sharded world-1 A/B: Y head beside X (default) vs serial; run-aggregated member histogram.
export TMPDIR=/tmp
O=gpurun_out/r3r
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_sharded.py -x -q --timeout 300 --timeout-method thread > $O/sharded_tests.log 2>&1 || exit 1
for rep in 1 2; do
  timeout -k 10 300 python3 bench.py --mode sharded --steps 20 --warmup 5 --no-cpu > $O/bench_sh_$rep.json 2> $O/bench_sh_$rep.err || exit 2
  RK_SH_YSERIAL=1 timeout -k 10 300 python3 bench.py --mode sharded --steps 20 --warmup 5 --no-cpu > $O/bench_shs_$rep.json 2> $O/bench_shs_$rep.err || exit 3
done
