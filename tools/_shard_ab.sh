#!/bin/bash
# Sharded path: parity tests, then world-1 benches of the Y schedules
# (default after X, RK_SH_YEARLY=1 the round-3 one), interleaved.
export TMPDIR=/tmp
O=${1:-gpurun_out/shab}
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_sharded.py -x -q --timeout 250 --timeout-method thread > $O/tests.log 2>&1 || exit 1
for r in 1 2; do
  timeout -k 10 300 python bench.py --mode sharded --no-cpu --steps 20 --warmup 5 > $O/late_$r.json 2> $O/late_$r.err || exit 2
  RK_SH_YEARLY=1 timeout -k 10 300 python bench.py --mode sharded --no-cpu --steps 20 --warmup 5 > $O/early_$r.json 2> $O/early_$r.err || exit 3
done
