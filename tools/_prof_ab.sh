#!/bin/bash
# the bench with only the roofline kernel's launches timed inside the timed
# steps (default) against every launch timed there (RK_BENCH_ALLPROF=1) and no
# timers (RK_BENCH_NOPROF=1); then the tests that read the timing
export TMPDIR=/tmp
O=gpurun_out/pab
mkdir -p $O
timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || exit 1
for r in 1 2; do
  timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu > $O/b_only_$r.json 2> $O/b_only_$r.err || exit 2
  RK_BENCH_ALLPROF=1 timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu > $O/b_all_$r.json 2> $O/b_all_$r.err || exit 3
  RK_BENCH_NOPROF=1 timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu > $O/b_none_$r.json 2> $O/b_none_$r.err || exit 4
done
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "profil or timing or bench or smoke or shard" > $O/tests.log 2>&1 || exit 5
