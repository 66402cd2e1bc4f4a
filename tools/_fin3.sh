#!/bin/bash
# round-3 close on HEAD: smoke, the GPU suite, the driver's bench command (with
# the CPU baseline), and the bench with the per-kernel timers off (their cost)
export TMPDIR=/tmp
O=gpurun_out/fin3
mkdir -p $O
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || exit 2
timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || exit 3
for r in 1 2; do
  RK_BENCH_NOPROF=1 timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu > $O/bench_noprof_$r.json 2> $O/bench_noprof_$r.err || exit 4
  timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu > $O/bench_prof_$r.json 2> $O/bench_prof_$r.err || exit 5
done
