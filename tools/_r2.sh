#!/bin/bash
# Round-2 check: smoke, GPU suite (without the full-size configs), bench,
# rocprofv3 kernel stats.  usage: tools/_r2.sh OUTDIR
export TMPDIR=/tmp
O=${1:-gpurun_out/r2}
mkdir -p $O
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --durations=15 --timeout 300 --timeout-method thread --deselect tests/test_large_configs.py > $O/gpu_tests.log 2>&1 || exit 2
timeout -k 10 300 python bench.py --no-cpu > $O/bench.json 2> $O/bench.err || exit 3
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o p -- python3 bench.py --no-cpu --steps 5 --warmup 2 > $O/prof.log 2>&1 || exit 4
