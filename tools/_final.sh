#!/bin/bash
# Round-end validation on the GPU box: smoke, the GPU suite, then the profile
# refresh (bench with the CPU baseline, rocprof stats, PMC passes) and cfg5.
export TMPDIR=/tmp
O=gpurun_out/final
mkdir -p $O
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || exit 2
bash tools/_refresh.sh $O/refresh > $O/refresh.log 2>&1 || exit 3
timeout -k 10 600 python -u tools/cfg5_check.py --out $O/cfg5_check.json > $O/cfg5_check.log 2>&1 || exit 4
