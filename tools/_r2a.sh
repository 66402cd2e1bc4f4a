#!/bin/bash
# Round-end first half (on the GPU box): smoke, the GPU suite, then the
# profile refresh (bench with the CPU baseline, rocprof stats, PMC passes).
export TMPDIR=/tmp
O=gpurun_out/final
mkdir -p $O
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || exit 2
tools/_refresh.sh $O/refresh > $O/refresh.log 2>&1 || exit 3
