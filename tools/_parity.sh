#!/bin/bash
# Quick GPU parity check of the device pipelines (test_gpu_parity.py), then
# the full-size configs.  usage: tools/_parity.sh OUTDIR
export TMPDIR=/tmp
O=${1:-gpurun_out/parity}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --durations=10 --timeout 120 --timeout-method thread > $O/parity.log 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest tests/test_large_configs.py -m gpu -x -v --durations=0 --timeout 300 --timeout-method thread > $O/large.log 2>&1 || exit 2
