#!/bin/bash
# Round 3: branch-free bit helpers in the window sweeps; lane-parallel deviations from 2 vs 3 per lane.
export TMPDIR=/tmp
O=gpurun_out/r3ab
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > $O/parity.log 2>&1 || exit 1
RK_LIB=tools/mb/dp2/librepkiller_amd.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q -k "oracle or fixture or edge" --timeout 300 --timeout-method thread > $O/parity_dp2.log 2>&1 || exit 1
for rep in 1 2 3; do
  for v in new base dp2; do
    if [ $v = new ]; then L=repkiller_amd/librepkiller_amd.so; else L=tools/mb/$v/librepkiller_amd.so; fi
    RK_LIB=$L timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu > $O/bench_${v}_$rep.json 2> $O/bench_${v}_$rep.err || exit 2
  done
done
