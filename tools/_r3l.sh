#!/bin/bash
# Round 3: compact wire format (parity suite through rk_classify, host-to-host A/B), look-back batch A/B.
export TMPDIR=/tmp
O=gpurun_out/r3l
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > $O/parity.log 2>&1 || exit 1
timeout -k 10 300 python3 bench.py --gpus 1 --steps 10 --warmup 3 --no-cpu > $O/bench_wire.json 2> $O/bench_wire.err || exit 2
RK_WIRE=0 timeout -k 10 300 python3 bench.py --gpus 1 --steps 10 --warmup 3 --no-cpu > $O/bench_soa.json 2> $O/bench_soa.err || exit 3
for rep in 1 2; do
  for v in lb4 lb8 def; do
    if [ $v = def ]; then L=repkiller_amd/librepkiller_amd.so; else L=tools/mb/$v/librepkiller_amd.so; fi
    RK_GS_WPB=1 RK_LIB=$L timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu > $O/bench_${v}_$rep.json 2> $O/bench_${v}_$rep.err || exit 4
  done
done
for rep in 1 2; do
  for v in 1 4; do
    RK_GS_WPB=$v timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu > $O/bench_wpb${v}_$rep.json 2> $O/bench_wpb${v}_$rep.err || exit 5
  done
done
