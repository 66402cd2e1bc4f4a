#!/bin/bash
# Full GPU suite, default bench, and the two-rank rehearsal of the N>1 line.
export TMPDIR=/tmp
O=gpurun_out/rc
mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || exit 1
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err || exit 2
timeout -k 10 300 python bench.py --mode sharded --no-cpu --steps 5 --warmup 2 > $O/sharded_w1.json 2> $O/sharded_w1.err || exit 3
RK_BENCH_SAME_GPU=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus 2 --config cfg2 --comm host --steps 3 --warmup 1 > $O/rehearsal2.json 2> $O/rehearsal2.err || exit 4
