#!/bin/bash
# Sharded path on a one-GPU box: multi-rank parity tests, the world-1 bench,
# and the two-rank rehearsal of the N > 1 line (both ranks on device 0).
export TMPDIR=/tmp
O=gpurun_out/sp
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_sharded.py -x -v --timeout 250 --timeout-method thread > $O/tests.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --mode sharded --no-cpu --steps 5 --warmup 2 > $O/p1_rccl.json 2> $O/p1_rccl.err || exit 2
RK_BENCH_SAME_GPU=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29613 bench.py --gpus 2 --config cfg2 --comm host --steps 3 --warmup 1 > $O/rehearsal2.json 2> $O/rehearsal2.err || exit 3
