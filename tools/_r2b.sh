#!/bin/bash
# Round-end second half (on the GPU box): cfg5 at full size (check + bench
# line), the sharded driver at world size 1, and the two-rank rehearsal.
export TMPDIR=/tmp
O=gpurun_out/final
mkdir -p $O
timeout -k 10 600 python -u tools/cfg5_check.py --out $O/cfg5_check.json > $O/cfg5_check.log 2>&1 || exit 1
timeout -k 10 400 python bench.py --config cfg5 --no-cpu --steps 3 --warmup 1 > $O/bench_cfg5.json 2> $O/bench_cfg5.err || exit 2
timeout -k 10 300 python bench.py --mode sharded --no-cpu --steps 5 --warmup 2 > $O/sharded_w1.json 2> $O/sharded_w1.err || exit 3
RK_BENCH_SAME_GPU=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus 2 --config cfg2 --comm host --steps 3 --warmup 1 > $O/rehearsal2.json 2> $O/rehearsal2.err || exit 4
