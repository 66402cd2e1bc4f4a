#!/bin/bash
# The N>1 bench line rehearsed on one GPU: two ranks on device 0, the sharded
# leg over gloo host callbacks (promoted to value) and over RCCL (which refuses
# two ranks on one GPU: the replicas value stands, with the error), then the
# sharded world-1 leg at cfg3.
export TMPDIR=/tmp
O=${1:-gpurun_out/reh}
mkdir -p $O
RK_BENCH_SAME_GPU=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus 2 --config cfg2 --comm host --steps 3 --warmup 1 > $O/host2.json 2> $O/host2.err || exit 1
RK_BENCH_SAME_GPU=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29612 bench.py --gpus 2 --config cfg2 --steps 3 --warmup 1 --sharded-timeout 60 > $O/rccl2.json 2> $O/rccl2.err
echo "rccl2 exit $?" > $O/rccl2.rc
timeout -k 10 300 python bench.py --mode sharded --no-cpu --steps 5 --warmup 2 > $O/sharded_w1.json 2> $O/sharded_w1.err || exit 3
