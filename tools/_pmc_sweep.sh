#!/bin/bash
export TMPDIR=/tmp
O=gpurun_out/pmcsw
mkdir -p $O
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_WR SQ_INSTS_VALU SQ_WAVES SQ_INSTS_BRANCH SQ_INSTS_SENDMSG --output-format csv -d $O/p1 -o p -- python3 bench.py --no-cpu --steps 2 --warmup 1 > $O/p1.log 2>&1 || exit 1
