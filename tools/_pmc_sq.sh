#!/bin/bash
# SQ instruction / occupancy counters per kernel (one pass), record pipeline, one stream
export TMPDIR=/tmp
O=${1:-gpurun_out/sq}
mkdir -p $O
export RK_ONE_STREAM=1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY --output-format csv -d $O/p1 -o p -- python3 bench.py --no-cpu --steps 1 --warmup 1 > $O/p1.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_ANY --output-format csv -d $O/p2 -o p -- python3 bench.py --no-cpu --steps 1 --warmup 1 > $O/p2.log 2>&1 || exit 2
