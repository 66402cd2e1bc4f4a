#!/bin/bash
# Separate rocprofv3 PMC passes over a short bench run (MI355X_MICROARCH.md
# "rocprofv3 PMC slots": FETCH_SIZE and WRITE_SIZE never share a pass).
# Usage (on the GPU box, from the repo root): tools/pmc_run.sh OUTDIR [bench args]
set -e
OUT=${1:-gpurun_out/pmc}; shift || true
ARGS=${@:---no-cpu --steps 3 --warmup 1}
export TMPDIR=/tmp
i=0
for C in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD" "TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $C --output-format csv -d $OUT/p$i -o p -- python3 bench.py $ARGS > $OUT.p$i.log 2>&1
done
