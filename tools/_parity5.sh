#!/bin/bash
# parity suite + full-size configs + cfg5 record/generic A/B.  usage: tools/_parity5.sh OUTDIR
export TMPDIR=/tmp
O=${1:-gpurun_out/parity5}
mkdir -p $O
tools/_parity.sh $O || exit $?
timeout -k 10 600 python -u tools/dbg/cfg5_ab.py > $O/cfg5_ab.log 2>&1 || exit 3
