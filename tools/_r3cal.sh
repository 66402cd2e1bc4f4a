#!/bin/bash
# FETCH_SIZE / WRITE_SIZE calibration on known byte counts (tools/mb/fetchcal.hip), separate PMC passes.
export TMPDIR=/tmp
O=gpurun_out/r3cal
mkdir -p $O
timeout -k 10 120 tools/mb/fetchcal > $O/run.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/f -o p -- tools/mb/fetchcal > $O/f.log 2>&1 || exit 2
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/w -o p -- tools/mb/fetchcal > $O/w.log 2>&1 || exit 3
