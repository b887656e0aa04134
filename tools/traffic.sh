#!/bin/bash
# HBM traffic per kernel launch: two rocprofv3 PMC passes (FETCH_SIZE and
# WRITE_SIZE cannot share a pass on gfx950), kernel-trace only, over
# tools/prof_bench.py.  Summarise with tools/pmc_summary.py.
set -e
OUT=${1:-gpurun_out/traffic}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -s KILL 240 rocprofv3 --kernel-trace --output-format csv -d $OUT/fetch -o run --pmc FETCH_SIZE -- python3 tools/prof_bench.py > $OUT/fetch.log 2>&1
timeout -s KILL 240 rocprofv3 --kernel-trace --output-format csv -d $OUT/write -o run --pmc WRITE_SIZE -- python3 tools/prof_bench.py > $OUT/write.log 2>&1
echo traffic-done
