#!/bin/bash
# Encoder WRITE_SIZE / FETCH_SIZE per configuration (tools/enc_writes.py):
# one PMC pass each, kernel-trace only; summarise with tools/enc_writes_sum.py.
set -e
OUT=${1:-gpurun_out/encw}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -s KILL 240 rocprofv3 --kernel-trace --output-format csv -d $OUT/write -o run --pmc WRITE_SIZE -- python3 tools/enc_writes.py > $OUT/write.log 2>&1
timeout -s KILL 240 rocprofv3 --kernel-trace --output-format csv -d $OUT/fetch -o run --pmc FETCH_SIZE -- python3 tools/enc_writes.py > $OUT/fetch.log 2>&1
echo encw-done
