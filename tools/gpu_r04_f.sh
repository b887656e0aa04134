#!/bin/bash
# where the per-call host decode time goes: kernel and HIP API traces of 4 KiB / 64 KiB calls
O=gpurun_out/r04_f
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --hip-runtime-trace --stats -d $O/prof -o run -- python3 tools/host_latency.py 4096 65536 > $O/lat.txt 2>&1 || { tail -30 $O/lat.txt; exit 1; }
cat $O/lat.txt | grep " B "
find $O/prof -name "*stats.csv" | head
