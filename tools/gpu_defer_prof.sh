#!/bin/bash
# Occupancy of the serial decoders, then kernel statistics of the sidecar-less
# C2 decode with the symbols deferred and without.
set -o pipefail
O=gpurun_out/defer_prof
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
true

for d in 1 0; do
  FSEHIP_SERIAL_DEFER=$d NS_BYTES=$((1<<30)) NS_CASES=c2_lut0155 timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/p$d -o run -- python3 -u tools/nosidecar_time.py > $O/prof$d.log 2>&1 || { tail -20 $O/prof$d.log; exit 1; }
  grep -v amdgpu.ids $O/prof$d.log | grep c2_
  f=$(find $O/p$d -name '*kernel_stats.csv' | head -1)
  python3 -c "
import csv,sys
for r in csv.DictReader(open('$f')):
    if any(k in r['Name'] for k in ('serial_ring','sym_map','dtable')): print(r['Name'][:70], r['Calls'], round(float(r['AverageNs'])/1e6,4),'ms')
"
done
