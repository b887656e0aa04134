#!/bin/bash
# 1-state sidecar-less decode with the symbols deferred (default) and without,
# then the round-end evidence.
set -o pipefail
O=gpurun_out/defer1
mkdir -p $O
for d in 1 0; do
  FSEHIP_SERIAL_DEFER=$d NS_STATES=1 NS_BYTES=$((1<<30)) NS_CASES=c2_lut0155 timeout -k 10 180 python -u tools/nosidecar_time.py > $O/ns1_defer$d.log 2>&1 || { cat $O/ns1_defer$d.log; exit 1; }
  echo "defer=$d"; grep -v amdgpu.ids $O/ns1_defer$d.log
done
bash tools/gpu_final_r03b.sh
