#!/bin/bash
# The deferred-symbol decode with its 8 chains in one decode wave (default)
# against two (FSEHIP_SERIAL_DW=2), then the round-end evidence.
set -o pipefail
O=gpurun_out/dw
mkdir -p $O
for dw in 1 2 1; do
  FSEHIP_SERIAL_DW=$dw NS_BYTES=$((1<<30)) NS_CASES=c2_lut0155,lut077_L12 timeout -k 10 180 python -u tools/nosidecar_time.py > $O/ns_dw$dw.log 2>&1 || { cat $O/ns_dw$dw.log; exit 1; }
  echo "dw=$dw"; grep -v amdgpu.ids $O/ns_dw$dw.log
done
bash tools/gpu_final_r03b.sh
