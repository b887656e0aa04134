#!/bin/bash
# Round 5, call H: the emit-from-guessed-starts probe against the product
# kernel at the same occupancy (8 workgroups per CU), and the product at 11.
set -o pipefail
O=gpurun_out/r05_h
mkdir -p $O
for cfg in "libfsehip_diag.so 0" "libfsehip_diag.so 5120" "libfsehip_eprobe.so 0" "libfsehip_diag.so 0"; do
  set -- $cfg
  FSEHIP_LIB=$1 FSEHIP_ENC_XLDS=$2 timeout -k 10 120 python3 tools/enc_probe.py 2>&1 | grep -v amdgpu.ids | tee -a $O/enc_probe.txt || exit 1
done
