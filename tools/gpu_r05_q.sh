#!/bin/bash
# Round 5, call Q: the emit ring's slot wrap: 24-word ring (product, compare
# wrap) padded to the 32-word ring's LDS (9 workgroups per CU) against the
# 32-word ring (mask wrap), and the product at 11 workgroups per CU.
set -o pipefail
O=gpurun_out/r05_q
mkdir -p $O
for i in 1 2; do
  for cfg in "libfsehip_diag.so 0" "libfsehip_diag.so 2048" "libfsehip_ring32.so 0"; do
    set -- $cfg
    FSEHIP_LIB=$1 FSEHIP_ENC_XLDS=$2 timeout -k 10 120 python3 tools/enc_probe.py 2>&1 | grep -v amdgpu.ids | tee -a $O/enc_ring.txt || exit 1
  done
done
