#!/bin/bash
# Round 5, call O: non-temporal 64-byte group stores (FSEHIP_ENC_ABL=16) against the product.
set -o pipefail
O=gpurun_out/r05_o
mkdir -p $O
for i in 1 2 3; do
  for v in libfsehip.so libfsehip_ntg.so; do
    FSEHIP_LIB=$v timeout -k 10 120 python3 tools/enc_probe.py 2>&1 | grep -v amdgpu.ids | tee -a $O/enc_nt.txt || exit 1
  done
done
