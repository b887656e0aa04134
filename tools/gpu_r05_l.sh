#!/bin/bash
# Round 5, call L: payload store shape probes (timing only, wrong output):
# the same bytes as whole aligned 64-byte pieces (FSEHIP_ENC_ABL=16) or
# 128-byte lines (32), against the product and the no-store probe (8).
set -o pipefail
O=gpurun_out/r05_l
mkdir -p $O
for i in 1 2 3; do
  for v in libfsehip.so libfsehip_st64.so libfsehip_st128.so libfsehip_nogst.so; do
    FSEHIP_LIB=$v timeout -k 10 120 python3 tools/enc_probe.py 2>&1 | grep -v amdgpu.ids | tee -a $O/enc_store_shape.txt || exit 1
  done
done
