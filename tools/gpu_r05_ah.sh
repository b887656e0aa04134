#!/bin/bash
# Round 5, call AH: is the encoder's LDS pad (pad11: LDS per workgroup =
# 160 KiB / 11 - 64) now costing it a workgroup per CU?  LDS is allocated in
# whole granules: 14,640 B static + the pad = 14,830 B may round past 160 KiB
# / 11.  The product against FSEHIP_ENC_WGS=12 (no pad at 14,640 B).
set -o pipefail
O=gpurun_out/r05_ah
mkdir -p $O
for i in 1 2 3; do
  for v in libfsehip.so libfsehip_wgs12.so; do
    AB_WIDE=1 FSEHIP_LIB=$v timeout -k 10 180 python3 tools/enc_ab.py 2>&1 | grep -v amdgpu.ids | tee -a $O/enc_pad.txt || exit 1
  done
done
