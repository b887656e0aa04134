#!/bin/bash
# Round 5, call Y: upper bound for taking the payload read off LDS (verdict
# r04 item 3's "payload words held in VGPRs"): FSEHIP_ABL=1024 takes each
# pair's payload word from registers (wrong output, timing only) -- the time
# a VGPR-window decoder could reach before paying for its window logic.
set -o pipefail
O=gpurun_out/r05_y
mkdir -p $O
for i in 1 2 3; do
  for v in libfsehip.so libfsehip_abl1024.so; do
    FSEHIP_LIB=$v timeout -k 10 180 python3 tools/time_dec.py 2>&1 | grep -v amdgpu.ids | tee -a $O/dec_nopayload.txt || exit 1
  done
done
