#!/bin/bash
# Round 5, call AD: the encoder's phase ablations at 11 workgroups per CU on
# the final kernel (diagnostics build), twice, for DESIGN's phase table.
set -o pipefail
O=gpurun_out/r05_ad
mkdir -p $O
for i in 1 2; do
  OCC_WGS=11 OCC_BASE_LDS=14640 timeout -k 10 300 python3 tools/enc_phase_occ.py 2>&1 | grep -v amdgpu.ids | tee -a $O/phases.txt || exit 1
done
