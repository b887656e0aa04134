#!/bin/bash
# Round 5, call F: phase stamps of the 4-wave table kernel, then the decode
# LDS split (tools/gpu_r05_e.sh).
set -o pipefail
O=gpurun_out/r05_f
mkdir -p $O
timeout -k 10 120 python3 tools/stamps_dtp.py > $O/stamps_dtp.txt 2>&1 || { tail -30 $O/stamps_dtp.txt; exit 1; }
cat $O/stamps_dtp.txt | grep -v amdgpu.ids
./tools/gpu_r05_e.sh
