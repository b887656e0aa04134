#!/bin/bash
# Round 5, call M: 64-byte emit groups (24-word ring): the GPU suite on the
# new kernel, then C2 encode against the previous commit's library
# (libfsehip_prev.so), alternated on one box.
set -o pipefail
O=gpurun_out/r05_m
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
for i in 1 2 3; do
  for v in libfsehip_prev.so libfsehip.so; do
    FSEHIP_LIB=$v timeout -k 10 120 python3 tools/enc_probe.py 2>&1 | grep -v amdgpu.ids | tee -a $O/enc_g64.txt || exit 1
  done
done
