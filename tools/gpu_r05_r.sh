#!/bin/bash
# Round 5, call R: the stateTable read as a whole dword (ds_read_b32 + extract,
# FSEHIP_ENC_ABL=32) against the product's ds_read_u16: encode-side parity on
# the variant, then C2 encode times alternating the two libraries.
set -o pipefail
O=gpurun_out/r05_r
mkdir -p $O
FSEHIP_LIB=libfsehip_stu32.so timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread > $O/pytest_stu32.log 2>&1 || { tail -30 $O/pytest_stu32.log; exit 1; }
tail -1 $O/pytest_stu32.log
for i in 1 2 3; do
  for v in libfsehip.so libfsehip_stu32.so; do
    FSEHIP_LIB=$v timeout -k 10 120 python3 tools/enc_probe.py 2>&1 | grep -v amdgpu.ids | tee -a $O/enc_stu32.txt || exit 1
  done
done
