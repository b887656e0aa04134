#!/bin/bash
# Round 5, call J: emit-pass source prefetch depth (FSEHIP_ENC_PF 4 = product,
# 6, 8): exactness of the variants on the parity tests, then C2 encode times
# alternated on one box.
set -o pipefail
O=gpurun_out/r05_j
mkdir -p $O
for v in pf8 pf6; do
  FSEHIP_LIB=libfsehip_$v.so timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_c3.py -x -q --timeout 200 --timeout-method thread > $O/pytest_$v.log 2>&1 || { tail -30 $O/pytest_$v.log; exit 1; }
  echo "$v: $(tail -1 $O/pytest_$v.log)"
done
for i in 1 2 3; do
  for v in libfsehip.so libfsehip_pf6.so libfsehip_pf8.so; do
    FSEHIP_LIB=$v timeout -k 10 120 python3 tools/enc_probe.py 2>&1 | grep -v amdgpu.ids | tee -a $O/enc_pf.txt || exit 1
  done
done
