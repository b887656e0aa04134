#!/bin/bash
# Round 5, call AC: atomic ranks behind the once-per-device lane-order check,
# peer-mask ranks as the fallback: the whole -m gpu suite, then decode-table
# and C2 encode times against the peer-rank build (ar0).
set -o pipefail
O=gpurun_out/r05_ac
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
for i in 1 2 3; do
  for v in libfsehip_ar0.so libfsehip.so; do
    FSEHIP_LIB=$v timeout -k 10 120 python3 tools/time_dt.py 2>&1 | grep -v amdgpu.ids | tee -a $O/dt_time.txt || exit 1
    FSEHIP_LIB=$v timeout -k 10 180 python3 tools/time_dec.py 2>&1 | grep -v amdgpu.ids | tee -a $O/dec_time.txt || exit 1
  done
done
