#!/bin/bash
# Round 5, call AE: decode tables built inside the decode workgroups (C2
# sidecar path).  The whole -m gpu suite, then C2 decode / C3 times: the
# diagnostics build with FSEHIP_DEC_TABLE_KERNEL=1 (table kernel, as before)
# against the same build without it, and the product.
set -o pipefail
O=gpurun_out/${1:-r05_ae}
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
for i in 1 2 3; do
  FSEHIP_LIB=libfsehip_diag.so FSEHIP_DEC_TABLE_KERNEL=1 timeout -k 10 180 python3 tools/time_dec.py 2>&1 | grep -v amdgpu.ids | sed 's/^/tablekernel /' | tee -a $O/dec_inwg.txt || exit 1
  FSEHIP_LIB=libfsehip_diag.so timeout -k 10 180 python3 tools/time_dec.py 2>&1 | grep -v amdgpu.ids | sed 's/^/inwg /' | tee -a $O/dec_inwg.txt || exit 1
  FSEHIP_LIB=libfsehip.so timeout -k 10 180 python3 tools/time_dec.py 2>&1 | grep -v amdgpu.ids | sed 's/^/product /' | tee -a $O/dec_inwg.txt || exit 1
done
