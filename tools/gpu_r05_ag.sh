#!/bin/bash
# Round 5, call AG: in-workgroup tables compiled out of the product: the
# -m gpu suite on the product, the in-workgroup route tests on the opt-in
# build (libfsehip_inwg.so), and product vs the pre-change library (ref).
set -o pipefail
O=gpurun_out/r05_ag
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
FSEHIP_LIB=libfsehip_inwg.so timeout -k 10 300 python3 -u -m pytest tests/test_gpu_inwg_tables.py -x -q --timeout 200 --timeout-method thread > $O/pytest_inwg.log 2>&1 || { tail -40 $O/pytest_inwg.log; exit 1; }
tail -1 $O/pytest_inwg.log
for i in 1 2 3; do
  for v in libfsehip_ref.so libfsehip.so; do
    FSEHIP_LIB=$v timeout -k 10 180 python3 tools/time_dec.py 2>&1 | grep -v amdgpu.ids | tee -a $O/dec_ab.txt || exit 1
  done
done
