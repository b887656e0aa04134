#!/bin/bash
# Round 5, call X: two decode pairs per payload read (LdsChain::pair2,
# FSEHIP_DEC_PAIR2).  The decode-side GPU tests on the new product, then
# C3 / C2 decode times alternating p2off (one read per pair) and the product.
set -o pipefail
O=gpurun_out/r05_x
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_c3.py tests/test_gpu_fuzz.py tests/test_gpu_edge.py tests/test_gpu_onestate.py tests/test_gpu_dtables.py -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
for i in 1 2 3; do
  for v in libfsehip_p2off.so libfsehip.so; do
    FSEHIP_LIB=$v timeout -k 10 180 python3 tools/time_dec.py 2>&1 | grep -v amdgpu.ids | tee -a $O/dec_pair2.txt || exit 1
  done
done
