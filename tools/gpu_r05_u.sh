#!/bin/bash
# Round 5, call U: symbol transforms loaded one chunk ahead (enc_chunk_pl,
# FSEHIP_ENC_TTPF).  The encode-side GPU tests on the new product, then
# C2 / geometric / skewed encode times alternating ttpf0 (the previous
# product) and the product, with a byte digest of the C2 output.
set -o pipefail
O=gpurun_out/r05_u
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_c3.py tests/test_gpu_fuzz.py tests/test_gpu_edge.py tests/test_gpu_onestate.py -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
rm -f $O/c2.sha
for i in 1 2 3; do
  for v in libfsehip_ttpf0.so libfsehip.so; do
    AB_WIDE=1 AB_DIGEST=$O/c2.sha FSEHIP_LIB=$v timeout -k 10 180 python3 tools/enc_ab.py 2>&1 | grep -v amdgpu.ids | tee -a $O/enc_ttpf.txt || exit 1
  done
done
