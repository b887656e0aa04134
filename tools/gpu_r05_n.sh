#!/bin/bash
# Round 5, call N: 64-byte emit groups with 4-word head / tail pieces: the
# encode-side GPU tests, then C2 encode against the previous commit's library.
set -o pipefail
O=gpurun_out/r05_n
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_c3.py tests/test_gpu_fuzz.py tests/test_gpu_edge.py tests/test_gpu_onestate.py -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
for i in 1 2 3; do
  for v in libfsehip_prev.so libfsehip.so; do
    FSEHIP_LIB=$v timeout -k 10 120 python3 tools/enc_probe.py 2>&1 | grep -v amdgpu.ids | tee -a $O/enc_g64q.txt || exit 1
  done
done
