#!/bin/bash
# Round 5, call AB: table-build ranks by one LDS atomic per 64 positions
# rank counters and one read per spread-walk step (wave_build_spread).  The
# table / encode / block-API GPU tests, then the decode-table kernel time and
# C2 encode, alternating the previous build (headref) and the product.
set -o pipefail
O=gpurun_out/${1:-r05_z}
mkdir -p $O
timeout -k 10 700 python3 -u -m pytest tests/test_gpu_dtables.py tests/test_gpu_blocks.py tests/test_gpu_parity.py tests/test_gpu_c3.py tests/test_gpu_edge.py tests/test_gpu_onestate.py tests/test_gpu_hygiene.py tests/test_gpu_fuzz.py -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
for i in 1 2 3; do
  for v in libfsehip_ar0.so libfsehip.so; do
    FSEHIP_LIB=$v timeout -k 10 120 python3 tools/time_dt.py 2>&1 | grep -v amdgpu.ids | tee -a $O/dt_time.txt || exit 1
    FSEHIP_LIB=$v timeout -k 10 180 python3 tools/enc_ab.py 2>&1 | grep -v amdgpu.ids | tee -a $O/enc_time.txt || exit 1
  done
done
