#!/bin/bash
# Round 5, call G: the 4-wave table kernel after hoisting the marker load and
# batching pass 1's reads: tests, stamps, A/B against the 4-wave kernel;
# the raw-call crossover of fse_decompress2_many.
set -o pipefail
O=gpurun_out/r05_g
mkdir -p $O
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_dtables.py tests/test_gpu_many.py -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 120 python3 tools/stamps_dtp.py > $O/stamps_dtp.txt 2>&1 || { tail -30 $O/stamps_dtp.txt; exit 1; }
grep -v amdgpu.ids $O/stamps_dtp.txt
for i in 1 2; do
timeout -k 10 120 python3 tools/time_dt.py 2>&1 | grep -v amdgpu.ids | tee -a $O/time_dt.txt
FSEHIP_LIB=libfsehip_diag.so FSEHIP_DT_PAR=1 timeout -k 10 120 python3 tools/time_dt.py 2>&1 | grep -v amdgpu.ids | sed 's/^/4-wave /' | tee -a $O/time_dt.txt
done
timeout -k 10 300 python3 -u tools/many_streams.py 1 16 32 64 256 1000 4000 > $O/many_streams.txt 2>&1 || { tail -20 $O/many_streams.txt; exit 1; }
cat $O/many_streams.txt
