#!/bin/bash
# Round 5, call S: shorter stateTable chains.  pkb: count / repair passes
# sum nb as packed 16-bit halves (the shift then takes nb as the sum's upper
# word, SDWA, no separate shift on the chain); sdwa: that shift forced in
# every pass (inline asm); sdpk: both.  Encode-side parity on each variant,
# then C2 encode times alternating the libraries.
set -o pipefail
O=gpurun_out/r05_s
mkdir -p $O
for v in pkb sdwa sdpk; do
  FSEHIP_LIB=libfsehip_$v.so timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_onestate.py -x -q --timeout 200 --timeout-method thread > $O/pytest_$v.log 2>&1 || { tail -30 $O/pytest_$v.log; exit 1; }
  echo "$v: $(tail -1 $O/pytest_$v.log)"
done
for i in 1 2 3; do
  for v in libfsehip.so libfsehip_pkb.so libfsehip_sdwa.so libfsehip_sdpk.so; do
    FSEHIP_LIB=$v timeout -k 10 120 python3 tools/enc_probe.py 2>&1 | grep -v amdgpu.ids | tee -a $O/enc_chain.txt || exit 1
  done
done
