#!/bin/bash
# Round 5, call K: where the emit pass's payload stores cost (timing probes,
# wrong output): no ring reads (FSEHIP_ENC_ABL=4), no group stores (8), stores
# into L2-resident lines (1), against the product, alternated on one box.
set -o pipefail
O=gpurun_out/r05_k
mkdir -p $O
for i in 1 2 3; do
  for v in libfsehip.so libfsehip_noringrd.so libfsehip_nogst.so libfsehip_l2st.so; do
    FSEHIP_LIB=$v timeout -k 10 120 python3 tools/enc_probe.py 2>&1 | grep -v amdgpu.ids | tee -a $O/enc_store.txt || exit 1
  done
done
