#!/bin/bash
# Round 5, call V: encoder LDS split -- one SQ/GRBM counter pass each over
# the product and two one-extra-gather probes (FSEHIP_ENC_ABL=64: one more
# stateTable gather per pair; 128: one more transform gather per pair), and
# the C2 encode time of each (what one more gather per pair costs).
set -o pipefail
O=gpurun_out/r05_v
mkdir -p $O
for v in libfsehip.so libfsehip_est.so libfsehip_ett.so; do
  FSEHIP_LIB=$v PROF_NO_SERIAL=1 PROF_NO_C3=1 timeout -k 10 300 tools/lds_pass.sh $O/lds_$v > $O/lds_$v.log 2>&1 || { tail -20 $O/lds_$v.log; exit 1; }
  python3 tools/lds_summary.py $O/lds_$v > $O/lds_$v.txt 2>&1 || { cat $O/lds_$v.txt; exit 1; }
  echo "== $v"; grep -E "encode_blocks " $O/lds_$v.txt || true
done
for i in 1 2; do
  for v in libfsehip.so libfsehip_est.so libfsehip_ett.so; do
    FSEHIP_LIB=$v timeout -k 10 180 python3 tools/enc_ab.py 2>&1 | grep -v amdgpu.ids | tee -a $O/enc_split_time.txt || exit 1
  done
done
