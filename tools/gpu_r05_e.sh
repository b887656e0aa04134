#!/bin/bash
# Round 5, call E: decode LDS split -- one SQ/GRBM counter pass each over the
# product and the two one-extra-read probes (FSEHIP_ABL=256: one more
# table-like gather per pair; 512: one more payload-like read per pair).
set -o pipefail
O=gpurun_out/r05_e
mkdir -p $O
for v in libfsehip.so libfsehip_abl256.so libfsehip_abl512.so; do
  FSEHIP_LIB=$v PROF_NO_SERIAL=1 timeout -k 10 300 tools/lds_pass.sh $O/lds_$v > $O/lds_$v.log 2>&1 || { tail -20 $O/lds_$v.log; exit 1; }
  python3 tools/lds_summary.py $O/lds_$v > $O/lds_$v.txt 2>&1 || { cat $O/lds_$v.txt; exit 1; }
  echo "== $v"; grep -E "decode_blocks|build_dtables|encode" $O/lds_$v.txt || true
done
