#!/bin/bash
# Round 5, call AF: the product after the in-workgroup-table code went in
# (off by default) against the library of the commit before it (ref): C3 and
# C2 decode / encode times, three rounds, same box.
set -o pipefail
O=gpurun_out/r05_af
mkdir -p $O
for i in 1 2 3; do
  for v in libfsehip_ref.so libfsehip.so; do
    FSEHIP_LIB=$v timeout -k 10 180 python3 tools/time_dec.py 2>&1 | grep -v amdgpu.ids | tee -a $O/dec_ab.txt || exit 1
  done
done
