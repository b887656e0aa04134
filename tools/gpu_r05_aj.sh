#!/bin/bash
# Round 5, call AJ: pooled-repair timing probe (encoder
# item 10).  Two blocks per 128-thread workgroup with barriers around the
# repair: pool1 = both waves repair (must give the product's bytes), pool2 =
# wave 1 skips its repair and waits (timing only).  Three rounds alternating
# with the product.
set -o pipefail
O=gpurun_out/r05_aj
mkdir -p $O
rm -f $O/digest
for i in 1 2 3; do
  AB_WIDE=1 AB_DIGEST=$O/digest FSEHIP_LIB=libfsehip.so timeout -k 10 180 python3 tools/enc_ab.py 2>&1 | grep -v amdgpu.ids | tee -a $O/pool.txt || exit 1
  AB_WIDE=1 AB_DIGEST=$O/digest FSEHIP_LIB=libfsehip_pool1.so timeout -k 10 180 python3 tools/enc_ab.py 2>&1 | grep -v amdgpu.ids | tee -a $O/pool.txt || exit 1
  AB_WIDE=1 FSEHIP_LIB=libfsehip_pool2.so timeout -k 10 180 python3 tools/enc_ab.py 2>&1 | grep -v amdgpu.ids | tee -a $O/pool.txt || exit 1
done
