#!/bin/bash
# Round-4 first probe: LDS access-pattern costs (tools/micro/lds_probe), the
# encoder's phase stamps at 64 and 32 lanes per block, and the encoder
# ablation timings.  Diagnostics only.
O=gpurun_out/r04_probe
mkdir -p $O
timeout -k 10 120 ./tools/micro/lds_probe > $O/lds_probe.txt 2>&1 || { cat $O/lds_probe.txt; exit 1; }
cat $O/lds_probe.txt
for T in 64 32; do
  FSEHIP_ENC_LANES=$T ST_BYTES=$((1<<30)) timeout -k 10 300 python3 tools/stamps.py > $O/stamps_T$T.log 2>&1 || { tail -20 $O/stamps_T$T.log; exit 1; }
  grep -a "stamps" $O/stamps_T$T.log | head -30
done
ABL_LANES=64,32 timeout -k 10 300 python3 tools/ablate.py > $O/ablate.txt 2>&1 || { tail -20 $O/ablate.txt; exit 1; }
cat $O/ablate.txt
