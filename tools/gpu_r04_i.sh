#!/bin/bash
# kernel durations of the table build: lane-parallel header parse vs the scalar parse
O=gpurun_out/r04_i
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
for v in 0 1; do
  FSEHIP_LIB=libfsehip_diag.so FSEHIP_DT_WAVE_PARSE=$v timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/p$v -o run -- python3 tools/time_dec.py > $O/td$v.json 2> $O/td$v.err || { tail -5 $O/td$v.err; exit 1; }
done
echo done
