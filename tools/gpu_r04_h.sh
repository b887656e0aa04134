#!/bin/bash
# lane-parallel header parse: table / parity tests, then C2 decode timing A/B
# (diagnostics build with FSEHIP_DT_WAVE_PARSE=1 = the scalar parse, =0 = lanes)
O=gpurun_out/r04_h
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_dtables.py tests/test_gpu_c3.py tests/test_gpu_parity.py tests/test_gpu_edge.py -x -q --timeout 180 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for v in 0 1 0 1; do
  FSEHIP_LIB=libfsehip_diag.so FSEHIP_DT_WAVE_PARSE=$v timeout -k 10 120 python3 tools/time_dec.py > $O/td_wave$v.json 2> $O/td_wave$v.err || { tail -5 $O/td_wave$v.err; exit 1; }
  echo "wave_parse=$v $(cat $O/td_wave$v.json)"
done
timeout -k 10 120 python3 tools/time_dec.py > $O/td_prod.json 2> $O/td_prod.err || { tail -5 $O/td_prod.err; exit 1; }
echo "product $(cat $O/td_prod.json)"
