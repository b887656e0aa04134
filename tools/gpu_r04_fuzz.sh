#!/bin/bash
# wider fuzzing of the host entry points (single-stream decoder, pinned staging)
O=gpurun_out/r04_fuzz
mkdir -p $O
FSEHIP_FUZZ_HOST_CASES=200 FSEHIP_FUZZ_DAMAGE_SEEDS=40 timeout -k 10 900 python3 -u -m pytest tests/test_gpu_fuzz.py -k "host" -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
