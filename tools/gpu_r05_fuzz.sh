#!/bin/bash
# Round 5: a widened randomized sweep of the GPU paths against the oracle
# (block batches through every decode route, crate streams through
# fsehip_decompress_streams and fse_decompress2_many, host calls).
set -o pipefail
O=gpurun_out/r05_fuzz
mkdir -p $O
FSEHIP_FUZZ_CASES=${CASES:-400} FSEHIP_FUZZ_STREAM_REPS=${REPS:-25} FSEHIP_FUZZ_SEED=${SEED:-515000} \
  timeout -k 10 1000 python3 -u -m pytest tests/test_gpu_fuzz.py -x -q --timeout 300 --timeout-method thread > $O/pytest_fuzz.log 2>&1 || { tail -40 $O/pytest_fuzz.log; exit 1; }
tail -2 $O/pytest_fuzz.log
