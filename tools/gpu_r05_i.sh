#!/bin/bash
# Round 5, call I: the grouped many-stream call (tests, fuzz of the stream
# sets, crossover).
set -o pipefail
O=gpurun_out/r05_i
mkdir -p $O
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_many.py tests/test_gpu_fuzz.py -k "many" -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python3 -u tools/many_streams.py 1 16 64 256 1000 4000 > $O/many_streams.txt 2>&1 || { tail -20 $O/many_streams.txt; exit 1; }
cat $O/many_streams.txt
