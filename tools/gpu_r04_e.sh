#!/bin/bash
# single-stream decoder: host tests + per-call latency (product library)
O=gpurun_out/r04_e
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_onestate.py tests/test_gpu_edge.py tests/test_gpu_fuzz.py -x -q --timeout 180 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python3 tools/host_latency.py > $O/host_latency.txt 2>&1 || { tail -20 $O/host_latency.txt; exit 1; }
cat $O/host_latency.txt
