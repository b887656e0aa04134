#!/bin/bash
# Single-stream decoder (host fse_decompress2 / fse_decompress): the -m gpu
# suite, the per-call latency, the chain-latency probe; then the encoder's
# column-ring A/B.
O=gpurun_out/r04_b
mkdir -p $O
timeout -k 10 60 ./tools/micro/chain_probe > $O/chain_probe.txt 2>&1; cat $O/chain_probe.txt
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
timeout -k 10 300 python3 tools/host_latency.py > $O/host_latency.txt 2>&1 || { tail -20 $O/host_latency.txt; exit 1; }
cat $O/host_latency.txt
bash tools/gpu_variants.sh ringcol ringcol12 - ringcol
