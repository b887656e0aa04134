#!/bin/bash
# refresh profiles/traffic.json and profiles/lds.json on the current kernels
set -o pipefail
O=gpurun_out/r04_traffic
bash tools/traffic.sh $O/traffic && python3 tools/pmc_summary.py $O/traffic --json $O/traffic.json > $O/traffic_summary.txt 2>&1 && \
bash tools/lds_pass.sh $O/lds && python3 tools/lds_summary.py $O/lds --json $O/lds.json > $O/lds_summary.txt 2>&1 && echo ok
