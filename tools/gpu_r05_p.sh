#!/bin/bash
# Round 5, call P: refresh the PMC inputs of the bench line on the current
# kernels -- HBM traffic (FETCH_SIZE, WRITE_SIZE passes) and the LDS pass.
set -o pipefail
O=gpurun_out/${1:-r05_p}
mkdir -p $O
PROF_NO_SERIAL=1 timeout -k 10 600 tools/traffic.sh $O/traffic > $O/traffic.log 2>&1 || { tail -20 $O/traffic.log; exit 1; }
python3 tools/pmc_summary.py $O/traffic --json $O/traffic.json | grep -E "encode_blocks\"|decode_blocks|build_dtables" || true
PROF_NO_SERIAL=1 timeout -k 10 300 tools/lds_pass.sh $O/lds > $O/lds.log 2>&1 || { tail -20 $O/lds.log; exit 1; }
python3 tools/lds_summary.py $O/lds --json $O/lds.json | grep -E "encode_blocks |decode_blocks" || true
