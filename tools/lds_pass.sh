#!/bin/bash
# One rocprofv3 SQ/GRBM counter pass over tools/prof_bench.py for the LDS-side
# roofline (bench.py roofline_lds): LDS-array cycles, bank-conflict cycles,
# LDS instructions and the GPU clock per launch.  Summarise with
#   python3 tools/lds_summary.py OUT --json profiles/lds.json
set -e
OUT=${1:-gpurun_out/lds}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -s KILL 240 rocprofv3 --kernel-trace --output-format csv -d $OUT/p1 -o run \
  --pmc SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS GRBM_GUI_ACTIVE -- python3 tools/prof_bench.py > $OUT/p1.log 2>&1
echo lds-pass-done
