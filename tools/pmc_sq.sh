#!/bin/bash
# SQ counter passes (8 SQ counters at most per pass, kernel-trace only) over
# tools/prof_bench.py.  Summarise with tools/pmc_sq.py.
set -e
OUT=${1:-gpurun_out/pmc}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
i=0
while read -r SET; do
  [ -z "$SET" ] && continue
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --kernel-trace --output-format csv -d $OUT/p$i -o run --pmc $SET -- python3 tools/prof_bench.py > $OUT/p$i.log 2>&1
done <<SETS
SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS
SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS
GRBM_GUI_ACTIVE GRBM_COUNT SQ_INST_LEVEL_LDS SQ_LDS_ADDR_CONFLICT SQ_ACTIVE_INST_SCA SQ_INSTS_SMEM SQ_LDS_UNALIGNED_STALL
SETS
echo pmc-done
