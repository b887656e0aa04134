#!/bin/bash
# One SQ counter pass over tools/enc_once.py per FSEHIP_ENC_LANES value.
set -e
OUT=${1:-gpurun_out/pmcvar}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for T in 64 32; do
  FSEHIP_ENC_LANES=$T timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $OUT/d$T -o run --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES -- python3 tools/enc_once.py > $OUT/d$T.log 2>&1
  FSEHIP_ENC_LANES=$T timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $OUT/e$T -o run --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INST_LEVEL_LDS -- python3 tools/enc_once.py > $OUT/e$T.log 2>&1
done
echo var-done
