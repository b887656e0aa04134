#!/bin/bash
# LDS cycles and bank-conflict cycles per encode ablation level (FSEHIP_DEBUG).
set -e
OUT=${1:-gpurun_out/pmclds}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for D in 8 1 18 2 4 0; do
  FSEHIP_DEBUG=$D timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $OUT/d$D -o run --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_LDS_ADDR_CONFLICT SQ_INSTS_VALU SQ_WAVE_CYCLES GRBM_GUI_ACTIVE -- python3 tools/enc_once.py > $OUT/d$D.log 2>&1
done
echo lds-done
