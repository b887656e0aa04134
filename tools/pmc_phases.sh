#!/bin/bash
# Instruction counts per encode phase: FSEHIP_DEBUG ablations x one SQ pass.
set -e
OUT=${1:-gpurun_out/pmcph}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for D in ${PH_LIST:-8 1 18 2 4 0}; do
  FSEHIP_DEBUG=$D timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $OUT/d$D -o run --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_BUSY_CYCLES -- python3 tools/enc_once.py > $OUT/d$D.log 2>&1
done
echo phases-done
