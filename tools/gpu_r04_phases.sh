#!/bin/bash
# Encoder phase ablations x occupancy, then SQ counters per ablation.
O=gpurun_out/r04_phases
mkdir -p $O
timeout -k 10 60 ./tools/micro/lds_probe > $O/lds_probe2.txt 2>&1 && grep hist $O/lds_probe2.txt
timeout -k 10 400 python3 tools/enc_phase_occ.py > $O/phase_occ.txt 2>&1 || { tail -20 $O/phase_occ.txt; exit 1; }
cat $O/phase_occ.txt
ABL_KIND=0 ABL_PROB=0.77 ABL_LOG=12 OCC_WGS=11,6 timeout -k 10 400 python3 tools/enc_phase_occ.py > $O/phase_occ_skew12.txt 2>&1 || { tail -20 $O/phase_occ_skew12.txt; exit 1; }
cat $O/phase_occ_skew12.txt
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for D in 8 1 18 2 4 0; do
  FSEHIP_DEBUG=$D timeout -s KILL 90 rocprofv3 --kernel-trace --output-format csv -d $O/pmc_d$D -o run --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU -- python3 tools/enc_once.py > $O/pmc_d$D.log 2>&1 || { tail -5 $O/pmc_d$D.log; exit 1; }
done
echo pmc-done
