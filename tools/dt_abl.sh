# dtable kernel ablation: kernel statistics with FSEHIP_DT_DEBUG = 0 (full), 2 (no stores), 1 (header only)
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for D in 0 2 1; do
  FSEHIP_DT_DEBUG=$D timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/dt$D -o run -- python3 tools/prof_decode.py > gpurun_out/dt$D.log 2>&1 || true
done
echo dt-done
