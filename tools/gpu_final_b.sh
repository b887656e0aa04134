# Round-end evidence, call B: rocprofv3 kernel statistics of the bench
# command, then the SQ counter passes (one counter set per pass,
# kernel-trace only).
set -e
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python3 bench.py --no-cpu --no-sweep --steps 5 > gpurun_out/prof.log 2>&1
echo prof-ok
bash tools/pmc_sq.sh gpurun_out/pmc
python3 tools/pmc_sq.py gpurun_out/pmc --json gpurun_out/pmc.json > gpurun_out/pmc_summary.txt
cat gpurun_out/pmc_summary.txt
