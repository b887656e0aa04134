# Refresh the committed evidence (one gpurun call): HBM traffic passes ->
# profiles/traffic.json, the bench line (which reads it), the 1-state bench,
# and the rocprofv3 kernel statistics of the bench command.
set -e
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out profiles
bash tools/traffic.sh gpurun_out/traffic
python3 tools/pmc_summary.py gpurun_out/traffic --json profiles/traffic.json > gpurun_out/traffic_summary.txt
timeout -k 10 300 python3 bench.py > gpurun_out/bench_full.log 2>&1
tail -1 gpurun_out/bench_full.log > profiles/r01_bench.json
timeout -k 10 300 python3 bench.py --nstates 1 --no-cpu > gpurun_out/bench_1state.log 2>&1
tail -1 gpurun_out/bench_1state.log > profiles/r01_bench_1state.json
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python3 bench.py --no-cpu --steps 5 > gpurun_out/prof.log 2>&1
cp $(find gpurun_out/prof -name "*kernel_stats.csv" | head -1) profiles/r01_bench_kernel_stats.csv
echo PROFILES-OK
