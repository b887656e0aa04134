# Refresh the committed evidence (one gpurun call): HBM traffic passes ->
# profiles/traffic.json, the bench line (which reads it), the 1-state bench,
# and the rocprofv3 kernel statistics of the bench command.  Results land in
# gpurun_out/; tools/collect_profiles.sh copies them into profiles/.
set -e
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out profiles
bash tools/traffic.sh gpurun_out/traffic
python3 tools/pmc_summary.py gpurun_out/traffic --json gpurun_out/traffic.json > gpurun_out/traffic_summary.txt && cp gpurun_out/traffic.json profiles/traffic.json
timeout -k 10 400 python3 bench.py > gpurun_out/bench_full.log 2>&1

timeout -k 10 300 python3 bench.py --nstates 1 --no-cpu > gpurun_out/bench_1state.log 2>&1

cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python3 bench.py --no-cpu --no-sweep --steps 5 > gpurun_out/prof.log 2>&1

echo PROFILES-OK
