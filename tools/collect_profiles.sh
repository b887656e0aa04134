# Copy the results of tools/gpu_profiles.sh (merged into gpurun_out/) into
# the committed profiles/ (round-1 names).
set -e
cd "$(dirname "$0")/.."
cp gpurun_out/traffic.json profiles/traffic.json
tail -1 gpurun_out/bench_full.log > profiles/r01_bench.json
tail -1 gpurun_out/bench_1state.log > profiles/r01_bench_1state.json
cp "$(find gpurun_out/prof -name '*kernel_stats.csv' | head -1)" profiles/r01_bench_kernel_stats.csv
mkdir -p profiles/r01_traffic
cp "$(find gpurun_out/traffic/fetch -name '*counter_collection.csv' | head -1)" profiles/r01_traffic/fetch_counter_collection.csv
cp "$(find gpurun_out/traffic/write -name '*counter_collection.csv' | head -1)" profiles/r01_traffic/write_counter_collection.csv
echo collected
