# Round-2 GPU call: tests, bench (1 GPU and a 2-rank gloo rehearsal of the
# self-launch on one card), kernel stats, traffic and SQ passes.
set -e
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
echo tests-ok
timeout -k 10 300 python3 bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err
echo bench-ok
FSEHIP_BENCH_BACKEND=gloo timeout -k 10 300 python3 bench.py --gpus 2 --bytes 268435456 --steps 5 --warmup 2 > gpurun_out/bench_gloo2.json 2> gpurun_out/bench_gloo2.err
echo gloo2-ok
FSEHIP_BENCH_BACKEND=gloo timeout -k 10 300 python3 bench.py --gpus 2 --strong --bytes 268435456 --steps 5 --warmup 2 --scheme contiguous > gpurun_out/bench_gloo2s.json 2> gpurun_out/bench_gloo2s.err
echo gloo2s-ok
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python3 bench.py --no-cpu --no-sweep --steps 5 > gpurun_out/prof.log 2>&1
echo prof-ok
bash tools/traffic.sh gpurun_out/traffic
python3 tools/pmc_summary.py gpurun_out/traffic --json gpurun_out/traffic.json > gpurun_out/traffic_summary.txt
bash tools/pmc_sq.sh gpurun_out/pmc
python3 tools/pmc_sq.py gpurun_out/pmc --json gpurun_out/r02_pmc.json > gpurun_out/pmc_summary.txt
echo ALL-OK
