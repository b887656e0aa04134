# Round-2 GPU call: full GPU tests (not stopping at the first failure), smoke,
# a short bench and its kernel stats.
set -e
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests -m gpu -q --maxfail=15 --timeout 180 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || echo tests-failed
tail -5 gpurun_out/pytest_gpu.log
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && echo smoke-ok
timeout -k 10 300 python3 bench.py --no-cpu --no-sweep > gpurun_out/bench.json 2> gpurun_out/bench.err && echo bench-ok
cat gpurun_out/bench.json | head -c 1500
