# Round-end evidence, call A: the whole -m gpu suite, smoke, the HBM traffic
# passes (bench.py reads profiles/traffic.json, so they go first), then the
# default bench line.
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests -m gpu -q --maxfail=20 --timeout 180 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -4 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
timeout -k 10 180 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo smoke-failed; exit 1; }
echo smoke-ok
bash tools/traffic.sh gpurun_out/traffic || exit 1
python3 tools/pmc_summary.py gpurun_out/traffic --json gpurun_out/traffic.json > gpurun_out/traffic_summary.txt || exit 1
cp gpurun_out/traffic.json profiles/traffic.json
timeout -k 10 400 python3 bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo bench-failed; exit 1; }
echo bench-ok
head -c 1200 gpurun_out/bench.json
