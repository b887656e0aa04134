# One gpurun call: the whole -m gpu suite, smoke, then the default bench
# line (BENCH_ARGS adds bench.py arguments).  Stops at the first failure.
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests -m gpu -q -x --timeout 180 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -4 gpurun_out/pytest_gpu.log
[ $rc -ne 0 ] && { echo "pytest rc=$rc: stopping"; exit $rc; }
timeout -k 10 180 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo smoke-failed; exit 1; }
echo smoke-ok
timeout -k 10 400 python3 bench.py $BENCH_ARGS > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo bench-failed; tail -5 gpurun_out/bench.err; exit 1; }
echo bench-ok
head -c 1500 gpurun_out/bench.json
