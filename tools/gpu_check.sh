# GPU parity tests + bench (one call).  Usage: bash tools/gpu_check.sh [bench args]
set -e
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
timeout -k 10 300 python -u bench.py --no-cpu "$@" > gpurun_out/bench.log 2>&1
echo CHECK-OK
