# A/B helper: GPU tests that cover the changed kernels, then a short bench
# (no CPU leg, no sweep) and the rocprof per-launch kernel times.
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 150 --timeout-method thread -m gpu tests > gpurun_out/t_ab.log 2>&1; rc=$?; tail -3 gpurun_out/t_ab.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --no-cpu --no-sweep > gpurun_out/b_ab.json 2> gpurun_out/b_ab.err || exit 1
python3 -c "
import json;d=json.load(open('gpurun_out/b_ab.json'))
print('value',d['value'],'enc',d['encode_ms'],'dec',d['decode_ms'],'c3',d['c3_decode_only']['decode_ms'],'serial',d['sidecar_less_decode']['decode_ms'],'ok',d['verified_roundtrip'])"
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_ab -o run -- python3 bench.py --no-cpu --no-sweep --no-serial --steps 5 > gpurun_out/prof_ab.log 2>&1 || exit 1
python3 tools/kernel_by_grid.py gpurun_out/prof_ab/run_kernel_trace.csv
