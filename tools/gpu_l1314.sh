cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_blocks.py tests/test_gpu_dtables.py tests/test_gpu_fuzz.py -m gpu -q -x --timeout 150 --timeout-method thread > gpurun_out/pt_l1314.log 2>&1
rc=$?; tail -3 gpurun_out/pt_l1314.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python3 bench.py --no-cpu --no-serial --no-c3 --steps 3 --warmup 1 > gpurun_out/bench_l1314.json 2> gpurun_out/bench_l1314.err || { tail -5 gpurun_out/bench_l1314.err; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/bench_l1314.json'))
for r in d['c5_sweep']['rows']: print(r['dist'][:12], r['table_log'], r['encode_GiB_s'], r['decode_GiB_s'], r['verified'])
"
