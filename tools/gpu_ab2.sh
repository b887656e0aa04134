# A/B: full GPU suite, then the default bench (incl. the C5 sweep), no CPU leg
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -q --timeout 150 --timeout-method thread -m gpu tests > gpurun_out/t_ab.log 2>&1; rc=$?; tail -2 gpurun_out/t_ab.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 400 python bench.py --no-cpu > gpurun_out/b_ab.json 2> gpurun_out/b_ab.err || exit 1
python3 -c "
import json;d=json.load(open('gpurun_out/b_ab.json'))
print('value',d['value'],'enc',d['encode_ms'],'dec',d['decode_ms'])
for r in d['c5_sweep']['rows']: print(r['dist'][:12], r['table_log'], 'enc', r['encode_GiB_s'], 'dec', r['decode_GiB_s'], r['verified'])"
