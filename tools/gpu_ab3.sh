mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -q --timeout 150 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_fuzz.py > gpurun_out/t_ab.log 2>&1; rc=$?; tail -1 gpurun_out/t_ab.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
python3 -c "
import ctypes
from entropy_coders_amd._lib import load
lib=load(); buf=ctypes.create_string_buffer(4096); lib.fsehipx_occupancy(buf, 4096); print(buf.value.decode()[:600])" 2>/dev/null | grep -i encode | head -3
for i in 1 2; do timeout -k 10 400 python bench.py --no-cpu > gpurun_out/b_ab$i.json 2> gpurun_out/b_ab$i.err || exit 1
python3 -c "
import json;d=json.load(open('gpurun_out/b_ab$i.json'))
print('value',d['value'],'enc',d['encode_ms'],'dec',d['decode_ms'])
for r in d['c5_sweep']['rows']: print(r['dist'][:12], r['table_log'], 'enc', r['encode_GiB_s'], 'dec', r['decode_GiB_s'], r['verified'])"; done
