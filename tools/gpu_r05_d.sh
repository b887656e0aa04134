#!/bin/bash
# Round 5, call D: the 4-wave decode-table kernel (dtable_par_kernel):
# table tests against the oracle, the C2 parity / C3 tests, its time against
# the one-wave kernel (diagnostics build, FSEHIP_DT_ONE_WAVE=1), the bench.
set -o pipefail
O=gpurun_out/r05_d
mkdir -p $O
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_dtables.py tests/test_gpu_parity.py tests/test_gpu_c3.py tests/test_gpu_many.py -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 120 python3 tools/time_dt.py > $O/time_dt.txt 2>&1 || { cat $O/time_dt.txt; exit 1; }
FSEHIP_LIB=libfsehip_diag.so timeout -k 10 120 python3 tools/time_dt.py >> $O/time_dt.txt 2>&1 || { cat $O/time_dt.txt; exit 1; }
FSEHIP_LIB=libfsehip_diag.so FSEHIP_DT_ONE_WAVE=1 timeout -k 10 120 python3 tools/time_dt.py >> $O/time_dt.txt 2>&1 || { cat $O/time_dt.txt; exit 1; }
cat $O/time_dt.txt
timeout -k 10 300 python3 -u tools/many_streams.py 1 4 16 32 64 256 1000 4000 > $O/many_streams.txt 2>&1 || { tail -20 $O/many_streams.txt; exit 1; }
cat $O/many_streams.txt
timeout -k 10 500 python3 bench.py --no-sweep > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
tail -1 $O/bench.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['encode_ms'], d['decode_ms'], d['c3_decode_only']['decode_ms'], json.dumps(d.get('host_call_latency',{}).get('fse_decompress2_many_1000')))"
