#!/bin/bash
# Round 5, call B: the batched host-call tests, the 8-rank C4 rehearsal on
# card 0, the crossover sweep, then a bench line.
set -o pipefail
O=gpurun_out/r05_b
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_many.py tests/test_gpu_dist.py -x -v --timeout 450 --timeout-method thread -s > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
grep -E "PASS|FAIL|value|c4|passed|failed" $O/pytest.log | tail -20
timeout -k 10 300 python3 -u tools/many_streams.py > $O/many_streams.txt 2>&1 || { tail -20 $O/many_streams.txt; exit 1; }
cat $O/many_streams.txt
timeout -k 10 500 python3 bench.py --no-sweep > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
tail -1 $O/bench.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['encode_ms'], d['decode_ms'], json.dumps(d.get('host_call_latency')))"
