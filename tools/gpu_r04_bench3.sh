#!/bin/bash
# the bench line three times on one box (run-to-run spread of value and its parts)
O=gpurun_out/r04_bench3
mkdir -p $O
for i in 1 2 3; do
  timeout -k 10 400 python3 bench.py --no-host-calls > $O/bench$i.json 2> $O/bench$i.err || { tail -5 $O/bench$i.err; exit 1; }
  tail -1 $O/bench$i.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['encode_ms'], d['decode_ms'], d['sidecar_less_decode']['decode_GiB_s'], d['c3_decode_only']['decode_ms'])"
done
