#!/bin/bash
# Round 5, call AI: three bench.py runs back to back on one box (the spread
# of the line).
set -o pipefail
O=gpurun_out/r05_ai
mkdir -p $O
for i in 1 2 3; do
  timeout -k 10 500 python3 bench.py > $O/bench$i.json 2> $O/bench$i.err || { tail -20 $O/bench$i.err; exit 1; }
  tail -1 $O/bench$i.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['encode_ms'], d['decode_ms'], d['c3_decode_only']['decode_ms'], d['sidecar_less_decode']['decode_GiB_s'])"
done
