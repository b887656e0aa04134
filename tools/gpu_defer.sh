#!/bin/bash
# One gpurun call: the -m gpu suite, then the sidecar-less decode with the
# symbols deferred (default) against the single-kernel serial decode
# (FSEHIP_SERIAL_DEFER=0), then the bench line.
set -o pipefail
O=gpurun_out/defer
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
for d in 1 0 1; do
  FSEHIP_SERIAL_DEFER=$d NS_BYTES=$((1<<30)) NS_CASES=c2_lut0155,lut077_L12 timeout -k 10 180 python -u tools/nosidecar_time.py > $O/ns_defer$d.log 2>&1 || { cat $O/ns_defer$d.log; exit 1; }
  echo "defer=$d"; grep -v amdgpu.ids $O/ns_defer$d.log
done
timeout -k 10 300 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
tail -1 $O/bench.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['sidecar_less_decode'])"
