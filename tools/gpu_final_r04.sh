#!/bin/bash
# Round-4 evidence on the current tree: the -m gpu suite, smoke, the bench
# line, and rocprofv3 kernel statistics of the bench command.
set -o pipefail
O=gpurun_out/${1:-final_r04}
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 180 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail $O/smoke.log; exit 1; }
echo smoke-ok
timeout -k 10 500 python3 bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
tail -1 $O/bench.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['encode_ms'], d['decode_ms'], d['roofline']['frac'], d.get('roofline_lds',{}).get('frac'), d['sidecar_less_decode']['decode_GiB_s'], d['c3_decode_only']['decode_ms'], d['c3_decode_only']['roofline']['frac'], d.get('host_call_latency'))"
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o bench -- python3 bench.py --steps 5 --no-host-calls > $O/bench_prof.json 2> $O/bench_prof.err || { tail -20 $O/bench_prof.err; exit 1; }
echo prof-ok
