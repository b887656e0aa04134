#!/bin/bash
# Round 5, call A: the symbol-transform source probe (tools/micro/tt_probe)
# and a rocprofv3 kernel trace of the bench without the C5 sweep, so each
# (kernel, grid) row holds only the bench's own launches.
set -o pipefail
O=gpurun_out/r05_a
mkdir -p $O
timeout -k 10 120 ./tools/micro/tt_probe > $O/tt_probe.txt 2>&1 || { tail -20 $O/tt_probe.txt; exit 1; }
cat $O/tt_probe.txt
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o bench -- python3 bench.py --no-sweep --no-cpu --no-host-calls > $O/bench_prof.json 2> $O/bench_prof.err || { tail -20 $O/bench_prof.err; exit 1; }
python3 tools/kernel_by_grid.py $(find $O/prof -name '*kernel_trace.csv' | head -1) > $O/kernel_by_grid.txt
head -20 $O/kernel_by_grid.txt
tail -1 $O/bench_prof.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['encode_ms'], d['decode_ms'], d['roofline']['frac'], d['c3_decode_only']['decode_ms'])"
