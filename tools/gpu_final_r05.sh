#!/bin/bash
# Round-5 evidence on the current tree: the -m gpu suite, smoke, the bench
# line, and a rocprofv3 kernel trace of the bench without the C5 sweep (so
# each (kernel, grid) row holds only the bench's own launches) with the
# fractions recomputed from it (tools/frac_check.py).
set -o pipefail
O=gpurun_out/${1:-final_r05}
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 180 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail $O/smoke.log; exit 1; }
echo smoke-ok
timeout -k 10 500 python3 bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
tail -1 $O/bench.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['encode_ms'], d['decode_ms'], d['roofline']['frac'], d['roofline_lds'].get('ceiling_hbm_frac'), d['sidecar_less_decode']['decode_GiB_s'], d['c3_decode_only']['decode_ms'], d['c3_decode_only']['roofline']['frac'], d['c3_decode_only']['roofline_lds'].get('ceiling_hbm_frac'), json.dumps(d.get('host_call_latency',{}).get('fse_decompress2_many_1000')))"
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o bench -- python3 bench.py --no-sweep --no-cpu --no-host-calls > $O/bench_prof.json 2> $O/bench_prof.err || { tail -20 $O/bench_prof.err; exit 1; }
python3 tools/kernel_by_grid.py $O/prof/bench_kernel_trace.csv > $O/kernel_by_grid.txt
python3 tools/frac_check.py $O/bench_prof.json $O/prof/bench_kernel_trace.csv | tee $O/frac_check.txt
