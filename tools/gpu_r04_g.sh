#!/bin/bash
# single-stream decoder tests + per-call latency, then the LDS counter pass
bash tools/gpu_r04_e.sh || exit 1
O=gpurun_out/r04_g
bash tools/lds_pass.sh $O/lds || { tail -20 $O/lds/p1.log; exit 1; }
python3 tools/lds_summary.py $O/lds --json $O/lds.json
