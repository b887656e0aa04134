"""Decode-loop repetition test (diagnostics): FSEHIP_DEBUG = reps << 8 runs
the segment decode reps times inside each workgroup, separating the loop's
own throughput from staging and launch effects."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from entropy_coders_amd import BlockCodec  # noqa: E402
from tools.ablate import timeit  # noqa: E402

n = 1 << 30
codec = BlockCodec(ckpt_interval=128)
src = codec.generate(0, 0.155, 0x5EED0002, n)
cb = codec.compress(src)
tabs = codec.build_dtables(cb)
out = torch.empty(n, dtype=torch.uint8, device="cuda")
st = torch.zeros(codec.n_blocks(n), dtype=torch.int32, device="cuda")
for var in (0, 2, 3):
    os.environ["FSEHIP_DEC_VAR"] = str(var)
    res = []
    for reps in (1, 2, 4):
        os.environ["FSEHIP_DEBUG"] = str(reps << 8)
        res.append(timeit(lambda: codec.decompress_dt_into(cb, tabs, out, st)))
    os.environ["FSEHIP_DEBUG"] = str(1 << 4)
    dma = timeit(lambda: codec.decompress_dt_into(cb, tabs, out, st))
    os.environ["FSEHIP_DEBUG"] = "0"
    print(f"var={var} dma_only={dma:.4f} reps1={res[0]:.4f} reps2={res[1]:.4f} reps4={res[2]:.4f} "
          f"loop_per_rep={(res[2]-res[0])/3:.4f} ms", flush=True)
