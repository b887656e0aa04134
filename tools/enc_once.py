"""One encode of 1 GiB of C2 data (for rocprofv3 counter passes; FSEHIP_DEBUG
selects an ablation: 8 = histogram only, 1 = + tables, 2 = + count/repair,
0 = full kernel)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
# the environment knobs this tool sets live only in the diagnostics build
os.environ.setdefault("FSEHIP_LIB", "libfsehip_diag.so")

import torch  # noqa: E402

from entropy_coders_amd import BlockCodec  # noqa: E402

n = int(os.environ.get("PROF_BYTES", 1 << 30))
codec = BlockCodec()
src = codec.generate(int(os.environ.get("PROF_KIND", 0)), float(os.environ.get("PROF_PROB", 0.155)), 0x5EED0002, n)
cb = codec.alloc(n)
codec.compress_into(src, cb)
torch.cuda.synchronize()
print("ok")
