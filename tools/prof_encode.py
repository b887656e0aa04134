"""Encode-only driver for rocprofv3: C2 data, 3 x encode (FSEHIP_* knobs pass through)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from entropy_coders_amd import BlockCodec  # noqa: E402

n = int(os.environ.get("PROF_BYTES", 1 << 30))
codec = BlockCodec()
src = codec.generate(0, 0.155, 0x5EED0002, n)
cb = codec.alloc(n)
for _ in range(3):
    codec.compress_into(src, cb)
torch.cuda.synchronize()
print("ok")
