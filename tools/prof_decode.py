"""Decode-only driver for rocprofv3 passes: C2 data compressed once, then
3 x decode (two-kernel path).  FSEHIP_* knobs pass through."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from entropy_coders_amd import BlockCodec  # noqa: E402

n = int(os.environ.get("PROF_BYTES", 1 << 30))
codec = BlockCodec(ckpt_interval=int(os.environ.get("PROF_CKPT", 128)))
src = codec.generate(0, 0.155, 0x5EED0002, n)
cb = codec.compress(src)
out = torch.empty(n, dtype=torch.uint8, device="cuda")
st = torch.zeros(codec.n_blocks(n), dtype=torch.int32, device="cuda")
for _ in range(3):
    codec.decompress_into(cb, out, st)
torch.cuda.synchronize()
assert torch.equal(out, src)
print("ok")
