"""Small driver for rocprofv3 PMC passes: 2 x (encode + decode) of C2 data."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from entropy_coders_amd import BlockCodec  # noqa: E402

n = int(os.environ.get("PROF_BYTES", 1 << 30))
codec = BlockCodec(nstates=int(os.environ.get("PROF_NSTATES", 2)))
src = codec.generate(0, 0.155, 0x5EED0002, n)
cb = codec.alloc(n)
out = torch.empty(n, dtype=torch.uint8, device="cuda")
st = torch.zeros(codec.n_blocks(n), dtype=torch.int32, device="cuda")
for _ in range(2):
    codec.compress_into(src, cb)
    codec.decompress_into(cb, out, st)
torch.cuda.synchronize()
assert torch.equal(out, src)
print("ok", float(cb["comp_len"].double().sum()))
