"""Decode phase stamps (FSEHIP_STAMPS=1) on C2 data: staging vs decode
cycles per workgroup, for the current decode settings (environment)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
# the environment knobs this tool sets live only in the diagnostics build
os.environ.setdefault("FSEHIP_LIB", "libfsehip_diag.so")

import torch  # noqa: E402

from entropy_coders_amd import BlockCodec  # noqa: E402

codec = BlockCodec()
src = codec.generate(0, 0.155, 0x5EED0002, 1 << 30)
cb = codec.compress(src)
tabs = codec.build_dtables(cb)
out = torch.empty_like(src)
st = torch.zeros(codec.n_blocks(1 << 30), dtype=torch.int32, device=src.device)
codec.decompress_dt_into(cb, tabs, out, st)
torch.cuda.synchronize()
os.environ["FSEHIP_STAMPS"] = "1"
codec.decompress_dt_into(cb, tabs, out, st)
torch.cuda.synchronize()
assert torch.equal(out, src)
