"""Decode-table kernel phase stamps (FSEHIP_STAMPS=1) on C2 data: header
parse, spread phases and rank passes, cycles per workgroup (stderr), at the
default occupancy and (FSEHIP_DT_XLDS) at one workgroup per CU."""
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
codec.build_dtables(cb)
torch.cuda.synchronize()
os.environ["FSEHIP_STAMPS"] = "1"
for x in ("0", "156096"):
    os.environ["FSEHIP_DT_XLDS"] = x
    print("xlds", x, file=sys.stderr, flush=True)
    codec.build_dtables(cb)
    torch.cuda.synchronize()
