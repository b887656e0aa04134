"""Phase stamps of the 4-wave decode-table kernel (dtable_par_kernel) on C2
data (FSEHIP_STAMPS=1, diagnostics build): cycles per workgroup at the
default occupancy and at one workgroup per CU (FSEHIP_DT_XLDS)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ.setdefault("FSEHIP_LIB", "libfsehip_diag.so")
import torch  # noqa: E402

from entropy_coders_amd import BlockCodec  # noqa: E402

codec = BlockCodec()
src = codec.generate(0, 0.155, 0x5EED0002, 1 << 30)
cb = codec.compress(src)
codec.build_dtables(cb)
torch.cuda.synchronize()
os.environ["FSEHIP_STAMPS"] = "1"
for x in sys.argv[1:] or ["0", "120000"]:
    os.environ["FSEHIP_DT_XLDS"] = x
    print("xlds", x, file=sys.stderr, flush=True)
    codec.build_dtables(cb)
    torch.cuda.synchronize()
