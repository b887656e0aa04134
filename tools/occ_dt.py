"""Decode-table kernel time against resident workgroups per CU:
FSEHIP_DT_XLDS adds dynamic LDS per workgroup (diagnostics)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
# the environment knobs this tool sets live only in the diagnostics build
os.environ.setdefault("FSEHIP_LIB", "libfsehip_diag.so")

from entropy_coders_amd import BlockCodec  # noqa: E402
from tools.ablate import timeit  # noqa: E402

LDS_CU, BASE = 160 * 1024, int(os.environ.get("OCC_BASE_LDS", 7680))
n = 1 << 30
codec = BlockCodec()
src = codec.generate(0, 0.155, 0x5EED0002, n)
cb = codec.compress(src)
for wg in [int(w) for w in os.environ.get("OCC_WGS", "20,16,20,12,10,8,20").split(",")]:
    x = max(0, LDS_CU // wg - BASE - 64) if wg < LDS_CU // BASE else 0
    os.environ["FSEHIP_DT_XLDS"] = str(x)
    t = timeit(lambda: codec.build_dtables(cb), reps=7)
    print(f"wg/cu<={wg} xlds={x}  {t:.4f} ms", flush=True)
