"""Timing probe for the "emit once from the guessed starts" encoder (verdict
r04 item 1; diagnostics): with FSEHIP_LIB=libfsehip_eprobe.so (built with
-DFSEHIP_ENC_ABL=2) the count and repair passes also do the emit pass's bit
packing and ring writes, and the final emit pass is skipped -- the kernel
then costs what an encoder that emits from the guessed starts and repairs
by re-emitting would cost before its placement pass.  Prints the C2 1 GiB
encode time (HIP events, median of 5) for FSEHIP_DEBUG 0 (whole kernel),
2 (no final emit) and 16 (no repair rounds) at the workgroups per CU set by
FSEHIP_ENC_XLDS."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ.setdefault("FSEHIP_LIB", "libfsehip_diag.so")
import torch  # noqa: E402

from entropy_coders_amd import BlockCodec  # noqa: E402
from tools.ablate import timeit  # noqa: E402

codec = BlockCodec()
n = 1 << 30
src = codec.generate(0, 0.155, 0x5EED0002, n)
cb = codec.alloc(n)
res = {}
for dbg in (0, 2, 16):
    os.environ["FSEHIP_DEBUG"] = str(dbg)
    res[dbg] = timeit(lambda: codec.compress_into(src, cb))
print(f"{os.environ['FSEHIP_LIB']} xlds={os.environ.get('FSEHIP_ENC_XLDS', '0')}: "
      f"full {res[0]:.4f} ms, no final emit {res[2]:.4f}, no repair {res[16]:.4f}", flush=True)
