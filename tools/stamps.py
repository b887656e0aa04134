"""Per-phase cycle stamps of the encode/decode kernels (FSEHIP_STAMPS=1)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
# the environment knobs this tool sets live only in the diagnostics build
os.environ.setdefault("FSEHIP_LIB", "libfsehip_diag.so")
os.environ["FSEHIP_STAMPS"] = "1"

import torch  # noqa: E402

from entropy_coders_amd import BlockCodec  # noqa: E402

n = int(os.environ.get("ST_BYTES", 1 << 30))
for kind, prob, log2 in [(0, 0.155, 0), (2, 0.0, 11), (0, 0.77, 11)]:
    codec = BlockCodec(table_log=log2)
    src = codec.generate(kind, prob, 0x5EED0002, n)
    print(f"== kind={kind} p={prob} L={log2 or 'opt'}", file=sys.stderr, flush=True)
    for _ in range(2):
        cb = codec.compress(src)
        out, st = codec.decompress(cb)
    torch.cuda.synchronize()
    assert torch.equal(out, src)
