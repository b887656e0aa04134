"""Encode A/B timing across library builds (diagnostics): the library named
by FSEHIP_LIB encodes 1 GiB of C2 data (and, with AB_WIDE=1, geometric and
skewed L = 11 / 12 data) and prints the median of 7 HIP-event timings per
input, plus a byte check of the compressed C2 blocks against a reference
digest file when AB_DIGEST names one (written by the first library run)."""
import hashlib
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ.setdefault("FSEHIP_LIB", "libfsehip.so")
import torch  # noqa: E402

from entropy_coders_amd import BlockCodec  # noqa: E402
from tools.ablate import timeit  # noqa: E402

n = 1 << 30
cases = [("C2", 0, 0.155, 0)]
if os.environ.get("AB_WIDE") == "1":
    cases += [("geometric", 1, 0.5, 0), ("skewed L11", 0, 0.77, 11), ("skewed L12", 0, 0.77, 12)]
if os.environ.get("AB_WIDE") == "2":  # the histogram's cases: skewed (C5) and near-uniform data at L = 9
    cases += [("skewed L9", 0, 0.77, 9), ("skewed L10", 0, 0.77, 10), ("uniform L9", 2, 0.0, 9)]
out = []
for name, kind, prob, tlog in cases:
    codec = BlockCodec(table_log=tlog)
    src = codec.generate(kind, prob, 0x5EED0002, n)
    cb = codec.alloc(n)
    ms = timeit(lambda: codec.compress_into(src, cb), reps=7)
    out.append(f"{name} {ms:.4f} ms")
    if name == "C2" and os.environ.get("AB_DIGEST"):
        torch.cuda.synchronize()
        h = hashlib.sha256()
        nb = cb["comp_len"].numel()
        blocks = cb["out"].view(nb, -1)
        keep = torch.arange(blocks.shape[1], device=blocks.device)[None, :] < cb["comp_len"][:, None]
        h.update(blocks[keep].cpu().numpy().tobytes())  # each block's compressed bytes, in order
        for key in ("comp_len", "payload_bits", "sidecar", "status"):
            h.update(cb[key].cpu().numpy().tobytes())
        d = h.hexdigest()
        del keep
        path = os.environ["AB_DIGEST"]
        if os.path.exists(path):
            ref = open(path).read().strip()
            out.append("bytes " + ("same" if ref == d else "DIFFER"))
            if ref != d:
                print(os.environ["FSEHIP_LIB"], ": ".join(out), flush=True)
                sys.exit(1)
        else:
            open(path, "w").write(d)
    del src, cb
    torch.cuda.empty_cache()
print(os.environ["FSEHIP_LIB"] + ": " + ", ".join(out), flush=True)
