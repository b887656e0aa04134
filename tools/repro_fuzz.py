"""Rebuild one case of tests/test_gpu_fuzz.py (FSEHIP_FUZZ_SEED + case) and
report where each decode route differs from the source (diagnostics)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

from entropy_coders_amd import BlockCodec  # noqa: E402
from tests.test_gpu_fuzz import draw_case  # noqa: E402

seed, case = int(sys.argv[1]), int(sys.argv[2])
draw = int(sys.argv[3]) if len(sys.argv) > 3 else 2
nstates, block, table_log, ckpt, sizes, blocks = draw_case(seed, case, draw)
host = np.concatenate(blocks)
print("case", nstates, block, len(sizes), sizes[-1], table_log, ckpt, flush=True)
codec = BlockCodec(block_size=block, table_log=table_log, ckpt_interval=ckpt, nstates=nstates)
src = torch.from_numpy(host).cuda()
cb = codec.compress(src)
torch.cuda.synchronize()
for name, use in (("serial", False), ("sidecar", True)):
    out, st = codec.decompress(cb, use_sidecar=use)
    torch.cuda.synchronize()
    o = out.cpu().numpy()
    for b, s in enumerate(blocks):
        lo = b * block
        got = o[lo: lo + len(s)]
        if not np.array_equal(got, s):
            bad = np.nonzero(got != s)[0]
            bb = codec.block_bytes(cb, b)
            print(name, "block", b, "status", int(st[b]), "n", len(s), "comp_len", len(bb), "first bad", int(bad[0]),
                  "count", len(bad), "last bad", int(bad[-1]), "L", table_log, flush=True)
            print("  got ", got[max(0, bad[0] - 4): bad[0] + 8].tolist())
            print("  want", s[max(0, bad[0] - 4): bad[0] + 8].tolist())

# checkpoints every 8 pairs: the encoder's sidecar against the one the serial
# decoder records (fsehip_build_sidecar), block by block
if nstates == 2:
    c8 = BlockCodec(block_size=block, table_log=table_log, ckpt_interval=8, nstates=nstates)
    cb8 = c8.compress(src)
    out8, side8, st8 = c8.build_sidecar(cb8)
    torch.cuda.synchronize()
    spb = c8.side_per_block
    enc = cb8["sidecar"].cpu().numpy().astype(np.uint64)
    dec = side8.cpu().numpy().astype(np.uint64)
    for b in range(len(blocks)):
        if int(cb8["status"][b]) != 0:
            continue
        e, d = enc[b * spb:(b + 1) * spb], dec[b * spb:(b + 1) * spb]
        diff = np.nonzero(e != d)[0]
        print("ckpt8 block", b, "status", int(st8[b]), "entries", spb, "differ at", diff[:6].tolist())
        for i in diff[:3]:
            f = lambda v: (int(v) & 0xFFFFFFFF, (int(v) >> 32) & 0xFFFF, int(v) >> 48)
            print("   entry", int(i), "enc", f(e[i]), "dec", f(d[i]))

# the last bytes of every valid block on each route, against the oracle's own decode
from oracle import oracle as O  # noqa: E402
for b, s in enumerate(blocks):
    if int(cb["status"][b]) != 0:
        continue
    comp = codec.block_bytes(cb, b)
    ref = np.frombuffer(O.decompress2(comp, raw_len=len(s)) if nstates == 2 else O.decompress(comp), dtype=np.uint8)
    lo = b * block
    for name, use in (("serial", False), ("sidecar", True)):
        out, st = codec.decompress(cb, use_sidecar=use)
        torch.cuda.synchronize()
        got = out[lo: lo + len(s)].cpu().numpy()
        print("block", b, name, "last", got[-3:].tolist(), "oracle decode", ref[-3:].tolist(), "source", s[-3:].tolist(),
              "== oracle:", bool(np.array_equal(got, ref)))
