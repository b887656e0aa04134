"""A/B timing of the decode kernels (library chosen by FSEHIP_LIB): C3
(32768 x 64 KiB blocks of C2 data, prebuilt tables + sidecar, decode only)
and the C2 step (encode; decode = tables + segments), HIP events, median of
reps.  Reports whether the output is exact (ablation builds are not)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from entropy_coders_amd import BlockCodec  # noqa: E402


def timed(fn, reps):
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(reps + 1)]
    fn()
    ev[0].record()
    for i in range(reps):
        fn()
        ev[i + 1].record()
    torch.cuda.synchronize()
    return sorted(ev[i].elapsed_time(ev[i + 1]) for i in range(reps))[reps // 2]


reps = int(os.environ.get("REPS", 10))
blocks = int(os.environ.get("C3_BLOCKS", 32768))
ckpt = int(os.environ.get("CKPT", 64))
codec = BlockCodec(block_size=65536, ckpt_interval=ckpt)
n = blocks * 65536
src = codec.generate(0, float(os.environ.get("P", 0.155)), 0x5EED0003, n)  # P: the LUT skew (probes)
cb = codec.compress(src)
tabs = codec.build_dtables(cb)
out = torch.empty_like(src)
st = torch.zeros(blocks, dtype=torch.int32, device=src.device)
c3 = timed(lambda: codec.decompress_dt_into(cb, tabs, out, st), reps)
ok3 = bool(torch.equal(out, src)) and int(st.abs().max()) == 0
n2 = 1 << 30
src2 = src[:n2]
cb2 = codec.alloc(n2)
enc = timed(lambda: codec.compress_into(src2, cb2), reps)
out2 = out[:n2]
st2 = st[: n2 // 65536]
dec = timed(lambda: codec.decompress_into(cb2, out2, st2), reps)
ok2 = bool(torch.equal(out2, src2)) and int(st2.abs().max()) == 0
# encoder variants: the bytes must be the reference's, not just round-trip
from oracle import oracle as O  # noqa: E402

host2 = src2.view(-1, 65536)
bytes_ok = all(codec.block_bytes(cb2, b) == O.compress2(host2[b].cpu().numpy())[0] for b in (0, 1, 777, 16383))
ok2 = ok2 and bytes_ok
comp3 = int(cb["comp_len"].to(torch.int64).sum())
side = blocks * codec.side_per_block * 8
frac = (comp3 + side + n) / (c3 * 1e-3) / 8e12
print(json.dumps({"lib": os.environ.get("FSEHIP_LIB", "libfsehip.so"), "p": float(os.environ.get("P", 0.155)), "ckpt": ckpt, "c3_ms": round(c3, 4), "c3_frac": round(frac, 3),
                  "c3_exact": ok3, "c2_encode_ms": round(enc, 4), "c2_decode_ms": round(dec, 4), "c2_exact": ok2}))
