"""Time the sidecar-less decode of C2 blocks (serial reference mode, one
lane per block) on a reduced size.  Diagnostics for SURVEY 8(f3)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from entropy_coders_amd import BlockCodec  # noqa: E402

n = int(os.environ.get("NS_BYTES", 256 << 20))
codec = BlockCodec(ckpt_interval=128)
src = codec.generate(0, 0.155, 0x5EED0002, n)
cb = codec.compress(src)
out = torch.empty(n, dtype=torch.uint8, device="cuda")
st = torch.zeros(codec.n_blocks(n), dtype=torch.int32, device="cuda")
for use in (True, False):
    codec.decompress_into(cb, out, st, use_sidecar=use)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    codec.decompress_into(cb, out, st, use_sidecar=use)
    torch.cuda.synchronize()
    t = time.perf_counter() - t0
    ok = bool(torch.equal(out, src)) and int(st.abs().max()) == 0
    print(f"sidecar={use}: {t * 1e3:.2f} ms for {n >> 20} MiB ({n / t / 2**30:.1f} GiB/s) ok={ok}", flush=True)
