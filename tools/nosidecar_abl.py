"""Sidecar-less decode ablation: with and without the bulk output stores."""
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
for dbg in ("0", str(2 << 4), "0"):
    os.environ["FSEHIP_DEBUG"] = dbg
    codec.decompress_into(cb, out, st, use_sidecar=False)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    codec.decompress_into(cb, out, st, use_sidecar=False)
    torch.cuda.synchronize()
    print(f"debug={dbg}: {(time.perf_counter() - t0) * 1e3:.2f} ms", flush=True)
