"""Driver for the encoder's WRITE_SIZE attribution (tools/enc_writes.sh):
the C2 encode (1 GiB, 16384 x 64 KiB) in four configurations, two launches
each, in this order:
  A  default (sidecar every 128 pairs)
  B  no sidecar (ckpt_interval 0)
  C  FSEHIP_DEBUG=4: no payload stores (header words, merge words, sidecar)
  D  FSEHIP_DEBUG=4 and no sidecar (header and merge words only)
so payload stores = A - C, sidecar = A - B, header + merge = D."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
# the environment knobs this tool sets live only in the diagnostics build
os.environ.setdefault("FSEHIP_LIB", "libfsehip_diag.so")
import torch  # noqa: E402

from entropy_coders_amd import BlockCodec  # noqa: E402

n = 1 << 30
for name, ckpt, dbg in (("A", 128, 0), ("B", 0, 0), ("C", 128, 4), ("D", 0, 4)):
    codec = BlockCodec(ckpt_interval=ckpt)
    src = codec.generate(0, 0.155, 0x5EED0002, n)
    cb = codec.alloc(n)
    os.environ["FSEHIP_DEBUG"] = str(dbg)
    for _ in range(2):
        codec.compress_into(src, cb)
    torch.cuda.synchronize()
    os.environ["FSEHIP_DEBUG"] = "0"
    comp = float(cb["comp_len"].double().sum())
    side = (float(codec.n_blocks(n)) * (codec.side_per_block - 1) * 8) if ckpt else 0.0
    print(name, "compressed", comp, "sidecar_written", side, flush=True)
    del src, cb
