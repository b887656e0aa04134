"""Decode-table kernel time (fsehip_build_dtables) on the C2 batch, HIP
events, median of 20 launches; FSEHIP_LIB picks a variant build."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from entropy_coders_amd import BlockCodec  # noqa: E402

codec = BlockCodec(ckpt_interval=64)
src = codec.generate(0, 0.155, 0x5EED0002, 1 << 30)
cb = codec.compress(src)
ts = []
for i in range(23):
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    codec.build_dtables(cb)
    b.record()
    torch.cuda.synchronize()
    if i >= 3:
        ts.append(a.elapsed_time(b))
ts.sort()
print(f"{os.environ.get('FSEHIP_LIB', 'libfsehip.so')}: dtables median {ts[len(ts) // 2]:.4f} ms min {ts[0]:.4f}", flush=True)
