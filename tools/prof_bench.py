"""Driver for the rocprofv3 PMC passes behind bench.py's roofline objects:
the bench's kernels on the bench's data, each launch twice (the summary takes
the last launch of each kind; the first may see a cold cache).

  C2: 16384 x 64 KiB (LUT p=0.155): encode, decode tables, decode
  C2 again without the sidecar: the serial (sidecar-less) decode
  C3: 32768 x 64 KiB of the same distribution: decode with prebuilt tables

The summariser (tools/pmc_summary.py) tells the launches apart by kernel
name and grid size."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from entropy_coders_amd import BlockCodec  # noqa: E402

# the bench's checkpoint interval (bench.py --ckpt default)
codec = BlockCodec(nstates=int(os.environ.get("PROF_NSTATES", 2)), ckpt_interval=int(os.environ.get("PROF_CKPT", 64)))
n = 1 << 30
src = codec.generate(0, 0.155, 0x5EED0002, n)
cb = codec.alloc(n)
out = torch.empty(n, dtype=torch.uint8, device="cuda")
st = torch.zeros(codec.n_blocks(n), dtype=torch.int32, device="cuda")
for _ in range(2):
    codec.compress_into(src, cb)
    codec.decompress_into(cb, out, st)
torch.cuda.synchronize()
assert torch.equal(out, src)
if not int(os.environ.get("PROF_NO_SERIAL", 0)):  # sidecar-less decode (serial_ring_kernel)
    for _ in range(2):
        out.fill_(0)
        codec.decompress_into(cb, out, st, use_sidecar=False)
    torch.cuda.synchronize()
    assert torch.equal(out, src)
del out
if not int(os.environ.get("PROF_NO_C3", 0)):
    n3 = 32768 * 65536
    src3 = codec.generate(0, 0.155, 0x5EED0003, n3)
    cb3 = codec.alloc(n3)
    codec.compress_into(src3, cb3)
    tabs = codec.build_dtables(cb3)
    out3 = torch.empty(n3, dtype=torch.uint8, device="cuda")
    st3 = torch.zeros(codec.n_blocks(n3), dtype=torch.int32, device="cuda")
    for _ in range(2):
        codec.decompress_dt_into(cb3, tabs, out3, st3)
    torch.cuda.synchronize()
    assert torch.equal(out3, src3)
print("ok", float(cb["comp_len"].double().sum()))
