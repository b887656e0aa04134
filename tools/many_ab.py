"""A/B timing of fse_decompress2_many / fse_decompress_many (host buffers,
PCIe included) at several stream counts for one library build (FSEHIP_LIB):
C2 64 KiB blocks encoded on the GPU and taken as crate-format streams,
median of REPS calls, every stream's bytes checked against its source."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

from entropy_coders_amd import BlockCodec, decompress2_many  # noqa: E402

reps = int(os.environ.get("REPS", 7))
counts = [int(x) for x in os.environ.get("COUNTS", "3,16,64,128,256,1000").split(",")]
res = {"lib": os.environ.get("FSEHIP_LIB", "libfsehip.so")}
for ns in (2, 1):
    codec = BlockCodec(ckpt_interval=0, nstates=ns)
    nmax = max(counts)
    src = codec.generate(0, 0.155, 0x5EED0007, nmax * 65536)
    cb = codec.compress(src)
    torch.cuda.synchronize()
    host = src.cpu().numpy()
    streams = [codec.block_bytes(cb, b) for b in range(nmax)]
    for m in counts:
        dst = np.empty(m * 65536, dtype=np.uint8)
        decompress2_many(streams[:m], 65536, nstates=ns, raw=True, dst=dst)
        ts = []
        for _ in range(reps):
            t0 = time.perf_counter()
            out, lens, st = decompress2_many(streams[:m], 65536, nstates=ns, raw=True, dst=dst)
            ts.append(time.perf_counter() - t0)
        ok = bool((st == 0).all()) and bool(np.array_equal(out[: m * 65536], host[: m * 65536]))
        res[f"ns{ns}_m{m}_ms"] = round(sorted(ts)[reps // 2] * 1e3, 3)
        res[f"ns{ns}_m{m}_ok"] = ok
print(json.dumps(res))
