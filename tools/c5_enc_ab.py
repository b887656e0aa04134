"""A/B timing of the C5 encode at table logs 12..15 (bench.py's C5 data:
near-uniform 0..239 and LUT p = 0.77, L = 15 blocks seeded so the crate's
new_first_symbol does not panic) for one library build (FSEHIP_LIB), 256 MiB
each, HIP events, median of REPS; each row's output digest (comp_len sum and
a sum over the compressed slots' bytes) must match across builds."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from entropy_coders_amd import BlockCodec  # noqa: E402

reps = int(os.environ.get("REPS", 3))
n = int(os.environ.get("NB", 256 << 20))
res = {"lib": os.environ.get("FSEHIP_LIB", "libfsehip.so")}
for name, kind, prob in (("uni", 2, 0.0), ("skew", 0, 0.77)):
    for L in (12, 13, 14, 15):
        codec = BlockCodec(ckpt_interval=64, table_log=L)
        src = codec.generate(kind, prob, 0x5EED0005, n)
        if L == 15:
            blocks = src.view(-1, 65536)
            blocks[:, -2] = 250
            blocks[:, -1] = 251
        cb = codec.alloc(n)
        codec.compress_into(src, cb)
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(reps + 1)]
        ev[0].record()
        for i in range(reps):
            codec.compress_into(src, cb)
            ev[i + 1].record()
        torch.cuda.synchronize()
        ms = sorted(ev[i].elapsed_time(ev[i + 1]) for i in range(reps))[reps // 2]
        out, st = codec.decompress(cb)
        torch.cuda.synchronize()
        cl = cb["comp_len"].to(torch.int64)
        res[f"{name}{L}_GiB_s"] = round(n / (ms * 1e-3) / 2**30, 1)
        res[f"{name}{L}_digest"] = [int(cl.sum()), int(cb["payload_bits"].to(torch.int64).sum()),
                                    int(cb["status"].to(torch.int64).abs().sum()), bool(torch.equal(out, src))]
        del codec, src, cb, out, st
        torch.cuda.empty_cache()
print(json.dumps(res))
