"""A/B timing of the C5 decode (sidecar segments) at table logs 12..15 on
bench.py's C5 data (near-uniform 0..239 and LUT p = 0.77; L = 15 blocks
seeded as bench.py does) for one library build (FSEHIP_LIB): 256 MiB each,
HIP events, median of REPS, output checked against the source."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from entropy_coders_amd import BlockCodec  # noqa: E402

reps = int(os.environ.get("REPS", 5))
n = int(os.environ.get("NB", 256 << 20))
res = {"lib": os.environ.get("FSEHIP_LIB", "libfsehip.so")}
for name, kind, prob in (("uni", 2, 0.0), ("skew", 0, 0.77)):
    for L in (12, 13, 14, 15):
        if os.environ.get("ROWS") and f"{name}{L}" not in os.environ["ROWS"].split(","):
            continue
        codec = BlockCodec(ckpt_interval=64, table_log=L)
        src = codec.generate(kind, prob, 0x5EED0005, n)
        if L == 15:
            blocks = src.view(-1, 65536)
            blocks[:, -2] = 250
            blocks[:, -1] = 251
        cb = codec.compress(src)
        out = torch.empty_like(src)
        st = torch.zeros(codec.n_blocks(n), dtype=torch.int32, device=src.device)
        codec.decompress_into(cb, out, st)
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(reps + 1)]
        out.fill_(0)
        ev[0].record()
        for i in range(reps):
            codec.decompress_into(cb, out, st)
            ev[i + 1].record()
        torch.cuda.synchronize()
        ms = sorted(ev[i].elapsed_time(ev[i + 1]) for i in range(reps))[reps // 2]
        res[f"{name}{L}_GiB_s"] = round(n / (ms * 1e-3) / 2**30, 1)
        res[f"{name}{L}_exact"] = bool(torch.equal(out, src)) and int(st.abs().max()) == 0
        del codec, src, cb, out, st
        torch.cuda.empty_cache()
print(json.dumps(res))
