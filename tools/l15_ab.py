"""A/B timing of the segment decode at table logs 14 and 15 (the L = 15 path
reads its payload through the global-memory window beside a 128 KiB table)
for one library build (FSEHIP_LIB): 256 MiB near-uniform and skewed data
with 64-pair checkpoints, HIP events, median of REPS, an output digest per case."""
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
for name, kind, prob, tl in (("u14", 2, 0.0, 14), ("u15", 2, 0.0, 15), ("s15", 0, 0.77, 15)):
    codec = BlockCodec(ckpt_interval=64, table_log=tl)
    src = codec.generate(kind, prob, 0x5EED0015, n)
    # bench.py's C5 rows: two seed symbols outside the alphabet end every
    # block, so the crate's new_first_symbol does not panic at L = 15
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
    res[name + "_GiB_s"] = round(n / (ms * 1e-3) / 2**30, 1)
    # L = 15 round trips can differ from the source where the crate's own
    # decode does (new_first_symbol): compare builds by a digest instead
    res[name + "_digest"] = [int(out.view(torch.int64).sum()), int(st.to(torch.int64).abs().sum())]
    del codec, src, cb, out, st
    torch.cuda.empty_cache()
print(json.dumps(res))
