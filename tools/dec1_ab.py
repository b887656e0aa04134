"""A/B timing of the 1-state segment decode (fse_compress blocks with a
sidecar, decode_pre_kernel<..., NS = 1>) and, for reference, the 2-state
one, for one library build (FSEHIP_LIB): the bench's C2 data at 1 GiB, HIP
events, median of REPS, output checked against the source."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from entropy_coders_amd import BlockCodec  # noqa: E402

reps = int(os.environ.get("REPS", 7))
n = int(os.environ.get("NB", 1 << 30))
res = {"lib": os.environ.get("FSEHIP_LIB", "libfsehip.so")}
for ns, ck, kind, prob in ((1, 128, 0, 0.155), (2, 64, 0, 0.155), (1, 128, 2, 0.0)):
    codec = BlockCodec(ckpt_interval=ck, nstates=ns)
    src = codec.generate(kind, prob, 0x5EED0002, n)
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
    key = f"ns{ns}_{'c2' if kind == 0 else 'uni'}"
    res[key + "_ms"] = round(ms, 4)
    res[key + "_exact"] = bool(torch.equal(out, src)) and int(st.abs().max()) == 0
    del codec, src, cb, out, st
    torch.cuda.empty_cache()
print(json.dumps(res))
