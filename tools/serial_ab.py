"""A/B timing of the sidecar-less decode (serial_ring_kernel + sym_map_kernel,
SURVEY 8(f3)) of one library build (FSEHIP_LIB): the bench's C2 1 GiB in both
formats, HIP events, median of REPS, every result checked against the source.
Run over several builds with tools/gpu_run.sh abpy:serial_ab:V1,V2,..."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from entropy_coders_amd import BlockCodec  # noqa: E402

reps = int(os.environ.get("REPS", 5))
n = int(os.environ.get("NS_BYTES", 1 << 30))
res = {"lib": os.environ.get("FSEHIP_LIB", "libfsehip.so")}
for ns in (2, 1):
    codec = BlockCodec(ckpt_interval=64 * ns, nstates=ns)
    src = codec.generate(0, 0.155, 0x5EED0002, n)
    cb = codec.compress(src)
    out = torch.empty_like(src)
    st = torch.zeros(codec.n_blocks(n), dtype=torch.int32, device=src.device)
    codec.decompress_into(cb, out, st, use_sidecar=False)  # warm-up
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(reps + 1)]
    out.fill_(0)
    ev[0].record()
    for i in range(reps):
        codec.decompress_into(cb, out, st, use_sidecar=False)
        ev[i + 1].record()
    torch.cuda.synchronize()
    ms = sorted(ev[i].elapsed_time(ev[i + 1]) for i in range(reps))[reps // 2]
    ok = bool(torch.equal(out, src)) and int(st.abs().max()) == 0
    res[f"ns{ns}_ms"] = round(ms, 4)
    res[f"ns{ns}_GiB_s"] = round(n / (ms * 1e-3) / 2**30, 2)
    res[f"ns{ns}_exact"] = ok
    del codec, src, cb, out, st
    torch.cuda.empty_cache()
# EXTRA=1: the kernels that write symbols themselves -- skewed data at L = 12
# (serial_ring_kernel<12, 3, 2>) and the sidecar rebuild of C2 (recording)
if os.environ.get("EXTRA"):
    def med(fn):
        fn()
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(reps + 1)]
        ev[0].record()
        for i in range(reps):
            fn()
            ev[i + 1].record()
        torch.cuda.synchronize()
        return sorted(ev[i].elapsed_time(ev[i + 1]) for i in range(reps))[reps // 2]

    codec = BlockCodec(ckpt_interval=64, table_log=12)
    src = codec.generate(0, 0.77, 0x5EED0002, n)
    cb = codec.compress(src)
    out = torch.empty_like(src)
    st = torch.zeros(codec.n_blocks(n), dtype=torch.int32, device=src.device)
    res["l12_skew_ms"] = round(med(lambda: codec.decompress_into(cb, out, st, use_sidecar=False)), 4)
    res["l12_skew_exact"] = bool(torch.equal(out, src)) and int(st.abs().max()) == 0
    codec = BlockCodec(ckpt_interval=64)
    src = codec.generate(0, 0.155, 0x5EED0002, n)
    cb = codec.compress(src)
    res["rebuild_ms"] = round(med(lambda: codec.build_sidecar(cb)), 4)
    o2, side, st2 = codec.build_sidecar(cb)
    torch.cuda.synchronize()
    k = codec.n_blocks(n) * codec.side_per_block
    res["rebuild_exact"] = (bool(torch.equal(o2[:n], src)) and int(st2.abs().max()) == 0
                            and bool(torch.equal(side[:k], cb["sidecar"][:k])))
print(json.dumps(res))
