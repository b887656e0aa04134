"""Ablation timing of the encode/decode kernels on one GPU (diagnostics).

Variants are selected by the FSEHIP_ENC_LANES / FSEHIP_DEBUG knobs read by
libfsehip at each call; all runs happen in one process on the same data.
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
# the environment knobs this tool sets live only in the diagnostics build
os.environ.setdefault("FSEHIP_LIB", "libfsehip_diag.so")

import torch  # noqa: E402

from entropy_coders_amd import BlockCodec  # noqa: E402


def timeit(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ts = []
    for _ in range(reps):
        s.record()
        fn()
        e.record()
        torch.cuda.synchronize()
        ts.append(s.elapsed_time(e))
    ts.sort()
    return ts[len(ts) // 2]


def main():
    n = int(os.environ.get("ABL_BYTES", 1 << 30))
    kind = int(os.environ.get("ABL_KIND", 0))
    prob = float(os.environ.get("ABL_PROB", 0.155))
    tlog = int(os.environ.get("ABL_LOG", 0))
    codec = BlockCodec(table_log=tlog)
    src = codec.generate(kind, prob, 0x5EED0002, n)
    cb = codec.alloc(n)
    out = torch.empty(n, dtype=torch.uint8, device="cuda")
    st = torch.zeros(codec.n_blocks(n), dtype=torch.int32, device="cuda")
    dst = torch.empty_like(src)
    res = {}
    res["copy_1GiB"] = timeit(lambda: dst.copy_(src))
    ref = None
    for lanes in [int(x) for x in os.environ.get("ABL_LANES", "32,64").split(",")]:
        os.environ["FSEHIP_ENC_LANES"] = str(lanes)
        for dbg, name in ((8, "histogram_only"), (1, "tables_only"), (2, "no_emit"), (4, "no_payload_stores"), (0, "full")):
            os.environ["FSEHIP_DEBUG"] = str(dbg)
            res[f"enc_T{lanes}_{name}"] = timeit(lambda: codec.compress_into(src, cb))
        os.environ["FSEHIP_DEBUG"] = "0"
        codec.compress_into(src, cb)
        torch.cuda.synchronize()
        ok = int(cb["status"].abs().max()) == 0
        sig = (cb["comp_len"].clone(), cb["sidecar"].clone())
        if ref is None:
            ref = sig
        else:
            ok = ok and torch.equal(ref[0], sig[0]) and torch.equal(ref[1], sig[1])
        res[f"enc_T{lanes}_ok"] = ok
    os.environ["FSEHIP_DEBUG"] = str(1 << 4)
    res["dec_header_table_only"] = timeit(lambda: codec.decompress_into(cb, out, st))
    os.environ["FSEHIP_DEBUG"] = "0"
    res["dec_full"] = timeit(lambda: codec.decompress_into(cb, out, st))
    torch.cuda.synchronize()
    res["dec_ok"] = bool(torch.equal(out, src)) and int(st.abs().max()) == 0
    res["ratio"] = float(cb["comp_len"].double().sum()) / n
    for k, v in res.items():
        print(f"{k:28s} {v:.4f}" if isinstance(v, float) else f"{k:28s} {v}")


if __name__ == "__main__":
    main()
