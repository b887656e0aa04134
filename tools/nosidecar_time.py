"""Time the sidecar-less decode against the sidecar decode on
a reduced size, for a few distributions and table logs; every result is
checked against the source.  FSEHIP_SERIAL_OLD=1 selects the previous
register-window serial kernel for A/B runs."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
# the environment knobs this tool sets live only in the diagnostics build
os.environ.setdefault("FSEHIP_LIB", "libfsehip_diag.so")
import torch  # noqa: E402

from entropy_coders_amd import BlockCodec  # noqa: E402

n = int(os.environ.get("NS_BYTES", 256 << 20))
# (name, generator kind, prob, table_log): C2, uniform C5 L=11, skewed L=12
cases = [("c2_lut0155", 0, 0.155, 0), ("uniform_L11", 1, 0.0, 11), ("lut077_L12", 0, 0.77, 12)]
only = os.environ.get("NS_CASES")
for name, kind, prob, tl in cases:
    if only and name not in only.split(","):
        continue
    ns = int(os.environ.get("NS_STATES", 2))
    codec = BlockCodec(ckpt_interval=128, table_log=tl, nstates=ns)
    src = codec.generate(kind, prob, 0x5EED0002, n)
    cb = codec.compress(src)
    out = torch.empty(n, dtype=torch.uint8, device="cuda")
    st = torch.zeros(codec.n_blocks(n), dtype=torch.int32, device="cuda")
    res = {}
    for use in (True, False):
        codec.decompress_into(cb, out, st, use_sidecar=use)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        codec.decompress_into(cb, out, st, use_sidecar=use)
        torch.cuda.synchronize()
        t = time.perf_counter() - t0
        ok = bool(torch.equal(out, src)) and int(st.abs().max()) == 0
        res[use] = (t, ok)
        out.fill_(0)
    # the same blocks as crate streams with no raw length (fsehip_decompress_streams)
    import ctypes as C
    nb = codec.n_blocks(n)
    ol = torch.zeros(nb, dtype=torch.int32, device="cuda")
    lib, hs = codec.lib, C.c_void_p(torch.cuda.current_stream().cuda_stream)
    args = (ns, codec.max_table_log, C.c_void_p(cb["out"].data_ptr()), codec.slot_bytes,
            C.c_void_p(cb["comp_len"].data_ptr()), nb, C.c_void_p(out.data_ptr()), codec.block_size,
            C.c_void_p(ol.data_ptr()), C.c_void_p(st.data_ptr()), hs)
    lib.fsehip_decompress_streams(*args)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    rc = lib.fsehip_decompress_streams(*args)
    torch.cuda.synchronize()
    t_str = time.perf_counter() - t0
    str_ok = rc == 0 and bool(torch.equal(out, src)) and int(st.abs().max()) == 0
    res["streams"] = (t_str, str_ok)
    o2, side2, st2 = codec.build_sidecar(cb)
    torch.cuda.synchronize()
    side_ok = bool(torch.equal(o2, src)) and int(st2.abs().max()) == 0 and bool(torch.equal(side2, cb["sidecar"]))
    ratio = int(cb["comp_len"].sum()) / n
    print(f"{name} ({ns}-state): ratio {ratio:.3f}  sidecar {res[True][0] * 1e3:.2f} ms ({n / res[True][0] / 2**30:.0f} GiB/s, "
          f"ok={res[True][1]})  no sidecar {res[False][0] * 1e3:.2f} ms ({n / res[False][0] / 2**30:.1f} GiB/s, "
          f"ok={res[False][1]})  streams {n / res['streams'][0] / 2**30:.1f} GiB/s ok={res['streams'][1]}  "
          f"build_sidecar ok={side_ok}", flush=True)
