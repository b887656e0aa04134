"""Occupancy probe (resident workgroups per CU, from the HIP runtime) and
the prebuilt-table decode timed at each LDS image size (FSEHIP_DEC_PP)."""
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from entropy_coders_amd import BlockCodec, load  # noqa: E402
from tools.ablate import timeit  # noqa: E402


def main():
    lib = load()
    buf = C.create_string_buffer(4096)
    lib.fsehipx_occupancy.argtypes = [C.c_char_p, C.c_int]
    lib.fsehipx_occupancy(buf, 4096)
    print(buf.value.decode(), flush=True)
    n = int(os.environ.get("ABL_BYTES", 1 << 30))
    codec = BlockCodec(ckpt_interval=int(os.environ.get("ABL_CKPT", 128)))
    src = codec.generate(0, 0.155, 0x5EED0002, n)
    cb = codec.compress(src)
    tabs = codec.build_dtables(cb)
    out = torch.empty(n, dtype=torch.uint8, device="cuda")
    st = torch.zeros(codec.n_blocks(n), dtype=torch.int32, device="cuda")
    clen = cb["comp_len"].to(torch.int64)
    print(f"comp_len max {int(clen.max())} mean {float(clen.double().mean()):.0f}", flush=True)
    for pp in (44, 40, 36, 44):
        os.environ["FSEHIP_DEC_PP"] = str(pp)
        out.zero_()
        t = timeit(lambda: codec.decompress_dt_into(cb, tabs, out, st))
        torch.cuda.synchronize()
        ok = bool(torch.equal(out, src)) and int(st.abs().max()) == 0
        print(f"PP={pp} KiB  decode(prebuilt) {t:.4f} ms  ok={ok}", flush=True)


if __name__ == "__main__":
    main()
