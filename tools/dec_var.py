"""Decode variants (FSEHIP_DEC_VAR / FSEHIP_DEC_WAVES) on C2 data, timed
both as C3 (prebuilt tables) and as the full two-kernel decode; every
variant verified.  Diagnostics only."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from entropy_coders_amd import BlockCodec  # noqa: E402
from tools.ablate import timeit  # noqa: E402


def main():
    n = int(os.environ.get("ABL_BYTES", 1 << 30))
    kind = int(os.environ.get("ABL_KIND", 0))
    prob = float(os.environ.get("ABL_PROB", 0.155))
    variants = [tuple(int(x) for x in (v + ":0").split(":")[:3]) for v in
                os.environ.get("ABL_VARS", "4:2,4:6,8:6,8:3,4:2,4:6").split(",")]
    for ckpt in [int(c) for c in os.environ.get("ABL_CKPTS", "128,64").split(",")]:
        codec = BlockCodec(ckpt_interval=ckpt)
        src = codec.generate(kind, prob, 0x5EED0002, n)
        cb = codec.compress(src)
        tabs = codec.build_dtables(cb)
        out = torch.empty(n, dtype=torch.uint8, device="cuda")
        st = torch.zeros(codec.n_blocks(n), dtype=torch.int32, device="cuda")
        for waves, var, dual in variants:
            os.environ["FSEHIP_DEC_WAVES"] = str(waves)
            os.environ["FSEHIP_DEC_VAR"] = str(var)
            os.environ["FSEHIP_DEC_DUAL"] = str(dual)
            out.zero_()
            t3 = timeit(lambda: codec.decompress_dt_into(cb, tabs, out, st), reps=7)
            torch.cuda.synchronize()
            ok3 = bool(torch.equal(out, src)) and int(st.abs().max()) == 0
            out.zero_()
            t = timeit(lambda: codec.decompress_into(cb, out, st), reps=7)
            torch.cuda.synchronize()
            ok = bool(torch.equal(out, src)) and int(st.abs().max()) == 0
            print(f"ckpt={ckpt:4d} waves={waves} var={var} dual={dual}  C3 {t3:.4f} ms ok={ok3}  full {t:.4f} ms ok={ok}",
                  flush=True)
        del cb, src, out, tabs


if __name__ == "__main__":
    main()
