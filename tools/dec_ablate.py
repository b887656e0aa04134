"""Decode variants on C2 data (diagnostics): checkpoint interval x waves per
block, plus the header+table-only ablation.  Each variant is verified."""
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
    for ckpt in (int(os.environ.get("ABL_CKPT", 64)),):
        codec = BlockCodec(ckpt_interval=ckpt)
        src = codec.generate(kind, prob, 0x5EED0002, n)
        cb = codec.compress(src)
        out = torch.empty(n, dtype=torch.uint8, device="cuda")
        st = torch.zeros(codec.n_blocks(n), dtype=torch.int32, device="cuda")
        for waves, var, dual in ((4, 2, 0), (4, 3, 0), (4, 5, 0), (4, 3, 1), (4, 5, 1), (8, 2, 0), (8, 3, 0), (8, 5, 0)):
            os.environ["FSEHIP_DEC_WAVES"] = str(waves)
            os.environ["FSEHIP_DEC_VAR"] = str(var)
            os.environ["FSEHIP_DEC_DUAL"] = str(dual)
            os.environ["FSEHIP_DEBUG"] = str(1 << 4)
            t_ht = timeit(lambda: codec.decompress_into(cb, out, st))
            os.environ["FSEHIP_DEBUG"] = "0"
            out.zero_()
            t = timeit(lambda: codec.decompress_into(cb, out, st))
            torch.cuda.synchronize()
            ok = bool(torch.equal(out, src)) and int(st.abs().max()) == 0
            print(f"ckpt={ckpt:4d} waves={waves} var={var} dual={dual}  header+table {t_ht:.4f} ms  full {t:.4f} ms  ok={ok}", flush=True)
        del cb, src, out


if __name__ == "__main__":
    main()
