"""Encode time against resident workgroups per CU: FSEHIP_ENC_XLDS adds
dynamic LDS to each encode workgroup, lowering occupancy step by step
(diagnostics: is the encoder latency-bound or throughput-bound?)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
# the environment knobs this tool sets live only in the diagnostics build
os.environ.setdefault("FSEHIP_LIB", "libfsehip_diag.so")

import torch  # noqa: E402

from entropy_coders_amd import BlockCodec  # noqa: E402
from tools.ablate import timeit  # noqa: E402

LDS_CU = 160 * 1024


def main():
    n = int(os.environ.get("ABL_BYTES", 1 << 30))
    base = int(os.environ.get("OCC_BASE_LDS", 17472))
    for kind, prob, tlog in [(0, 0.155, 0), (2, 0.0, 11)]:
        codec = BlockCodec(table_log=tlog)
        src = codec.generate(kind, prob, 0x5EED0002, n)
        cb = codec.alloc(n)
        for wg in tuple(int(x) for x in os.environ.get("OCC_WGS", "9,8,7,6,5,4").split(",")):
            x = max(0, LDS_CU // wg - base - 64) if wg < LDS_CU // base else 0
            os.environ["FSEHIP_ENC_XLDS"] = str(x)
            t = timeit(lambda: codec.compress_into(src, cb), reps=5)
            print(f"kind={kind} p={prob} wg/cu<={wg} xlds={x}  {t:.4f} ms", flush=True)
        os.environ["FSEHIP_ENC_XLDS"] = "0"
        del cb, src


if __name__ == "__main__":
    main()
