"""Encoder phase ablations x occupancy (diagnostics build): the time of each
cumulative ablation (FSEHIP_DEBUG: 8 = histogram only, 1 = + normalise,
header and tables, 18 = + the count pass without repair rounds, 2 = + the
repair rounds (no emit), 4 = + the emit pass without payload stores, 0 = the
whole kernel) at several resident workgroups per CU (FSEHIP_ENC_XLDS pads
the dynamic LDS).  A phase whose time difference grows as workgroups fall is
latency-bound; one whose difference stays flat is throughput-bound."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ.setdefault("FSEHIP_LIB", "libfsehip_diag.so")

import torch  # noqa: E402

from entropy_coders_amd import BlockCodec  # noqa: E402
from tools.ablate import timeit  # noqa: E402

LDS_CU = 160 * 1024
BASE = int(os.environ.get("OCC_BASE_LDS", 14656))


def main():
    n = int(os.environ.get("ABL_BYTES", 1 << 30))
    kind, prob, tlog = int(os.environ.get("ABL_KIND", 0)), float(os.environ.get("ABL_PROB", 0.155)), int(
        os.environ.get("ABL_LOG", 0))
    codec = BlockCodec(table_log=tlog)
    src = codec.generate(kind, prob, 0x5EED0002, n)
    cb = codec.alloc(n)
    wgs = [int(x) for x in os.environ.get("OCC_WGS", "11,8,6,4").split(",")]
    abl = [(8, "hist"), (1, "tables"), (18, "count"), (2, "repair"), (4, "emit"), (0, "stores")]
    print(f"kind={kind} p={prob} L={tlog or 'opt'}: ms per ablation (cumulative) and phase deltas", flush=True)
    for wg in wgs:
        x = max(0, LDS_CU // wg - BASE - 64) if wg < 11 else 0
        os.environ["FSEHIP_ENC_XLDS"] = str(x)
        prev, row = 0.0, []
        for dbg, name in abl:
            os.environ["FSEHIP_DEBUG"] = str(dbg)
            t = timeit(lambda: codec.compress_into(src, cb), reps=5)
            row.append(f"{name} {t:.3f} (+{t - prev:.3f})")
            prev = t
        print(f"wg/cu={wg:2d} xlds={x:6d}  " + "  ".join(row), flush=True)
    os.environ["FSEHIP_ENC_XLDS"] = "0"
    os.environ["FSEHIP_DEBUG"] = "0"


if __name__ == "__main__":
    main()
