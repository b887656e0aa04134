"""Encode path comparison (FSEHIP_ENC_PATH 1 = repair, 2 = scratch; FSEHIP_ENC_WARM
warm-up pairs) on C2, skewed and uniform data: median ms per 1 GiB and
whether every variant's blocks, lengths and sidecar equal the repair path's.
Diagnostics only."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from entropy_coders_amd import BlockCodec  # noqa: E402
from entropy_coders_amd.dist import pack_device  # noqa: E402
from tools.ablate import timeit  # noqa: E402


def sig(codec, cb):
    packed, _ = pack_device(cb["out"], codec.slot_bytes, cb["comp_len"])
    return (cb["comp_len"].clone(), cb["sidecar"].clone(), cb["status"].clone(), packed)


def main():
    n = int(os.environ.get("EP_BYTES", 1 << 30))
    variants = os.environ.get("EP_VARS", "1:0,2:0,2:32,2:64,2:128").split(",")
    for kind, prob, tlog in [(0, 0.155, 0), (0, 0.77, 11), (2, 0.0, 11)]:
        codec = BlockCodec(table_log=tlog)
        src = codec.generate(kind, prob, 0x5EED0002, n)
        cb = codec.alloc(n)
        ref = None
        for v in variants:
            path, warm = v.split(":")
            os.environ["FSEHIP_ENC_PATH"] = path
            os.environ["FSEHIP_ENC_WARM"] = warm
            os.environ["FSEHIP_ENC_PMAX"] = "256"
            t = timeit(lambda: codec.compress_into(src, cb), reps=7)
            torch.cuda.synchronize()
            s = sig(codec, cb)
            if ref is None:
                ref = s
            ok = all(torch.equal(a, b) for a, b in zip(ref, s)) and int(s[2].abs().max()) == 0
            print(f"kind={kind} p={prob} path={path} warm={warm:>4s}  {t:.4f} ms  same={ok}", flush=True)
        del cb, src


if __name__ == "__main__":
    main()
