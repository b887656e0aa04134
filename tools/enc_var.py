"""Encode variants by environment knobs (EV_VARS: ';'-separated lists of
NAME=VALUE[,NAME=VALUE]) on C2, skewed and uniform data: median ms per
1 GiB and whether each variant's blocks, lengths and sidecar equal the first
variant's.  Diagnostics only."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from entropy_coders_amd import BlockCodec  # noqa: E402
from tools.ablate import timeit  # noqa: E402
from tools.enc_path import sig  # noqa: E402


def main():
    n = int(os.environ.get("EV_BYTES", 1 << 30))
    variants = [v for v in os.environ.get("EV_VARS", "FSEHIP_ENC_LANES=64;FSEHIP_ENC_LANES=32").split(";") if v]
    dists = os.environ.get("EV_DISTS", "0:0.155:0,0:0.77:11,2:0:11")
    for d in dists.split(","):
        kind, prob, tlog = d.split(":")
        kind, prob, tlog = int(kind), float(prob), int(tlog)
        codec = BlockCodec(table_log=tlog)
        src = codec.generate(kind, prob, 0x5EED0002, n)
        cb = codec.alloc(n)
        ref = None
        for v in variants:
            saved = {}
            for kv in v.split(","):
                k, x = kv.split("=")
                saved[k] = os.environ.get(k)
                os.environ[k] = x
            t = timeit(lambda: codec.compress_into(src, cb), reps=7)
            torch.cuda.synchronize()
            s = sig(codec, cb)
            if ref is None:
                ref = s
            ok = all(torch.equal(a, b) for a, b in zip(ref, s)) and int(s[2].abs().max()) == 0
            print(f"kind={kind} p={prob} L={tlog or 'opt'} {v:40s} {t:.4f} ms  same={ok}", flush=True)
            for k, x in saved.items():
                if x is None:
                    os.environ.pop(k, None)
                else:
                    os.environ[k] = x
        del cb, src


if __name__ == "__main__":
    main()
