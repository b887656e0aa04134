"""Two batches in flight: step k + 1's encode (stream A) beside step k's
decode (stream B), against the bench's one-stream step, on the bench's C2
workload (1 GiB, 64 KiB blocks, 64-pair checkpoints).  A measurement of how
much the kernels' ramps and tails leave on the table, not the bench metric.

    python tools/pipe_probe.py [STEPS]
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from entropy_coders_amd.fse import BlockCodec  # noqa: E402

K = int(sys.argv[1]) if len(sys.argv) > 1 else 20
dev = torch.device("cuda:0")
n = 1 << 30
codec = BlockCodec(block_size=65536, ckpt_interval=64)
src = codec.generate(0, 0.155, 0x5EED0002, n)
cbs = [codec.alloc(n), codec.alloc(n)]
outs = [torch.empty(n, dtype=torch.uint8, device=dev) for _ in range(2)]
sts = [torch.zeros(codec.n_blocks(n), dtype=torch.int32, device=dev) for _ in range(2)]


def serial(steps):
    for _ in range(steps):
        codec.compress_into(src, cbs[0])
        codec.decompress_into(cbs[0], outs[0], sts[0])


sA, sB = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
enc_done = [torch.cuda.Event() for _ in range(2)]
dec_done = [torch.cuda.Event() for _ in range(2)]


def piped(steps):
    cur = torch.cuda.current_stream(dev)
    sA.wait_stream(cur)
    sB.wait_stream(cur)
    for k in range(steps):
        i = k & 1
        with torch.cuda.stream(sA):
            if k >= 2:
                sA.wait_event(dec_done[i])  # step k - 2's decode has read cbs[i]
            codec.compress_into(src, cbs[i])
            enc_done[i].record(sA)
        with torch.cuda.stream(sB):
            sB.wait_event(enc_done[i])
            codec.decompress_into(cbs[i], outs[i], sts[i])
            dec_done[i].record(sB)
    cur.wait_stream(sA)
    cur.wait_stream(sB)


def timed(fn):
    fn(3)
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    fn(K)
    torch.cuda.synchronize(dev)
    return (time.perf_counter() - t0) / K


for rnd in range(3):
    for name, fn in (("one stream", serial), ("two in flight", piped)):
        for o in outs:
            o.fill_(0xA5)
        ms = timed(fn) * 1e3
        ok = all(bool(torch.equal(o, src)) for o in outs[: 1 if fn is serial else 2])
        ok = ok and all(int(s.abs().max()) == 0 for s in sts) and int(cbs[0]["status"].abs().max()) == 0
        print(f"round {rnd} {name:14s} {ms:.4f} ms/step  {n / 2**30 / (ms / 1e3):.1f} GiB/s  verified={ok}",
              flush=True)
