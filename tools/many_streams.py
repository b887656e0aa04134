"""Crossover of the batched host call against one host core (diagnostics):
N crate-format 64 KiB C2 streams (the oracle's fse_compress2 bytes) decoded
by fse_decompress2_many (one call, host buffers in and out), by a loop of
fse_decompress2 calls (small N), and by the C restatement of the crate on
one host core; per-stream microseconds and the crossover N.

    python tools/many_streams.py [N ...]
"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from entropy_coders_amd import decompress2, decompress2_many  # noqa: E402
from oracle import oracle as O  # noqa: E402


def best(fn, reps=3):
    fn()
    t = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        t.append(time.perf_counter() - t0)
    return min(t)


def main():
    ns = [int(x) for x in sys.argv[1:]] or [1, 2, 4, 8, 16, 32, 64, 128, 256, 1000, 4000, 8000]
    pool = [O.compress2(O.generate(0, 0.155, 0x5EED0002, i, 65536))[0] for i in range(256)]
    got = decompress2_many(pool[:64], 65536)
    assert got == [O.generate(0, 0.155, 0x5EED0002, i, 65536).tobytes() for i in range(64)]
    one = best(lambda: [O.decompress2(c, 65536) for c in pool[:64]]) / 64
    print(f"oracle (one host core): {one * 1e6:.1f} us per 64 KiB stream")
    rows = []
    for n in ns:
        streams = [pool[i % len(pool)] for i in range(n)]
        bufs = [np.frombuffer(c, dtype=np.uint8) for c in streams]
        dst = np.empty(n * 65536, dtype=np.uint8)
        # the C call as a caller sees it: host buffers in, one output buffer back
        t_many = best(lambda: decompress2_many(bufs, 65536, raw=True, dst=dst))
        t_loop = best(lambda: [decompress2(c, 65536) for c in streams]) if n <= 16 else None
        rows.append((n, t_many, t_loop))
        print(f"N={n:5d}  many {t_many * 1e3:9.3f} ms ({t_many / n * 1e6:8.1f} us/stream, "
              f"{n * 65536 / t_many / 2**30:6.2f} GiB/s)"
              + (f"  loop {t_loop * 1e3:8.3f} ms" if t_loop else "")
              + f"  one core {n * one * 1e3:8.3f} ms  16 cores {n * one / 16 * 1e3:8.3f} ms")
    x1 = next((n for n, t, _ in rows if t < n * one), None)
    x16 = next((n for n, t, _ in rows if t < n * one / 16), None)
    print(f"crossover: beats one core from N={x1}, 16 cores from N={x16} (of the N measured)")


if __name__ == "__main__":
    main()
