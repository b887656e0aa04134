"""Per-call latency of the reference-shaped host entry points (one block
through PCIe per call) against the oracle on one host core.

    python tools/host_latency.py [SIZE ...]   (default 4096 65536 1048576)
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from entropy_coders_amd import compress, compress2, decompress, decompress2  # noqa: E402
from oracle import oracle as O  # noqa: E402

SIZES = [int(a) for a in sys.argv[1:]] or [4096, 65536, 1 << 20]
for n in SIZES:
    src = O.generate(0, 0.155, 0x5EED0002, 0, n)
    comp, _ = compress2(src)
    comp1, _ = compress(src)
    for name, fn in (("fse_compress2", lambda: compress2(src)), ("fse_decompress2", lambda: decompress2(comp)),
                     ("fse_compress", lambda: compress(src)), ("fse_decompress", lambda: decompress(comp1)),
                     ("oracle compress2", lambda: O.compress2(src)), ("oracle decompress2", lambda: O.decompress2(comp))):
        fn()
        reps = 200 if n <= 65536 else 20
        t0 = time.perf_counter()
        for _ in range(reps):
            fn()
        dt = (time.perf_counter() - t0) / reps
        print(f"{n:8d} B  {name:18s} {dt * 1e6:9.1f} us  {n / dt / 2**20:8.1f} MiB/s", flush=True)
