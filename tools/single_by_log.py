"""fse_decompress2 per-call time by table log (one 64 KiB C2 block; profiles/r06/hl/by_log.txt)."""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from entropy_coders_amd import decompress2
from entropy_coders_amd.fse import compress2_log
from oracle import oracle as O
src = O.generate(0, 0.155, 0x5EED0002, 0, 65536)
for L in (7, 8, 9, 10, 11, 12):
    comp, bits = compress2_log(src, L)
    assert decompress2(comp) == bytes(src)
    reps = 100
    t0 = time.perf_counter()
    for _ in range(reps):
        decompress2(comp)
    dt = (time.perf_counter() - t0) / reps
    print(f"L={L} comp={len(comp)} decompress2 {dt*1e6:.1f} us  {dt*1e9/32768:.1f} ns/pair", flush=True)
