"""Generate tests/golden/ fixtures from the C oracle, cross-checked by spec.py.

TEST INFRASTRUCTURE ONLY.  The reference ships no golden vectors (its tests
draw from an unseeded rand::thread_rng, lib.rs:272), so exact bytes are pinned
by two independent restatements agreeing: every stored output is produced by
oracle/fse_oracle.c and re-derived byte-for-byte by oracle/spec.py before it
is written.  Run:  python oracle/gen_golden.py
"""
from __future__ import annotations

import hashlib
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))

from oracle import oracle as O  # noqa: E402
from oracle import spec as S  # noqa: E402

OUT = os.path.join(os.path.dirname(HERE), "tests", "golden")

# (name, generator kind, prob, seed, n, tableLog or None, format)
CASES = [
    ("c1_geometric_64k", 1, 0.5, 0x5EED0001, 65536, None, 2),
    ("bench_lut020_32k", 0, 0.2, 0x5EED0001, 32768, None, 2),
    ("c2_lut0155_64k", 0, 0.155, 0x5EED0002, 65536, None, 2),
    ("c5_uniform240_L9", 2, 0.0, 0x5EED0005, 65536, 9, 2),
    ("c5_uniform240_L10", 2, 0.0, 0x5EED0005, 65536, 10, 2),
    ("c5_uniform240_L11", 2, 0.0, 0x5EED0005, 65536, 11, 2),
    ("c5_uniform240_L12", 2, 0.0, 0x5EED0005, 65536, 12, 2),
    ("c5_skew077_L9", 0, 0.77, 0x5EED0005, 65536, 9, 2),
    ("c5_skew077_L10", 0, 0.77, 0x5EED0005, 65536, 10, 2),
    ("c5_skew077_L11", 0, 0.77, 0x5EED0005, 65536, 11, 2),
    ("c5_skew077_L12", 0, 0.77, 0x5EED0005, 65536, 12, 2),
    ("c5_slow_lut005_L9", 0, 0.05, 0x5EED0005, 65536, 9, 2),
    ("odd_lut020_4099", 0, 0.2, 11, 4099, None, 2),
    ("tiny_n2", 0, 0.2, 12, 2, None, 2),
    ("tiny_n3", 0, 0.2, 13, 3, None, 2),
    ("tiny_n5", 0, 0.5, 14, 5, None, 2),
    ("small_1001", 1, 0.5, 15, 1001, None, 2),
    # table logs across the reference's whole range (histogram.rs:96 clamps
    # requests to 5..15 and raises them to ilog2(table_len - 1) + 2)
    ("skew077_L5", 0, 0.77, 0x5EED0006, 65536, 5, 2),
    ("skew077_L8", 0, 0.77, 0x5EED0006, 65536, 8, 2),
    ("lut0155_L8", 0, 0.155, 0x5EED0006, 65536, 8, 2),
    ("lut0155_L13", 0, 0.155, 0x5EED0006, 65536, 13, 2),
    ("lut0155_L14", 0, 0.155, 0x5EED0006, 65536, 14, 2),
    ("lut0155_L15", 0, 0.155, 0x5EED0006, 65536, 15, 2),
    ("uniform240_L13", 2, 0.0, 0x5EED0006, 65536, 13, 2),
    ("uniform240_L15", 2, 0.0, 0x5EED0006, 65536, 15, 2),
    ("skew077_L15_odd", 0, 0.77, 0x5EED0006, 40001, 15, 2),
    # at L = 15 new_first_symbol only stays inside the table for seeds of
    # norm -1/1 (or some powers of two): two rare symbols as the seeds
    ("lut0155_L15_rare_seeds", 0, 0.155, 0x5EED0006, 65536, 15, 2, {65534: 200, 65535: 201}),
    ("lut020_log0", 0, 0.2, 0x5EED0006, 8192, 0, 2),  # normalize(0) acts as 5, raised to 8
    ("lut020_log20", 0, 0.2, 0x5EED0006, 8192, 20, 2),  # clamped to 15
    ("onestate_lut020_32k", 0, 0.2, 0x5EED0001, 32768, None, 1),
    ("onestate_odd_777", 0, 0.3, 16, 777, None, 1),
]


def _spec_compress(data: bytes, log2, fmt):
    if fmt == 1:
        return S.compress(data)
    return S.compress2(data, log2)


def main() -> None:
    os.makedirs(OUT, exist_ok=True)
    arrays: dict[str, np.ndarray] = {}
    manifest = {"generator": "oracle/gen_golden.py", "cases": []}
    for name, kind, prob, seed, n, log2, fmt, *patch in CASES:
        src = O.generate(kind, prob, seed, 0, n)
        assert S.generate(kind, prob, seed, 0, n) == src.tobytes(), name
        for i, v in (patch[0] if patch else {}).items():
            src[i] = v
        try:
            if fmt == 1:
                comp, bits = O.compress(src)
            else:
                comp, bits = O.compress2(src, log2)
        except O.OracleError as e:  # a reference panic: recorded as its status
            try:
                _spec_compress(src.tobytes(), log2, fmt)
                raise AssertionError(f"spec accepts {name}, oracle says {e.code}")
            except S.SpecError as se:
                assert str(se) == e.code, (name, str(se), e.code)
            arrays[name + "__src"] = src
            manifest["cases"].append({"name": name, "kind": kind, "prob": prob, "seed": seed, "n": n,
                                      "log2": log2, "format": fmt, "status": e.code,
                                      "patch": {str(k): v for k, v in (patch[0] if patch else {}).items()}})
            print(f"{name:24s} n={n:6d} status={e.code}")
            continue
        scomp, sbits = _spec_compress(src.tobytes(), log2, fmt)
        assert comp == scomp and bits == sbits, f"C oracle and spec disagree on {name}"
        if fmt == 2:
            dec = O.decompress2(comp, raw_len=n)
        else:
            dec = O.decompress(comp)
        # the reference's own stream at L = 15 may not round-trip (a seed state
        # from another symbol's range); everything else must
        assert dec == src.tobytes() or log2 == 15, name
        arrays[name + "__src"] = src
        arrays[name + "__comp"] = np.frombuffer(comp, dtype=np.uint8)
        manifest["cases"].append({
            "name": name, "kind": kind, "prob": prob, "seed": seed, "n": n, "log2": log2,
            "format": fmt, "payload_bits": bits, "comp_len": len(comp),
            "sha256_comp": hashlib.sha256(comp).hexdigest(), "roundtrip": dec == src.tobytes(),
            "patch": {str(k): v for k, v in (patch[0] if patch else {}).items()},
        })
        print(f"{name:24s} n={n:6d} comp={len(comp):6d} bits={bits}")

    # 1 MiB of C2 data as 16 x 64 KiB blocks: digests only (inputs regenerate).
    digests = []
    for b in range(16):
        src = O.generate(0, 0.155, 0x5EED0002, b, 65536)
        comp, bits = O.compress2(src)
        digests.append({"block": b, "comp_len": len(comp), "payload_bits": bits,
                        "sha256_comp": hashlib.sha256(comp).hexdigest()})
    manifest["c2_blocks_1mib"] = {"kind": 0, "prob": 0.155, "seed": 0x5EED0002, "n": 65536,
                                  "blocks": digests}
    # Spec check of two of those blocks (slow path, a few seconds each).
    for b in (0, 15):
        src = O.generate(0, 0.155, 0x5EED0002, b, 65536).tobytes()
        assert hashlib.sha256(S.compress2(src)[0]).hexdigest() == digests[b]["sha256_comp"]

    np.savez_compressed(os.path.join(OUT, "golden_v1.npz"), **arrays)
    with open(os.path.join(OUT, "golden_v1.json"), "w") as f:
        json.dump(manifest, f, indent=1)
    print("wrote", OUT)


if __name__ == "__main__":
    main()
