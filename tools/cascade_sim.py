"""Repair-cascade depth of the encoder's guess-and-repair lanes (diagnostics,
on the spec model oracle/spec.py; DESIGN.md section 5, verdict r04 item 6).

For each block and lane boundary: does a lane started from the guessed state
2^L meet the exact trajectory within its S pairs?  A lane whose start is a
guess and that never meets it passes a wrong end state to the lane below,
so the exact state has to travel through every such lane in turn: the
longest run of consecutive non-converging lanes above a lane is the number
of dependent re-encodes (repair rounds) it needs, whatever the lane grouping
(a two-level scheme still has to carry the exact state through the same
lanes, S pairs each).  Prints, per distribution / table log / lane count:
the share of lanes that converge, the per-block maximum run (the round
count the cascade needs), and that run x S as the serial pair-steps floor
against the block's pairs.

    python tools/cascade_sim.py
"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import spec as S  # noqa: E402


def tables(data, L):
    counts, _, tl = S.histogram(data)
    if L is None:
        L = S.optimal_log2(len(data), tl)
    norm = S.normalize(counts, len(data), tl, L)
    if isinstance(norm, tuple):
        norm = norm[0]
    st, dnb, dfs = S.encode_table(norm, L, tl)
    pad = [0] * (256 - len(dnb))
    return np.array(st, np.int64), np.array(list(dnb) + pad, np.int64), np.array(list(dfs) + pad, np.int64), L


def block_runs(kind, prob, L, T, b):
    data = S.generate(kind, prob, 0x5EED0002, b, 65536)
    st, dnb, dfs, L = tables(data, L)
    sym = np.frombuffer(data, np.uint8).astype(np.int64)
    n = len(sym)
    P = n // 2 - 1
    Sl = P // T

    def step(x, s):
        nb = (dnb[s] + x) >> 16
        return st[(x >> nb) + dfs[s]]

    def init(s):
        bo = ((dnb[s] + (1 << 15)) & 0xFFFFFFFF) >> 16
        v = ((bo << 16) - dnb[s]) & 0xFFFFFFFF
        return st[(v >> bo) + dfs[s]]

    x0, x1 = init(sym[n - 2]), init(sym[n - 1])
    tr0 = np.zeros(P + 1, np.int64)
    tr1 = np.zeros(P + 1, np.int64)
    for p in range(P - 1, -1, -1):
        tr0[p + 1], tr1[p + 1] = x0, x1
        x1, x0 = step(x1, sym[2 * p + 1]), step(x0, sym[2 * p])
    tr0[0], tr1[0] = x0, x1
    tops = (np.arange(T - 1) + 1) * Sl  # lanes 0..T-2 (the top lane starts exact)
    y0 = np.full(T - 1, 1 << L)
    y1 = np.full(T - 1, 1 << L)
    met = np.zeros(T - 1, bool)
    for t in range(Sl):
        p = tops - 1 - t
        met |= (y0 == tr0[p + 1]) & (y1 == tr1[p + 1])
        y1 = step(y1, sym[2 * p + 1])
        y0 = step(y0, sym[2 * p])
    met |= (y0 == tr0[tops - Sl]) & (y1 == tr1[tops - Sl])
    # run of non-converging lanes ending at each lane, from the top down
    runs, r = [], 0
    for k in range(T - 2, -1, -1):
        r = 0 if met[k] else r + 1
        runs.append(r)
    return met.mean(), max(runs), Sl, P


def main():
    cases = [("C2 LUT p=0.155", 0, 0.155, None), ("skewed p=0.77", 0, 0.77, 11), ("skewed p=0.77", 0, 0.77, 12)]
    for name, kind, prob, L in cases:
        for T in (64, 16):
            conv, mx, sl = [], [], 0
            for b in range(3):
                c, m, sl, P = block_runs(kind, prob, L, T, b)
                conv.append(c)
                mx.append(m)
            print(f"{name:16s} L={L or 'opt':>3} lanes={T:2d} S={sl:4d}: converge {np.mean(conv):.2f}  "
                  f"per-block max run {mx}  floor {max(mx) * sl:6d} of {P} pair-steps serial "
                  f"({max(mx) * sl / P:.2f} of the block)", flush=True)


if __name__ == "__main__":
    main()
