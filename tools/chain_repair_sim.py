"""Repair rounds of the encoder with per-chain convergence (diagnostics, on the
spec model oracle/spec.py).

The two states of fse_compress2 are independent tANS chains (even / odd
symbols, lib.rs:167-176).  The kernel's repair compares the packed state pair
at each trajectory slot (every 64 pairs), so a lane runs both chains until
both have met the record, and a lane whose neighbour's end changed in one
chain only still re-runs the other one.  This simulates the same lanes and
rounds (64 lanes, S = 512, 8 slots) and prints the wave's repair pair-steps
per block for

  A  the product: a round lasts the slowest bad lane's packed convergence,
     every step runs both chains (4 LDS gathers per pair);
  B  per-chain: chain c's steps run while any lane still has chain c bad,
     each costing half a pair-step (2 gathers), plus an overhead per step
     for the source loads, the slot compare and the loop.

    python tools/chain_repair_sim.py [nblocks] [overhead]
"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import spec as S  # noqa: E402

T, SLOT = 64, 64


def block(kind, prob, L, b):
    data = S.generate(kind, prob, 0x5EED0002, b, 65536)
    counts, _, tl = S.histogram(data)
    if L is None:
        L = S.optimal_log2(len(data), tl)
    norm = S.normalize(counts, len(data), tl, L)
    if isinstance(norm, tuple):
        norm = norm[0]
    st, dnb, dfs = S.encode_table(norm, L, tl)
    pad = [0] * (256 - len(dnb))
    st = np.array(st, np.int64)
    dnb = np.array(list(dnb) + pad, np.int64)
    dfs = np.array(list(dfs) + pad, np.int64)
    sym = np.frombuffer(data, np.uint8).astype(np.int64)
    n = len(sym)
    Pm = (n - 2) // 2
    Sl = max(8, ((Pm + T - 1) // T + 7) & ~7)
    ktop = (Pm - 1) // Sl

    def init(s):
        bo = ((dnb[s] + (1 << 15)) & 0xFFFFFFFF) >> 16
        v = ((bo << 16) - dnb[s]) & 0xFFFFFFFF
        return st[(v >> bo) + dfs[s]]

    # chain c of lane k encodes sym[2p + c] for p = pb-1 .. pa
    lanes = np.arange(ktop)  # the non-top lanes (all full, Sl pairs)
    tops = (lanes + 1) * Sl
    nslot = Sl // SLOT

    def run(c, ks, y):
        """states after every SLOT pairs (slot 1..nslot) of chain c, lanes ks from y"""
        y = y.copy()
        out = np.zeros((len(ks), nslot), np.int64)
        tp = (ks + 1) * Sl
        for t in range(Sl):
            s = sym[2 * (tp - 1 - t) + c]
            nb = (dnb[s] + y) >> 16
            y = st[(y >> nb) + dfs[s]]
            if (t + 1) % SLOT == 0:
                out[:, (t + 1) // SLOT - 1] = y
        return out

    # exact top lane (odd n: chain 0 takes one extra step first)
    x0, x1 = init(sym[n - 2]), init(sym[n - 1])
    if n & 1:
        x0, x1 = init(sym[n - 1]), init(sym[n - 2])
    top_end = []
    for c, x in ((0, x0), (1, x1)):
        y = x
        for p in range(Pm - 1, ktop * Sl - 1, -1):
            s = sym[2 * p + c]
            nb = (dnb[s] + y) >> 16
            y = st[(y >> nb) + dfs[s]]
        top_end.append(y)

    rec, start, end = [], [], []
    for c in (0, 1):
        y = np.full(ktop, 1 << L)
        r = run(c, lanes, y)
        rec.append(r)
        start.append(y)
        end.append(r[:, -1].copy())
    costA = 0.0
    costB = [0.0, 0.0]
    rounds = 0
    while True:
        steps = np.zeros((2, ktop), np.int64)
        bad = []
        for c in (0, 1):
            nbr = np.append(end[c][1:], top_end[c])
            bc = nbr != start[c]
            bad.append(bc)
            if not bc.any():
                continue
            ks = np.nonzero(bc)[0]
            start[c][ks] = nbr[ks]
            tr = run(c, ks, start[c][ks])
            eq = tr == rec[c][ks]
            met = eq.any(axis=1)
            j = np.where(met, eq.argmax(axis=1) + 1, nslot)
            steps[c, ks] = j * SLOT
            for i, k in enumerate(ks):  # slots above the meeting point are rewritten
                rec[c][k, : j[i]] = tr[i, : j[i]]
                if not met[i]:
                    end[c][k] = tr[i, -1]
        anyb = bad[0] | bad[1]
        if not anyb.any():
            break
        rounds += 1
        # A: a bad lane runs both chains; a chain whose start did not change meets at slot 1
        sa = np.where(anyb, np.maximum(np.where(bad[0], steps[0], SLOT), np.where(bad[1], steps[1], SLOT)), 0)
        costA += sa.max()
        costB[0] += steps[0].max()
        costB[1] += steps[1].max()
    return costA, costB, rounds


def main():
    nb = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    ov = float(sys.argv[2]) if len(sys.argv) > 2 else 0.2
    for name, kind, prob, L in (("C2 LUT p=0.155", 0, 0.155, None), ("geometric", 1, 0.2, None)):
        A, B0, B1, R = [], [], [], []
        for b in range(nb):
            a, (b0, b1), r = block(kind, prob, L, b)
            A.append(a)
            B0.append(b0)
            B1.append(b1)
            R.append(r)
        A, B0, B1 = np.array(A), np.array(B0), np.array(B1)
        B = 0.5 * (B0 + B1) + ov * np.maximum(B0, B1)
        Aov = A * (1 + ov)
        print(f"{name}: rounds {R}  A pair-steps {A.tolist()}  B chain steps {list(zip(B0.tolist(), B1.tolist()))}  "
              f"cost A {Aov.mean():.0f} B {B.mean():.0f} ({B.mean() / Aov.mean():.2f} of A, overhead {ov})", flush=True)


if __name__ == "__main__":
    main()
