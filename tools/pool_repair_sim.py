"""Repair of the encoder's guess-and-repair lanes as a job pool (diagnostics, on
the spec model oracle/spec.py; DESIGN.md section 5, round-5 encoder item 10).

The product repairs a block's 63 non-top lanes in lockstep rounds on the
block's own wave: a round lasts as long as its slowest lane (~470 of 512
pairs on C2), and the exec-masked lanes still cost the wave its issued
instructions (round-5 item 9: the encoder's time follows its LDS instructions
issued).  This simulates the same lanes (64 lanes, S = 512, 8 trajectory
slots, both chains per lane as the product runs them) and prints the repair's
wave pair-steps per block for

  rounds   the product: sum over rounds of the slowest lane's steps;
  pool G   one wave repairs the lanes of G blocks from a job queue: a lane
           that meets its record takes the next job (a bad lane, released
           when its upper neighbour's job ended), so the wave's steps are the
           list-scheduling makespan of the jobs on 64 lanes, divided by G.
           ``sw`` pair-steps are added per job for the job switch (source
           pointers, states, slot counters reloaded).

    python tools/pool_repair_sim.py [nblocks] [switch_cost]
"""
import heapq
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import spec as S  # noqa: E402

T, SLOT = 64, 64


def block_jobs(kind, prob, L, b):
    """(round, lane, steps) of every repair job of one block, and the rounds' cost"""
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
    lanes = np.arange(ktop)
    nslot = Sl // SLOT

    def run(c, ks, y):
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

    def init(s):
        bo = ((dnb[s] + (1 << 15)) & 0xFFFFFFFF) >> 16
        v = ((bo << 16) - dnb[s]) & 0xFFFFFFFF
        return st[(v >> bo) + dfs[s]]

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
    jobs = []
    cost = 0
    rnd = 0
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
            for i, k in enumerate(ks):
                rec[c][k, : j[i]] = tr[i, : j[i]]
                if not met[i]:
                    end[c][k] = tr[i, -1]
        anyb = bad[0] | bad[1]
        if not anyb.any():
            break
        sa = np.where(anyb, np.maximum(np.where(bad[0], steps[0], SLOT), np.where(bad[1], steps[1], SLOT)), 0)
        cost += int(sa.max())
        for k in np.nonzero(anyb)[0]:
            jobs.append((rnd, int(k), int(sa[k])))
        rnd += 1
    return jobs, cost


def makespan(blocks, lanes, sw):
    """list scheduling: job (r, k) of block b is released when job (r - 1, k + 1)
    of the same block ends (round 0 at time 0); a free lane takes the earliest
    released job."""
    end = {}
    pend = []
    for b, jobs in enumerate(blocks):
        for r, k, d in jobs:
            pend.append((b, r, k, d))
    pend.sort(key=lambda j: (j[1], -j[2]))
    free = [0.0] * lanes
    heapq.heapify(free)
    done = 0.0
    todo = pend
    while todo:
        rest = []
        progress = False
        for b, r, k, d in todo:
            if r == 0:
                rel = 0.0
            elif (b, r - 1, k + 1) in end:
                rel = end[(b, r - 1, k + 1)]
            elif any(jb == b and jr == r - 1 and jk == k + 1 for jb, jr, jk, _ in todo):
                rest.append((b, r, k, d))
                continue
            else:
                rel = 0.0  # released by a lane that was exact in count mode
            t0 = max(heapq.heappop(free), rel)
            t1 = t0 + d + sw
            end[(b, r, k)] = t1
            heapq.heappush(free, t1)
            done = max(done, t1)
            progress = True
        if not progress:
            raise RuntimeError("dependency cycle")
        todo = rest
    return done


def main():
    nb = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    sw = float(sys.argv[2]) if len(sys.argv) > 2 else 8.0
    for name, kind, prob, L in (("C2 LUT p=0.155", 0, 0.155, None), ("geometric", 1, 0.2, None)):
        blocks, costs = [], []
        for b in range(nb):
            jobs, c = block_jobs(kind, prob, L, b)
            blocks.append(jobs)
            costs.append(c)
        njobs = np.mean([len(j) for j in blocks])
        work = np.mean([sum(d for _, _, d in j) for j in blocks])
        line = f"{name}: rounds {np.mean(costs):.0f} pair-steps per block ({njobs:.0f} jobs, {work / 64:.0f} lane-work / 64)"
        for G in (1, 2, 4, 8):
            if nb % G:
                continue
            ms = [makespan(blocks[i:i + G], 64, sw) / G for i in range(0, nb, G)]
            line += f"  pool{G} {np.mean(ms):.0f}"
        print(line, flush=True)


if __name__ == "__main__":
    main()
