"""CPU model of the per-table rank check in wave_build_spread
(entropy_coders_amd/csrc/fse_device.hpp, RankAtomic): both check modes are
restated in numpy over random spreads, with the LDS atomics' lane order
either kept (ascending, as gfx950 does) or scrambled inside random 64-lane
chunks (what a GPU breaking that order could produce).  The check must pass
every correct table and flag every wrong one, since a missed violation would
mean wrong bytes with status OK and a false alarm a needless rebuild.

Reference order: fse.rs:157-162 (stateTable), fse.rs:312-337 (DecodeTable):
the positions of one symbol take consecutive ranks in ascending position
order."""
import numpy as np
import pytest

WAVE = 64


def spread(rng, L, nsym):
    """sym_at for a random normalised histogram: any symbol multiset of 2^L."""
    size = 1 << L
    counts = rng.multinomial(size - nsym, rng.dirichlet(np.ones(nsym) * 0.7)) + 1
    sym_at = np.repeat(np.arange(nsym), counts)
    rng.shuffle(sym_at)
    return sym_at, counts


def atomic_ranks(sym_at, counts, rng, scramble):
    """Slot g (= cumul[s] + rank) taken by each position, chunk by chunk; the
    lanes of a chunk hitting one counter get their values in ascending lane
    order, or (scramble) in a random order per chunk.  Also the counter value
    after each chunk for each position's symbol (the read-back)."""
    size = len(sym_at)
    cumul = np.concatenate([[0], np.cumsum(counts)[:-1]])
    cnt = cumul.copy()
    g = np.empty(size, np.int64)
    end = np.empty(size, np.int64)
    for i0 in range(0, size, WAVE):
        lanes = np.arange(i0, min(i0 + WAVE, size))
        order = rng.permutation(len(lanes)) if scramble else np.arange(len(lanes))
        for k in order:
            i = lanes[k]
            g[i] = cnt[sym_at[i]]
            cnt[sym_at[i]] += 1
        end[lanes] = cnt[sym_at[lanes]]
    return g, end, cumul


def correct(sym_at, g):
    """Ranks follow positions inside every symbol."""
    pos_of = np.empty_like(g)
    pos_of[g] = np.arange(len(g))
    s_of = sym_at[pos_of]
    same = s_of[1:] == s_of[:-1]
    return bool(np.all(pos_of[1:][same] > pos_of[:-1][same]))


def check_inverse(g, end):
    """Inverse mode (decode tables): inv8[g] = lane | last-in-chunk << 6;
    flag a non-last slot whose successor holds a lane not above it."""
    size = len(g)
    inv8 = np.empty(size, np.int64)
    lane = np.arange(size) % WAVE
    inv8[g] = lane | np.where(g + 1 == end, 0x40, 0)
    cur, nxt = inv8, np.append(inv8[1:], 0x40)
    bad = ((cur & 0x40) == 0) & ((cur & 63) >= (nxt & 63))
    return not bad.any()


def check_statetable(sym_at, g):
    """stateTable mode (encoder): st[g] = size + position; a descent between
    consecutive slots is allowed only across a symbol boundary."""
    size = len(g)
    st = np.empty(size, np.int64)
    st[g] = size + np.arange(size)
    a, b = st[:-1], st[1:]
    desc = a > b
    bad = desc & (sym_at[a - size] == sym_at[b - size])
    return not bad.any()


@pytest.mark.parametrize("L,nsym", [(5, 3), (6, 40), (9, 20), (11, 48), (11, 200), (12, 9), (15, 256)])
def test_rank_check_model(L, nsym):
    rng = np.random.default_rng(0xC4EC + L * 1000 + nsym)
    n_bad = 0
    for trial in range(24):
        sym_at, counts = spread(rng, L, min(nsym, (1 << L) - 1))
        for scramble in (False, True):
            g, end, _ = atomic_ranks(sym_at, counts, rng, scramble)
            ok = correct(sym_at, g)
            if not scramble:
                assert ok
            n_bad += not ok
            assert check_inverse(g, end) == ok, (L, nsym, trial, scramble)
            assert check_statetable(sym_at, g) == ok, (L, nsym, trial, scramble)
    assert n_bad > 0  # the scrambled runs did produce wrong tables to catch


def test_descending_injection_is_caught():
    """The diagnostics build's fault injection (chunk 0's ranks in
    descending lane order) yields a wrong table whenever a symbol occurs twice
    in the first 64 positions, and both checks see it."""
    rng = np.random.default_rng(7)
    sym_at, counts = spread(rng, 11, 48)
    size = len(sym_at)
    cumul = np.concatenate([[0], np.cumsum(counts)[:-1]])
    cnt = cumul.copy()
    g = np.empty(size, np.int64)
    end = np.empty(size, np.int64)
    for i0 in range(0, size, WAVE):
        lanes = np.arange(i0, i0 + WAVE)
        for i in (lanes[::-1] if i0 == 0 else lanes):
            g[i] = cnt[sym_at[i]]
            cnt[sym_at[i]] += 1
        end[lanes] = cnt[sym_at[lanes]]
    assert len(set(sym_at[:64])) < 64 and not correct(sym_at, g)
    assert not check_inverse(g, end) and not check_statetable(sym_at, g)
