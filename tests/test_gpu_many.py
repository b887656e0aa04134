"""The batching drop-in for a caller with many crate streams:
fse_decompress2_many / fse_decompress_many (include/fsehip.h) through the
C ABI (ctypes), 1,000 crate-format streams per call, each checked against
the oracle's fse_decompress2 / fse_decompress (lib.rs:215-248 / 187-211):
bytes for the good streams, the status name for damaged and degenerate
ones (reference mode, within the stride)."""
import numpy as np
import pytest

from oracle import oracle as O

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch_cuda():
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch


def _streams(rng, n, nstates):
    streams = []
    for i in range(n):
        size = int(rng.choice([65536, 65536, int(rng.integers(2, 65537))]))
        kind = i % 5
        if kind == 0:
            src = O.generate(0, 0.155, 0x5EED0002, i, size)  # the bench's C2 data
        elif kind == 1:
            src = O.generate(0, float(rng.uniform(0.05, 0.8)), int(rng.integers(1 << 30)), 0, size)
        elif kind == 2:
            alpha = rng.choice(256, size=int(rng.integers(2, 200)), replace=False).astype(np.uint8)
            src = alpha[rng.integers(0, len(alpha), size)]
        elif kind == 3:
            src = np.minimum(rng.geometric(0.5, size) - 1, 255).astype(np.uint8)  # C1's shape
        else:
            src = rng.integers(0, 256, size).astype(np.uint8)
        try:
            if nstates == 2:
                L = int(rng.choice([0, 0, 0, 9, 10, 12]))
                comp = O.compress2(src, L or None)[0]
            else:
                comp = O.compress(src)[0]
        except O.OracleError:
            continue
        comp = bytearray(comp)
        if i % 97 == 13:  # damaged
            comp[int(rng.integers(0, len(comp)))] ^= 0x3C
        if i % 211 == 7:  # truncated
            comp = comp[: max(1, len(comp) // 3)]
        streams.append(bytes(comp))
    streams.append(b"")  # EMPTY, as the single call returns it
    return streams


@pytest.mark.parametrize("nstates", [2, 1])
def test_many_streams_exact(torch_cuda, nstates):
    from entropy_coders_amd import decompress2_many

    rng = np.random.default_rng(0x4A11 + nstates)
    streams = _streams(rng, 1000, nstates)
    stride = 65536
    got = decompress2_many(streams, stride, nstates=nstates)
    ref = O.decompress2 if nstates == 2 else O.decompress
    n_ok = n_err = 0
    for i, (x, g) in enumerate(zip(streams, got)):
        try:
            want = ref(x, stride) if x else None
        except O.OracleError as e:
            assert g == e.code, (i, e.code, g)
            n_err += 1
            continue
        if want is None:
            assert g == "EMPTY", (i, g)
            continue
        assert g == want, i
        n_ok += 1
    assert n_ok >= 950 and n_err >= 1 and n_ok + n_err == len(streams) - 1, (n_ok, n_err)


@pytest.mark.parametrize("nstates", [2, 1])
@pytest.mark.parametrize("m", [3, 17, 32, 33])
def test_many_streams_scalar_batches(torch_cuda, nstates, m):
    """Batches of up to 32 streams at table log <= 11 run one scalar-unit
    chain per stream (single_decode_kernel over the batch), larger ones the
    ring kernel: both sides of that boundary, with damaged, truncated,
    ragged and empty streams and short strides, against the oracle."""
    from entropy_coders_amd import decompress2_many

    rng = np.random.default_rng(0x5CA1 + 7 * m + nstates)
    streams = _streams(rng, 3 * m, nstates)
    # keep m (the EMPTY one last), with a damaged and a truncated one among them
    streams = streams[: m - 1] + [streams[-1]]
    streams[1] = bytes(bytearray(streams[1])[: max(1, len(streams[1]) // 2)])
    if m > 3:  # (index m - 1 is the empty stream)
        b = bytearray(streams[2])
        b[len(b) // 2] ^= 0x55
        streams[2] = bytes(b)
    ref = O.decompress2 if nstates == 2 else O.decompress
    for stride in (65536, 30000):
        got = decompress2_many(streams, stride, nstates=nstates)
        for i, (x, g) in enumerate(zip(streams, got)):
            if not x:
                assert g == "EMPTY", (i, g)
                continue
            try:
                want = ref(x, stride)
            except O.OracleError as e:
                assert g == e.code, (m, stride, i, e.code, g)
                continue
            assert g == want, (m, stride, i)


def test_many_streams_short_stride_and_small_batches(torch_cuda):
    """DST_TOO_SMALL per stream when the stride is short, and the one- and
    two-stream batches (which take the single-stream path) agree with the
    batch path."""
    from entropy_coders_amd import decompress2, decompress2_many

    srcs = [O.generate(0, 0.155, 0x5EED0002, i, 65536) for i in range(5)]
    comps = [O.compress2(s)[0] for s in srcs]
    got = decompress2_many(comps, 40000)
    assert got == ["DST_TOO_SMALL"] * 5
    for k in (1, 2, 3):
        got = decompress2_many(comps[:k], 65536)
        assert got == [s.tobytes() for s in srcs[:k]]
    assert decompress2_many([], 16) == []
    assert decompress2(comps[0]) == srcs[0].tobytes()


def test_many_streams_mixed_sizes_and_groups(torch_cuda):
    """Streams above the batch's 4 MiB take the single-stream path inside the
    same call, and a stride large enough to split the batch into several
    staging groups gives the same per-stream results."""
    from entropy_coders_amd import decompress2_many

    big = O.generate(2, 0.0, 0x5EED0009, 0, (5 << 20) + 333)  # near-uniform: > 4 MiB compressed
    smalls = [O.generate(0, 0.155, 0x5EED0002, i, 65536) for i in range(6)]
    comps = [O.compress2(s)[0] for s in smalls[:3]] + [O.compress2(big)[0]] + [O.compress2(s)[0] for s in smalls[3:]]
    assert len(comps[3]) > 4 << 20
    got = decompress2_many(comps, 6 << 20)
    want = [s.tobytes() for s in smalls[:3]] + [big.tobytes()] + [s.tobytes() for s in smalls[3:]]
    assert got == want
    # 96 MiB strides: 5 streams per 512 MiB staging group -> two groups
    got = decompress2_many([O.compress2(s)[0] for s in smalls] * 2, 96 << 20)
    assert got == [s.tobytes() for s in smalls] * 2


def test_many_streams_log_classes(torch_cuda):
    """Streams are grouped by the table log in their header (<= 11, 12,
    13..15), so one L = 15 stream and one header whose log nibble is corrupt
    (L > 15) do not move the other streams off the L <= 11 kernels or fail
    the call: every stream gets its single-call result."""
    from entropy_coders_amd import decompress2_many

    smalls = [O.generate(0, 0.155, 0x5EED0002, i, 4096) for i in range(300)]
    comps = [O.compress2(s)[0] for s in smalls]
    l12 = O.generate(0, 0.155, 0x5EED0005, 0, 65536)
    l15 = O.generate(2, 0.0, 0x5EED0006, 0, 65536).copy()
    l15[-2:] = 250  # rare seeds: the crate's new_first_symbol panics at L = 15 on frequent ones
    c12, c15 = O.compress2(l12, 12)[0], O.compress2(l15, 15)[0]
    assert (c12[0] & 15) + 5 == 12 and (c15[0] & 15) + 5 == 15
    bad = bytearray(comps[7])
    bad[0] = (bad[0] & 0xF0) | 0x0F  # log nibble 15: L = 20
    streams = comps[:100] + [c15] + comps[100:200] + [bytes(bad)] + [c12] + comps[200:]
    # three of each large log too, so the L = 12 and L = 13..15 groups take the batch path
    streams += [c15, c12, c15, c12, c15, c12]
    got = decompress2_many(streams, 65536)
    for i, (x, g) in enumerate(zip(streams, got)):
        try:
            want = O.decompress2(x, 65536)
        except O.OracleError as e:
            assert g == e.code, (i, e.code, g)
            continue
        assert g == want, i
    assert got[100] == l15.tobytes() and got[202] == l12.tobytes()
    assert got[-6:] == [l15.tobytes(), l12.tobytes()] * 3


def test_many_rejects_bad_dst_and_nstates(torch_cuda):
    """The Python mirror refuses an output buffer the C call would overrun
    (too small, wrong dtype, strided, read-only) and an unknown format."""
    from entropy_coders_amd import decompress2_many

    comps = [O.compress2(O.generate(0, 0.155, 0x5EED0002, i, 4096))[0] for i in range(4)]
    for dst in (np.empty(4 * 4096 - 1, np.uint8), np.empty(8 * 4096, np.uint8)[::2], np.empty(4 * 4096, np.uint16),
                [0] * (4 * 4096)):
        with pytest.raises(ValueError):
            decompress2_many(comps, 4096, raw=True, dst=dst)
    ro = np.empty(4 * 4096, np.uint8)
    ro.flags.writeable = False
    with pytest.raises(ValueError):
        decompress2_many(comps, 4096, raw=True, dst=ro)
    with pytest.raises(ValueError):
        decompress2_many(comps, 4096, nstates=3)
    d, lens, st = decompress2_many(comps, 4096, raw=True, dst=np.empty(4 * 4096, np.uint8))
    assert (st == 0).all() and (lens == 4096).all()
