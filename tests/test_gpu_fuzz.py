"""Seeded randomized parity sweep of the batched path against the oracle:
block sizes, ragged lengths, distributions (LUT-skewed, uniform subsets,
sparse alphabets, occasional degenerate blocks), table logs 5..15, both
formats (fse_compress2 / fse_compress) and checkpoint intervals.  Every
block's bytes and status are compared with the oracle, and each batch is
decoded through every route: the sidecar segments, the sidecar-less serial
decoder, and the serial decoder that rebuilds the sidecar."""
import os

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


def _block(rng, n):
    kind = rng.integers(0, 6)
    if kind == 0:  # the bench's LUT generator at a random skew
        return O.generate(0, float(rng.uniform(0.03, 0.9)), int(rng.integers(1 << 30)), 0, n)
    if kind == 1:  # uniform over a random subset of the alphabet
        alpha = rng.choice(256, size=int(rng.integers(2, 257)), replace=False).astype(np.uint8)
        return alpha[rng.integers(0, len(alpha), n)]
    if kind == 2:  # sparse alphabet with long zero runs in the header, skewed weights
        alpha = np.sort(rng.choice(256, size=int(rng.integers(2, 9)), replace=False)).astype(np.uint8)
        w = rng.random(len(alpha)) ** 3 + 1e-3
        return alpha[rng.choice(len(alpha), size=n, p=w / w.sum())]
    if kind == 3:  # geometric symbols (C1's shape)
        return np.minimum(rng.geometric(float(rng.uniform(0.2, 0.8)), n) - 1, 255).astype(np.uint8)
    if kind == 4:  # degenerate: a single symbol, all zeros (a reference panic) or two symbols
        return [np.full(n, int(rng.integers(1, 256)), np.uint8), np.zeros(n, np.uint8),
                (rng.random(n) < 0.001).astype(np.uint8) * 200][int(rng.integers(0, 3))]
    return rng.integers(0, 256, n).astype(np.uint8)  # near-uniform full alphabet


# FSEHIP_FUZZ_CASES / FSEHIP_FUZZ_SEED widen the sweep for a one-off run (default: 48 cases)
@pytest.mark.parametrize("case", range(int(os.environ.get("FSEHIP_FUZZ_CASES", 48))))
def test_random_batches(torch_cuda, case):
    _random_batch(torch_cuda, int(os.environ.get("FSEHIP_FUZZ_SEED", 0xF0220)), case)


# cases the wide sweeps found: (seed, case) -> what they caught
# (draw version 1: the block-size and checkpoint lists those sweeps used)
REGRESSIONS = [
    (77000, 3),  # L = 15: the crate's own decode changes the last symbols (new_first_symbol)
    (910000, 107),  # L = 13, LDS-staged segments: a 26-bit pair below the old 24-bit window
]


@pytest.mark.parametrize("seed,case", REGRESSIONS)
def test_random_batch_regressions(torch_cuda, seed, case):
    _random_batch(torch_cuda, seed, case, draw=1)


def draw_case(seed, case, draw=2):
    """The batch of (seed, case): (nstates, block, table_log, ckpt, sizes,
    blocks).  draw 1: the lists of the sweeps that found REGRESSIONS; draw 2
    adds 128 KiB blocks (the windowed reader above the 66 KiB stage) and 8..32
    checkpoints (several segment rounds per workgroup)."""
    rng = np.random.default_rng(seed + case)
    nstates = int(rng.choice([1, 2]))
    block = int(rng.choice([512, 1040, 4096, 20000, 65536] if draw == 1 else [512, 1040, 4096, 20000, 65536, 65536, 131072]))
    nblocks = int(rng.integers(1, 9))
    last = int(rng.integers(2, block + 1))
    table_log = 0 if nstates == 1 else int(rng.choice([0, 0, 5, 7, 9, 11, 12, 13, 14, 15]))
    if draw == 1:
        ckpt = int(rng.choice([0, 64, 128, 256]))
    else:
        ckpt = int(rng.choice([0, 16, 32, 64, 64, 128, 256] if nstates == 1 else [0, 8, 16, 32, 64, 64, 128, 256]))
    sizes = [block] * (nblocks - 1) + [last]
    blocks = [_block(rng, s) for s in sizes]
    return nstates, block, table_log, ckpt, sizes, blocks


def _random_batch(torch_cuda, seed, case, draw=2):
    torch = torch_cuda
    from entropy_coders_amd import BlockCodec
    from entropy_coders_amd._lib import STATUS

    nstates, block, table_log, ckpt, sizes, blocks = draw_case(seed, case, draw)
    host = np.concatenate(blocks)
    n = len(host)

    codec = BlockCodec(block_size=block, table_log=table_log, ckpt_interval=ckpt, nstates=nstates)
    src = torch.from_numpy(host).cuda()
    cb = codec.compress(src)
    routes = [("serial", codec.decompress(cb, use_sidecar=False))]
    if ckpt:
        routes.append(("sidecar", codec.decompress(cb)))
        rebuilt = codec.build_sidecar(cb)
        routes.append(("rebuild", rebuilt[::2]))
    torch.cuda.synchronize()
    est = cb["status"].cpu().numpy()
    spb = codec.side_per_block
    for b, s in enumerate(blocks):
        what = (case, b, nstates, block, table_log, ckpt)
        try:
            if nstates == 2:
                want, wbits = O.compress2(s, table_log or None)
            else:
                want, wbits = O.compress(s)
        except O.OracleError as e:
            assert STATUS.get(int(est[b])) == e.code, what
            for name, (out, st) in routes:
                assert int(st[b]) != 0, (name, what)
            continue
        assert est[b] == 0, (what, STATUS.get(int(est[b])))
        assert codec.block_bytes(cb, b) == want, what
        assert int(cb["payload_bits"][b]) == wbits, what
        # the reference's own decode of its bytes: the source, except at L = 15
        # when new_first_symbol's wrapped index lands on another symbol's state
        # (fse.rs:210-218): then the crate's round trip changes the last symbols,
        # and the GPU must decode as the crate does
        ref = s
        if nstates == 2 and table_log == 15:
            ref = np.frombuffer(O.decompress2(want, raw_len=len(s)), np.uint8)
        lo = b * block
        for name, (out, st) in routes:
            assert int(st[b]) == 0, (name, what, STATUS.get(int(st[b])))
            assert np.array_equal(out[lo: lo + len(s)].cpu().numpy(), ref), (name, what)
        if ckpt:
            side = rebuilt[1]
            assert torch.equal(side[b * spb: (b + 1) * spb], cb["sidecar"][b * spb: (b + 1) * spb]), what
    assert n == sum(sizes)


@pytest.mark.parametrize("case", range(int(os.environ.get("FSEHIP_FUZZ_HOST_CASES", 16))))
def test_random_host_calls(torch_cuda, case):
    """The reference-shaped host entry points on random blocks: fse_compress2
    (and with an explicit table log, clamped as Histogram::normalize does),
    fse_decompress2, fse_compress, fse_decompress, against the oracle."""
    from entropy_coders_amd import FseError, compress, compress2, compress2_log, decompress, decompress2

    rng = np.random.default_rng(int(os.environ.get("FSEHIP_FUZZ_SEED", 0xA110)) + case)
    s = _block(rng, int(rng.integers(2, 65537)))
    L = int(rng.integers(0, 21))
    for enc, ref, dec, rdec in ((compress2, O.compress2, decompress2, O.decompress2),
                                (compress, O.compress, decompress, O.decompress),
                                (lambda x: compress2_log(x, L), lambda x: O.compress2(x, L), decompress2,
                                 O.decompress2)):
        try:
            want, wbits = ref(s)
        except O.OracleError as e:
            with pytest.raises(FseError) as g:
                enc(s)
            assert g.value.code == e.code, (case, L)
            continue
        got, bits = enc(s)
        assert got == want and bits == wbits, (case, L)
        if len(set(s.tolist())) > 1:  # a single-symbol stream never ends in the reference
            # the crate's own decode (= s, except for L = 15 blocks whose
            # new_first_symbol state belongs to another symbol)
            assert dec(got) == rdec(want), (case, L)


@pytest.mark.parametrize("rep", range(int(os.environ.get("FSEHIP_FUZZ_STREAM_REPS", 1))))
@pytest.mark.parametrize("nstates", [2, 1])
def test_decompress_streams(torch_cuda, nstates, rep):
    """fsehip_decompress_streams: a batch of crate streams of random sizes (no
    sidecar, no raw length), some damaged, some single-symbol, some above
    the table-log limit, each decoded as the crate's fse_decompress2 /
    fse_decompress (reference mode, the oracle) would within the stride."""
    _streams_case(nstates, 0x57AE + nstates + 2 * rep + int(os.environ.get("FSEHIP_FUZZ_SEED", 0)), draw=2)


# a wide sweep's finding: a 1-state stream longer than the stride whose state
# at the cut has nb = 0 was reported SINGLE_SYMBOL instead of DST_TOO_SMALL
@pytest.mark.parametrize("seed", [0x57AE + 1 + 2 * 13 + 123000, 0x57AE + 1 + 2 * 23 + 123000])
def test_decompress_streams_regressions(torch_cuda, seed):
    _streams_case(1, seed, draw=1)


@pytest.mark.parametrize("rep", range(int(os.environ.get("FSEHIP_FUZZ_STREAM_REPS", 1))))
@pytest.mark.parametrize("nstates", [2, 1])
def test_decompress_many_random(torch_cuda, nstates, rep):
    """fse_decompress2_many / fse_decompress_many (host buffers, the batching
    drop-in) on the same random stream sets as test_decompress_streams:
    every stream's bytes or status equal the oracle's single-stream call."""
    _streams_case(nstates, 0x3A11 + nstates + 2 * rep + int(os.environ.get("FSEHIP_FUZZ_SEED", 0)), draw=2,
                  host=True)


def _streams_case(nstates, seed, draw, host=False):
    """60 crate streams of one seed.  draw 1: the lists of the sweep that found
    the regressions above; draw 2 adds table logs 5..8, 14, 15, longer streams
    and other strides.  host: through fse_decompress2_many (any table log in
    one call) instead of fsehip_decompress_streams at each bound."""
    from entropy_coders_amd import decompress2_many, decompress_streams

    rng = np.random.default_rng(seed)
    stride = 24000 if draw == 1 else int(rng.choice([24000, 40016, 65536]))
    streams, logs = [], []
    for i in range(60):
        s = _block(rng, int(rng.integers(2, 20000 if draw == 1 else 48000)))
        if nstates == 1:
            L = 0
        elif draw == 1:
            L = int(rng.choice([0, 0, 0, 9, 12, 13]))
        else:
            L = int(rng.choice([0, 0, 0, 5, 8, 9, 11, 12, 13, 14, 15]))
        try:
            comp = O.compress2(s, L or None)[0] if nstates == 2 else O.compress(s)[0]
        except O.OracleError:
            continue
        comp = bytearray(comp)
        if i % 11 == 5:  # damage
            comp[int(rng.integers(0, len(comp)))] ^= 0x5A
        streams.append(bytes(comp))
        logs.append((comp[0] & 15) + 5)
    ref_dec = O.decompress2 if nstates == 2 else O.decompress
    if host:
        got = decompress2_many(streams, stride, nstates=nstates)
        for i, (x, g) in enumerate(zip(streams, got)):
            try:
                want = ref_dec(x, stride)
            except O.OracleError as e:
                assert g == e.code, (i, e.code, g)
                continue
            assert g == want, i
        return
    for mtl in (11, 12, 13, 14, 15):
        got = decompress_streams(streams, stride, nstates=nstates, max_table_log=mtl)
        for i, (x, g) in enumerate(zip(streams, got)):
            if logs[i] > mtl and logs[i] <= 15:
                assert g == "UNSUPPORTED", (i, mtl, g)
                continue
            try:
                want = ref_dec(x, stride)
            except O.OracleError as e:
                assert g == e.code, (i, mtl, e.code, g)
                continue
            assert g == want, (i, mtl)


def _check_serial(torch, nstates: int) -> None:
    """Sidecar-less decode of ragged batches (several block sizes, the
    bench's data at random skews) and of crate streams (the oracle's bytes,
    some damaged) in the crate's own termination, against the oracle."""
    from entropy_coders_amd import BlockCodec, decompress_streams

    rng = np.random.default_rng(0xDEF0 + nstates)
    for block in (512, 1040, 20000, 65536):
        sizes = [block] * int(rng.integers(9, 41)) + [int(rng.integers(2, block + 1))]
        host = np.concatenate([O.generate(0, float(rng.uniform(0.05, 0.8)), int(rng.integers(1 << 30)), 0, s)
                               for s in sizes])
        codec = BlockCodec(block_size=block, ckpt_interval=64 * nstates, nstates=nstates)
        src = torch.from_numpy(host).cuda()
        cb = codec.compress(src)
        out, st = codec.decompress(cb, use_sidecar=False)
        torch.cuda.synchronize()
        assert int(st.abs().max()) == 0, block
        assert torch.equal(out[: len(host)], src), block
    comp_fn = (lambda x: O.compress2(x, None)[0]) if nstates == 2 else (lambda x: O.compress(x)[0])
    dec_fn = O.decompress2 if nstates == 2 else O.decompress
    streams = []
    for i in range(40):
        comp = bytearray(comp_fn(O.generate(0, float(rng.uniform(0.05, 0.8)), i, 0, int(rng.integers(2, 30000)))))
        if i % 7 == 3:
            comp[int(rng.integers(0, len(comp)))] ^= 0x5A
        streams.append(bytes(comp))
    got = decompress_streams(streams, 24000, nstates=nstates, max_table_log=11)
    for i, (x, g) in enumerate(zip(streams, got)):
        try:
            want = dec_fn(x, 24000)
        except O.OracleError as e:
            assert g == e.code, (i, e.code, g)
            continue
        assert g == want, i


@pytest.mark.parametrize("nstates", [2, 1])
@pytest.mark.parametrize("defer", ["1", "0"])
def test_serial_deferred_symbols(torch_cuda, defer, nstates):
    """Both formats' sidecar-less decode at L <= 11: with the symbols deferred
    to sym_map_kernel (the product default: state pairs in the workspace,
    then the map) and with the single-kernel serial decode (the product's
    fallback when that workspace cannot be allocated), selected in a child
    process on the diagnostics build (FSEHIP_SERIAL_DEFER=0; the product
    library reads no environment)."""
    if defer == "1":
        _check_serial(torch_cuda, nstates)
        return
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    if not os.path.exists(os.path.join(root, "entropy_coders_amd", "libfsehip_diag.so")):
        pytest.fail("libfsehip_diag.so missing: build it (make -C entropy_coders_amd diag / __graft_entry__.build())")
    env = dict(os.environ, FSEHIP_LIB="libfsehip_diag.so", FSEHIP_SERIAL_DEFER="0", PYTHONPATH=root)
    code = ("import torch, tests.test_gpu_fuzz as t; import entropy_coders_amd._lib as L; "
            "assert L.LIB_PATH.endswith('libfsehip_diag.so'); "
            f"t._check_serial(torch, {nstates}); print('child-ok')")
    r = subprocess.run([sys.executable, "-c", code], cwd=root, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and "child-ok" in r.stdout, (r.stdout[-2000:], r.stderr[-4000:])


@pytest.mark.parametrize("nstates", [2, 1])
@pytest.mark.parametrize("seed", range(int(os.environ.get("FSEHIP_FUZZ_DAMAGE_SEEDS", 4))))
def test_host_decode_damaged_streams(torch_cuda, nstates, seed):
    """The host fse_decompress2 / fse_decompress (single_decode_kernel at table
    logs <= 11, the serial kernels above) on damaged crate streams and at
    random capacities: the decoded bytes, or the status, equal the oracle's
    reference-mode result (lib.rs:187-248: None -> a status, a full Vec ->
    DST_TOO_SMALL)."""
    from entropy_coders_amd import FseError, compress, compress2, compress2_log, decompress, decompress2

    rng = np.random.default_rng(0xDA3A6E + 17 * seed + nstates)
    for case in range(24):
        n = int(rng.integers(3, 9000))
        s = O.generate(int(rng.integers(0, 3)), float(rng.uniform(0.05, 0.8)), int(rng.integers(1 << 30)), 0, n)
        if len(set(s.tolist())) < 2:
            continue
        L = int(rng.choice([0, 0, 9, 11, 12]))
        try:
            if nstates == 2:
                comp = (compress2_log(s, L) if L else compress2(s))[0]
                dec, rdec = decompress2, O.decompress2
            else:
                comp = compress(s)[0]
                dec, rdec = decompress, O.decompress
        except FseError:  # e.g. a table log the histogram cannot take (the oracle agrees: test_random_host_calls)
            continue
        b = bytearray(comp)
        what = int(rng.integers(0, 5))
        if what == 1 and len(b) > 8:  # flip a payload bit
            i = int(rng.integers(len(b) // 2, len(b)))
            b[i] ^= 1 << int(rng.integers(0, 8))
        elif what == 2 and len(b) > 4:  # truncate
            b = b[: int(rng.integers(1, len(b)))]
        elif what == 3:  # a different last byte (the marker)
            b[-1] = int(rng.integers(0, 256))
        elif what == 4 and len(b) > 2:  # damage the header
            b[int(rng.integers(0, min(len(b), 6)))] ^= 1 << int(rng.integers(0, 8))
        cap = int(rng.choice([n + 64, max(1, n // 2), n, 4 * n + 4096]))
        try:
            want = rdec(bytes(b), cap=cap)
        except O.OracleError as e:
            with pytest.raises(FseError) as g:
                dec(bytes(b), cap=cap)
            assert g.value.code == e.code, (seed, case, what, cap)
            continue
        assert dec(bytes(b), cap=cap) == want, (seed, case, what, cap)
