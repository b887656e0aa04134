"""CPU tests of the parity oracle: pinned against the reference's own KATs and
properties, the committed golden vectors, and the independent spec model."""
import hashlib
import random

import numpy as np
import pytest

from oracle import oracle as O
from oracle import spec as S


# ---- reference KATs (histogram.rs:589-656) and their normalised tables
def test_flat_256():  # histogram.rs:589-593
    data = bytes(range(256))
    h = O.hist_count(data)
    L = O.optimal_log2(h)
    nh, _ = O.normalize(h, L)
    assert L == 9 and list(nh.norm) == [2] * 256


@pytest.mark.parametrize("log2", range(8, 16))
def test_uniform_dist_256(log2):  # histogram.rs:595-619
    data = b"".join(bytes([x]) * (1 << (log2 - 8)) for x in range(256))
    h = O.hist_count(data)
    assert list(h.counts) == [1 << (log2 - 8)] * 256
    nh, _ = O.normalize(h, log2)
    L = max(log2, 9)
    assert nh.log2 == L and list(nh.norm) == [1 << (L - 8)] * 256
    _hist_verify(h, log2)


@pytest.mark.parametrize("log2", range(8, 16))
def test_exp_dist(log2):  # histogram.rs:621-656
    size = 1 << log2
    rem, data, sym = size, [], 0
    while True:
        data += [sym] * (rem >> 1)
        rem -= rem >> 1
        sym += 1
        if rem == 1:
            data.append(sym)
            break
    h = O.hist_count(bytes(data))
    exp = [(size >> (1 + j)) if j < log2 else (1 if j == log2 else 0) for j in range(256)]
    assert list(h.counts) == exp
    nh, _ = O.normalize(h, log2)
    want = [size >> (1 + j) for j in range(log2 - 1)] + [-1, -1]
    assert list(nh.norm)[: log2 + 1] == want
    _hist_verify(h, log2)


def _hist_verify(h, log2):  # histogram.rs:553-587
    nh, _ = O.normalize(h, log2)
    assert sum(abs(x) for x in nh.norm) == 1 << nh.log2
    for c, v in zip(h.counts, nh.norm):
        assert (c == 0) == (v == 0)
    enc = O.header_write(nh)
    test = b"I am a test"
    nh2, used = O.header_read(enc + test)
    assert (enc + test)[used:] == test
    assert list(nh2.norm) == list(nh.norm) and nh2.log2 == nh.log2
    assert nh2.table_len == nh.table_len


@pytest.mark.parametrize("log2", range(8, 16))
def test_rand_dist_uniform(log2):  # histogram.rs:658-670, seeded here
    rng = np.random.default_rng(log2)
    for _ in range(8):
        data = rng.integers(0, 256, size=1 << (log2 + 2), dtype=np.uint8)
        _hist_verify(O.hist_count(data), log2)


# ---- bitstream properties (bitstream/mod.rs:29-165) at all 8 offsets
@pytest.mark.parametrize("offset", range(8))
def test_stack_roundtrip_offsets(offset):
    rng = random.Random(offset)
    for trial in range(20):
        widths = [rng.randint(1, 16) for _ in range(rng.randint(1, 100))]
        vals = [rng.getrandbits(w) for w in widths]
        stream, wbits = O.bits_write(vals, widths, True)
        assert wbits == sum(widths)
        assert len(stream) == (sum(widths) + 1 + 7) // 8  # mod.rs:52-59
        # the stack reader must be independent of where the slice starts
        buf = bytes(offset) + stream
        got, left = O.bits_read_stack(buf[offset:], widths)
        assert got == vals and left == 0


def test_stack_reader_framing():  # stack_reader.rs:18-20, 77-83
    with pytest.raises(O.OracleError) as e:
        O.bits_read_stack(b"", [])
    assert e.value.code == "NO_MARKER"
    with pytest.raises(O.OracleError) as e:
        O.bits_read_stack(b"\x05\x00", [])
    assert e.value.code == "NO_MARKER"


# ---- codec round trips (lib.rs:280-302), seeded
@pytest.mark.parametrize("fmt", [1, 2])
@pytest.mark.parametrize("n", [2, 3, 4, 5, 17, 1000, 1001, 65536, 65537])
def test_roundtrip(fmt, n):
    src = O.generate(0, 0.2, 99, n, n)
    if len(set(src.tolist())) == 1:
        pytest.skip("single-symbol input")
    if fmt == 2:
        comp, _ = O.compress2(src)
        assert O.decompress2(comp) == src.tobytes()
    else:
        comp, _ = O.compress(src)
        assert O.decompress(comp) == src.tobytes()


@pytest.mark.parametrize("prob,log2", [(0.77, 9), (0.77, 12), (0.05, 9), (0.995, 11)])
def test_roundtrip_skewed_and_slow(prob, log2):
    src = O.generate(0, prob, 5, 0, 65536)
    comp, _ = O.compress2(src, log2)
    assert O.decompress2(comp) == src.tobytes()


def test_error_codes():
    with pytest.raises(O.OracleError) as e:
        O.compress2(b"")
    assert e.value.code == "EMPTY"
    with pytest.raises(O.OracleError) as e:
        O.compress2(b"\x07")
    assert e.value.code == "TOO_SHORT"
    with pytest.raises(O.OracleError) as e:
        O.compress2(bytes(100))
    assert e.value.code == "ALL_ZERO_SYMBOL0"
    comp, _ = O.compress2(b"\x09" * 100)  # single non-zero symbol encodes fine
    with pytest.raises(O.OracleError) as e:
        O.decompress2(comp)  # ... but the reference decoder never terminates
    assert e.value.code == "SINGLE_SYMBOL"
    assert O.decompress2(comp, raw_len=100) == b"\x09" * 100
    with pytest.raises(O.OracleError) as e:
        O.decompress2(comp[:-1] + b"\x00")
    assert e.value.code in ("NO_MARKER", "BAD_HEADER")


def test_release_wrap_small_inputs():
    # n = 2..4: (size-1).ilog2()-2 wraps in a release build -> tableLog 11
    for n in (2, 3, 4):
        h = O.hist_count(bytes(range(1, n + 1)))
        assert O.optimal_log2(h) == 11


# ---- golden vectors
def test_golden_vectors(golden):
    manifest, arrays = golden
    for case in manifest["cases"]:
        src = arrays[case["name"] + "__src"]
        regen = O.generate(case["kind"], case["prob"], case["seed"], 0, case["n"])
        for i, v in case.get("patch", {}).items():
            regen[int(i)] = v
        assert np.array_equal(regen, src)
        if "status" in case:  # a reference panic, e.g. new_first_symbol at tableLog 15
            with pytest.raises(O.OracleError) as e:
                O.compress2(src, case["log2"]) if case["format"] == 2 else O.compress(src)
            assert e.value.code == case["status"], case["name"]
            continue
        comp = arrays[case["name"] + "__comp"].tobytes()
        assert hashlib.sha256(comp).hexdigest() == case["sha256_comp"]
        if case["format"] == 2:
            got, bits = O.compress2(src, case["log2"])
            dec = O.decompress2(comp, raw_len=case["n"])
        else:
            got, bits = O.compress(src)
            dec = O.decompress(comp)
        assert (dec == src.tobytes()) == case.get("roundtrip", True), case["name"]
        assert got == comp and bits == case["payload_bits"], case["name"]


def test_golden_table_log_range(golden):
    """Golden cases cover the reference's whole tableLog range 5..15 (and the
    clamps of Histogram::normalize, histogram.rs:96): the effective L is in
    each header's first 4 bits."""
    manifest, arrays = golden
    seen = set()
    for case in manifest["cases"]:
        if case["format"] == 2 and "status" not in case:
            seen.add((arrays[case["name"] + "__comp"][0] & 15) + 5)
    assert {5, 8, 9, 10, 11, 12, 13, 14, 15} <= seen, sorted(seen)
    statuses = {c["status"] for c in manifest["cases"] if "status" in c}
    assert "ENCODER_INIT" in statuses


def test_golden_block_digests(golden):
    manifest, _ = golden
    g = manifest["c2_blocks_1mib"]
    for d in g["blocks"]:
        src = O.generate(g["kind"], g["prob"], g["seed"], d["block"], g["n"])
        comp, bits = O.compress2(src)
        assert hashlib.sha256(comp).hexdigest() == d["sha256_comp"]
        assert bits == d["payload_bits"]


@pytest.mark.parametrize("kind,prob", [(0, 0.2), (1, 0.5), (2, 0.0), (0, 0.77), (0, 0.05)])
def test_oracle_matches_spec(kind, prob):
    for n in (2, 3, 9, 64, 333, 2048, 4097):
        src = O.generate(kind, prob, 1234, n, n).tobytes()
        assert S.generate(kind, prob, 1234, n, n) == src
        for log2 in (None, 9, 12):
            try:
                want = S.compress2(src, log2)
            except S.SpecError as e:
                with pytest.raises(O.OracleError) as ei:
                    O.compress2(src, log2)
                assert ei.value.code == e.code
                continue
            assert O.compress2(src, log2) == want


def test_checkpoints_consistent():
    src = O.generate(0, 0.155, 3, 0, 65536)
    comp, _ = O.compress2(src)
    bp, s0, s1 = O.checkpoints2(comp, 512)
    assert len(bp) == 64
    assert bp[0] > bp[-1]  # decoding walks the stack downward


def test_checkpoints1_consistent():
    """1-state checkpoints: one per `interval` symbols of the n-1 decoded by
    the loop plus the one before the final state symbol when it lands on the
    grid; the first holds the seed state popped first (lib.rs:197)."""
    for n, iv in [(65536, 512), (5000, 16), (4097, 64)]:
        src = O.generate(1, 0.5, 4, 1, n)
        comp, _ = O.compress(src)
        bp, s0 = O.checkpoints1(comp, iv)
        assert len(bp) == (n - 1) // iv + 1
        assert np.all(np.diff(bp.astype(np.int64)) < 0)


@pytest.mark.parametrize("case", range(40))
def test_oracle_matches_spec_random(case):
    """The two independent restatements agree on seeded random blocks (the
    fuzz generator's distributions, lengths up to 3 KiB, table logs 5..15,
    both formats), including the error statuses and the decode."""
    from test_gpu_fuzz import _block

    rng = np.random.default_rng(0x5BEC + case)
    src = _block(rng, int(rng.integers(2, 3073))).tobytes()
    log2 = [None, 5, 8, 11, 12, 15][int(rng.integers(0, 6))]
    for enc_o, enc_s, dec_s in ((lambda b: O.compress2(b, log2), lambda b: S.compress2(b, log2), S.decompress2),
                                (O.compress, S.compress, S.decompress)):
        try:
            want = enc_s(src)
        except S.SpecError as e:
            with pytest.raises(O.OracleError) as ei:
                enc_o(src)
            assert ei.value.code == e.code, case
            continue
        got = enc_o(src)
        assert got == want, case
        if len(set(src)) > 1:
            assert dec_s(want[0]) == src, case


@pytest.mark.parametrize("prob,n", [(0.2, 1 << 15), (0.5, 333), (0.05, 4096), (0.77, 1001)])
def test_headerless_variant(prob, n):
    """fse.rs:394-434 (the crate's own compress / decompress tests): the
    headerless 1-state stream is lib.rs's fse_compress output after its
    header, and decodes back with the caller's NormHistogram."""
    src = O.generate(0, prob, 0x5EED0001, 0, n).tobytes()
    norm, L, tl, payload, bits = S.compress_headerless(src)
    whole, wbits = O.compress(src)
    head = S.header_write(norm, L, tl)
    assert whole == head + payload and wbits == bits
    assert S.decompress_headerless(norm, L, tl, payload) == src
