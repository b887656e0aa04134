"""GPU parity of the building blocks and the bitstream behind the C ABI
(histogram.rs, fse.rs, bitstream/*.rs twins), the table-log range 5..15 on
the batched codec, and the sidecar cross-check.  Every call runs the HIP
kernels; the oracle (oracle/) is the checker."""
import threading

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


def _inputs():
    yield O.generate(0, 0.155, 21, 0, 65536)       # C2-like, 48 symbols
    yield O.generate(0, 0.77, 22, 0, 65536)        # skewed, 7 symbols
    yield O.generate(2, 0.0, 23, 0, 65536)         # near-uniform 0..239
    yield O.generate(0, 0.05, 24, 0, 65536)        # normalize_slow at low L
    yield O.generate(1, 0.5, 25, 0, 1001)          # geometric, short
    yield np.frombuffer(bytes([0, 5, 5, 200] * 40 + [255]), dtype=np.uint8)  # sparse alphabet, long zero runs
    from test_gpu_fuzz import _block  # seeded random distributions and lengths

    rng = np.random.default_rng(0xB10C)
    for _ in range(8):
        yield _block(rng, int(rng.integers(2, 65537)))


def _norm_eq(a, b):
    assert a.log2 == b.log2 and a.table_len == b.table_len
    assert list(a.norm) == list(b.norm)


def test_histogram_and_normalize(torch_cuda):
    from entropy_coders_amd import histogram_new, norm_histogram_new, normalize, normalize_optimal

    for src in _inputs():
        h = histogram_new(src)
        ho = O.hist_count(src)
        assert list(h.counts) == list(ho.counts) and h.size == ho.size and h.table_len == ho.table_len
        for L in (0, 5, 6, 8, 9, 11, 12, 13, 14, 15, 20):
            try:
                want, _ = O.normalize(ho, L)
            except O.OracleError as e:
                from entropy_coders_amd import FseError

                with pytest.raises(FseError) as ge:
                    normalize(h, L)
                assert ge.value.code == e.code
                continue
            _norm_eq(normalize(h, L), want)
        want, _ = O.normalize(ho, O.optimal_log2(ho))
        _norm_eq(normalize_optimal(h), want)
        _norm_eq(norm_histogram_new(src), O.norm_new(src))


def test_normalize_errors(torch_cuda):
    from entropy_coders_amd import FseError, histogram_new, norm_histogram_new, normalize

    with pytest.raises(FseError) as e:
        norm_histogram_new(bytes(64))  # table_len 1: (table_len - 1).ilog2() panics
    assert e.value.code == "ALL_ZERO_SYMBOL0"
    with pytest.raises(FseError) as e:
        normalize(histogram_new(b""), 11)
    assert e.value.code in ("ALL_ZERO_SYMBOL0", "EMPTY")


def test_header_write_read(torch_cuda):
    from entropy_coders_amd import FseError, norm_histogram_read, norm_histogram_write, normalize, histogram_new

    for src in _inputs():
        ho = O.hist_count(src)
        for L in (5, 9, 11, 12, 15):
            try:
                nh, _ = O.normalize(ho, L)
            except O.OracleError:
                continue
            want = O.header_write(nh)
            got, bits = norm_histogram_write(normalize(histogram_new(src), L))
            assert got == want
            assert (bits + 7) // 8 == len(want) and bits > 0
            # read back, with trailing bytes after the header (histogram.rs tests)
            tail = bytes(range(7))
            back, used = norm_histogram_read(want + tail)
            ref, rused = O.header_read(want + tail)
            _norm_eq(back, ref)
            assert used == rused == len(want)
    # errors: table log beyond 15 (4-bit field 11 -> 16), truncated header, empty slice
    with pytest.raises(FseError) as e:
        norm_histogram_read(b"\x0b\xff\xff")
    assert e.value.code == "BAD_HEADER"
    nh, _ = O.normalize(O.hist_count(O.generate(0, 0.155, 21, 0, 65536)), 11)
    hdr = O.header_write(nh)
    with pytest.raises(FseError) as e:
        norm_histogram_read(hdr[: len(hdr) // 2])
    assert e.value.code == "BAD_HEADER"
    with pytest.raises(FseError) as e:
        norm_histogram_read(b"")
    assert e.value.code == "EMPTY"


def test_encode_decode_tables(torch_cuda):
    from entropy_coders_amd import decode_table_new, encode_table_new, histogram_new, normalize

    for src in _inputs():
        ho = O.hist_count(src)
        h = histogram_new(src)
        for L in (5, 8, 11, 12, 13, 15):
            try:
                nh_o, _ = O.normalize(ho, L)
            except O.OracleError:
                continue
            nh = normalize(h, L)
            log2, st, dnb, dfs, spread = O.ctable(nh_o)
            et = encode_table_new(nh)
            size = 1 << log2
            assert et.table_log == log2
            assert np.array_equal(np.ctypeslib.as_array(et.table)[:size], st)
            assert np.array_equal(np.ctypeslib.as_array(et.symbols)[:size], spread)
            tt = np.ctypeslib.as_array(et.symbol_tt)
            assert [t[0] for t in tt] == list(dnb) and [t[1] for t in tt] == list(dfs)
            log2, ns, sym, nb = O.dtable_nh(nh_o)
            dt = decode_table_new(nh)
            e = np.ctypeslib.as_array(dt.table)[:size]
            assert dt.table_log == log2
            assert np.array_equal(e["new_state"], ns) and np.array_equal(e["symbol"], sym)
            assert np.array_equal(e["num_bits"], nb)
            big = any(v >= 1 << (log2 - 1) for v in list(nh_o.norm)[: nh_o.table_len])
            assert dt.fast_mode == (0 if big else 1)


def test_compress_returns_its_norm_histogram(torch_cuda):
    from entropy_coders_amd import compress_nh

    src = O.generate(0, 0.2, 0x5EED0001, 0, 32768)
    comp, bits, nh = compress_nh(src)
    want, wbits = O.compress(src)
    assert comp == want and bits == wbits
    _norm_eq(nh, O.norm_new(src))


@pytest.mark.parametrize("offset", range(8))
def test_bitstack_write_read(torch_cuda, offset):
    """bitstream/mod.rs stack_tests_offset: random widths 1..16 (and 0 / up to
    32 here), the writer appending after `offset` existing bytes, the marker
    bit, then the stack read back top down: exact bits, bytes and finish()."""
    from entropy_coders_amd import bitstack_read, bitstack_write

    rng = np.random.default_rng(100 + offset)
    for count in (1, 2, 7, 64, 100, 1000, 5000):
        widths = rng.integers(0, 33 if offset % 2 else 17, count).astype(np.uint8)
        vals = rng.integers(0, 1 << 32, count, dtype=np.uint64)
        masked = (vals & ((np.uint64(1) << widths.astype(np.uint64)) - np.uint64(1))).astype(np.uint64)
        want, wbits = O.bits_write(masked, widths, True)
        prefix = bytes(range(1, offset + 1))
        enc, bits = bitstack_write(np.append(vals, 1).astype(np.uint32), np.append(widths, 1), prefix)
        assert bits == wbits + 1 and enc[:offset] == prefix
        assert len(enc) == offset + (bits + 7) // 8
        got = enc[offset:]
        assert got == want
        read, n_read, fin = bitstack_read(got, widths[::-1])
        assert n_read == count and fin
        assert read == [int(x) for x in masked[::-1]]
        # one read too many fails (None) and leaves finish() false
        read, n_read, fin = bitstack_read(got, np.append(widths[::-1], 1))
        assert n_read == count and not fin


def test_bitstack_read_marker(torch_cuda):
    from entropy_coders_amd import FseError, bitstack_read

    for data in (b"", b"\x12\x00"):
        with pytest.raises(FseError) as e:
            bitstack_read(data, [1])
        assert e.value.code == "NO_MARKER"


def test_bitstream_read(torch_cuda):
    """bitstream/mod.rs stream_tests_offset: fields written without a marker
    and read back FIFO with total_bits; reads past it fail (UnexpectedEof)."""
    from entropy_coders_amd import FseError, bitstream_read

    rng = np.random.default_rng(7)
    for count in (1, 5, 100, 3000):
        widths = rng.integers(1, 17, count).astype(np.uint8)
        vals = rng.integers(0, 1 << 16, count, dtype=np.uint64) & ((1 << widths.astype(np.uint64)) - 1)
        data, total = O.bits_write(vals, widths, False)
        read, n_read, left = bitstream_read(data, total, widths)
        assert n_read == count and left == 0 and read == [int(x) for x in vals]
        read, n_read, left = bitstream_read(data, total, np.append(widths, 3))
        assert n_read == count and left == 0
    with pytest.raises(FseError) as e:
        bitstream_read(b"\x01\x02", 20, [4])  # slice length must be exactly ceil(total_bits / 8)
    assert e.value.code == "BAD_ARG"


def test_bitstream_peek_advance(torch_cuda):
    """BitStreamReader's peek / advance_by / read mixed per field
    (stream_reader.rs:56-119) against the spec model, including the failing
    call at the end and finish()'s remaining bits."""
    from oracle import spec
    from entropy_coders_amd import BITS_ADVANCE, BITS_PEEK, FseError, bitstream_read

    rng = np.random.default_rng(9)
    for count in (1, 7, 200, 5000):
        widths = rng.integers(1, 17, count).astype(np.uint8)
        vals = rng.integers(0, 1 << 16, count, dtype=np.uint64) & ((1 << widths.astype(np.uint64)) - 1)
        data, total = O.bits_write(vals, widths, False)
        ops = rng.integers(0, 3, count).astype(np.uint8)
        # a tail of calls that runs past total_bits
        ops = np.append(ops, [BITS_PEEK, BITS_ADVANCE, 0]).astype(np.uint8)
        w2 = np.append(widths, [16, 16, 16]).astype(np.uint8)
        want = spec.stream_steps(bytes(data), total, w2.tolist(), ops.tolist())
        got = bitstream_read(data, total, w2, ops)
        assert got == (want[0], want[1], want[2]), count
    with pytest.raises(FseError) as e:
        bitstream_read(b"\x01", 8, [1], [3])  # unknown op
    assert e.value.code == "BAD_ARG"


def test_bitstack_device_batched(torch_cuda):
    """fsehip_bitstack_write / read on 3M device-resident fields against the
    oracle's writer."""
    import ctypes as C

    torch = torch_cuda
    from entropy_coders_amd._lib import load

    lib = load()
    rng = np.random.default_rng(11)
    count = 3_000_000
    widths = rng.integers(0, 25, count).astype(np.uint8)
    vals = rng.integers(0, 1 << 32, count, dtype=np.uint64)
    masked = vals & ((np.uint64(1) << widths.astype(np.uint64)) - np.uint64(1))
    want, wbits = O.bits_write(masked, widths, False)
    d_v = torch.from_numpy(vals.astype(np.uint32).view(np.int32)).cuda()
    d_w = torch.from_numpy(widths).cuda()
    d_out = torch.zeros(count * 4 + 16, dtype=torch.uint8, device="cuda")
    d_tot = torch.zeros(1, dtype=torch.int64, device="cuda")
    s = C.c_void_p(torch.cuda.current_stream().cuda_stream)
    assert lib.fsehip_bitstack_write(C.c_void_p(d_v.data_ptr()), C.c_void_p(d_w.data_ptr()), count,
                                     C.c_void_p(d_out.data_ptr()), count * 4 + 16, C.c_void_p(d_tot.data_ptr()),
                                     s) == 0
    torch.cuda.synchronize()
    assert int(d_tot.item()) == wbits
    assert d_out[: len(want)].cpu().numpy().tobytes() == want
    # forward read of the same fields
    d_in = d_out[: (len(want) + 3) // 4 * 4 + 8].clone()
    d_r = torch.zeros(3, dtype=torch.int64, device="cuda")
    d_vals = torch.zeros(count, dtype=torch.int32, device="cuda")
    assert lib.fsehip_bitstream_read(C.c_void_p(d_in.data_ptr()), len(want), wbits, C.c_void_p(d_w.data_ptr()),
                                     count, C.c_void_p(d_vals.data_ptr()), C.c_void_p(d_r.data_ptr()), s) == 0
    torch.cuda.synchronize()
    r = d_r.cpu().numpy()
    assert r[0] == count and r[1] == 1 and r[2] == 0
    assert np.array_equal(d_vals.cpu().numpy().view(np.uint32), masked.astype(np.uint32))


@pytest.mark.parametrize("L", [5, 8, 13, 14, 15])
def test_batched_codec_table_logs(torch_cuda, L):
    """The batched codec across the reference's table-log range: blocks equal
    the oracle's bytes (or carry its panic status), and the ones the
    reference round-trips decode back, with and without the sidecar."""
    torch = torch_cuda
    from entropy_coders_amd import BlockCodec
    from entropy_coders_amd._lib import STATUS

    kind, prob = (0, 0.77) if L < 8 else (0, 0.155)
    codec = BlockCodec(block_size=65536, table_log=L, ckpt_interval=128)
    n = 6 * 65536 + (0 if L == 15 else 1234)
    src = codec.generate(kind, prob, 0x5EED00A0 + L, n)
    host = src.cpu().numpy().copy()
    if L == 15:
        # seeds of norm -1 keep new_first_symbol inside its table (the
        # reference panics on most other seeds: test_oracle golden cases);
        # block 5 keeps its own and must carry the reference's status
        for b in range(5):
            host[(b + 1) * 65536 - 2:(b + 1) * 65536] = [211, 212]
        src = torch.from_numpy(host).cuda()
    cb = codec.compress(src)
    torch.cuda.synchronize()
    status = cb["status"].cpu().numpy()
    ok = []
    for b in range(codec.n_blocks(n)):
        blk = host[b * 65536:(b + 1) * 65536]
        try:
            want, _ = O.compress2(blk, L)
        except O.OracleError as e:
            assert STATUS[int(status[b])] == e.code, (b, status[b])
            continue
        assert status[b] == 0, (b, status[b])
        assert codec.block_bytes(cb, b) == want, b
        ok.append(O.decompress2(want, raw_len=len(blk)) == blk.tobytes())
    assert any(ok)
    if L == 15:  # decode the blocks the reference accepts
        keep = 5 * 65536
        cb = dict(cb, n_total=keep, out=cb["out"][: 5 * codec.slot_bytes])  # blocks 0..4: the first 5 slots
        src = src[:keep]
        status = status[:5]
    if all(ok) and (status == 0).all():
        for side in (True, False):
            out, st = codec.decompress(cb, use_sidecar=side)
            torch.cuda.synchronize()
            assert int(st.abs().max()) == 0 and torch.equal(out, src), side


def test_sidecar_cross_check(torch_cuda):
    """A sidecar that does not belong to the stream is reported, not decoded
    into garbage: another checkpoint interval, or a flipped checkpoint state."""
    torch = torch_cuda
    from entropy_coders_amd import BlockCodec
    from entropy_coders_amd._lib import STATUS

    codec = BlockCodec(block_size=65536, ckpt_interval=128)
    n = 4 * 65536
    src = codec.generate(0, 0.155, 0x5EED00B0, n)
    cb = codec.compress(src)
    out, st = codec.decompress(cb)
    torch.cuda.synchronize()
    assert int(st.abs().max()) == 0 and torch.equal(out, src)
    other = BlockCodec(block_size=65536, ckpt_interval=256)
    cb2 = dict(cb)
    out2 = torch.empty_like(src)
    st2 = torch.zeros(4, dtype=torch.int32, device=src.device)
    other.decompress_into(cb2, out2, st2)
    torch.cuda.synchronize()
    assert all(STATUS[int(x)] == "BAD_SIDECAR" for x in st2.cpu().numpy())
    side = cb["sidecar"].clone()
    per = codec.side_per_block
    side[2 * per + 5] ^= 1 << 33  # block 2, checkpoint 5: decoder state 0
    cb3 = dict(cb, sidecar=side)
    out3, st3 = codec.decompress(cb3)
    torch.cuda.synchronize()
    s3 = st3.cpu().numpy()
    assert STATUS[int(s3[2])] == "BAD_SIDECAR" and s3[0] == 0 and s3[1] == 0 and s3[3] == 0


def test_workspace_shared_stream_two_threads(torch_cuda):
    """Two host threads decoding on the same stream (the decode workspace is
    per stream, grown under its lock): both outputs exact."""
    torch = torch_cuda
    from entropy_coders_amd import BlockCodec

    codec = BlockCodec(block_size=65536, ckpt_interval=128)
    jobs = []
    for i, nb in enumerate((3, 40, 7, 64)):
        src = codec.generate(0, 0.155, 0x5EED00C0 + i, nb * 65536)
        jobs.append((src, codec.compress(src)))
    torch.cuda.synchronize()
    errors = []

    def work(k):
        try:
            for _ in range(6):
                for src, cb in jobs[k::2]:
                    out, st = codec.decompress(cb)
                    torch.cuda.synchronize()
                    if int(st.abs().max()) != 0 or not torch.equal(out, src):
                        errors.append(k)
        except Exception as e:  # noqa: BLE001
            errors.append(repr(e))

    th = [threading.Thread(target=work, args=(k,)) for k in range(2)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert not errors, errors


@pytest.mark.parametrize("nstates,ckpt", [(2, 128), (2, 64), (1, 64)])
@pytest.mark.parametrize("L", [13, 14])
def test_lds_stage_decode_table_logs_13_14(torch_cuda, L, nstates, ckpt):
    """Table logs 13 and 14 decode through the LDS-staged segment kernel (32 /
    64 KiB tables beside the block image): skewed blocks in the 44 KiB stage,
    near-uniform ones (~65 KB) deferred to the 66 KiB list pass, mixed in one
    batch.  Sampled blocks equal the oracle's bytes; every block decodes
    back to its source, with and without the sidecar."""
    torch = torch_cuda
    from entropy_coders_amd import BlockCodec

    B = 65536
    codec = BlockCodec(block_size=B, table_log=L, ckpt_interval=ckpt, nstates=nstates)
    kinds = [(0, 0.77), (2, 0.0), (0, 0.155), (2, 0.0), (0, 0.77), (0, 0.155)]  # 2: near-uniform
    src = torch.cat([codec.generate(k, p, 0x5EED00C0 + 7 * i + L, B) for i, (k, p) in enumerate(kinds)])
    src = src[: len(kinds) * B - 333]  # a ragged last block
    host = src.cpu().numpy()
    cb = codec.compress(src)
    torch.cuda.synchronize()
    assert int(cb["status"].abs().max()) == 0, cb["status"].cpu().numpy()
    for b in (0, 1, 5):  # (the reference's 1-state fse_compress has no table-log argument)
        want = O.compress2(host[b * B:(b + 1) * B], L)[0] if nstates == 2 else O.compress(host[b * B:(b + 1) * B])[0]
        if nstates == 2:
            assert codec.block_bytes(cb, b) == want, b
    lens = cb["comp_len"].cpu().numpy()
    assert lens.max() > 44 * 1024 and lens.min() < 44 * 1024  # both passes run
    for side in (True, False):
        out, st = codec.decompress(cb, use_sidecar=side)
        torch.cuda.synchronize()
        assert int(st.abs().max()) == 0 and torch.equal(out, src), side
