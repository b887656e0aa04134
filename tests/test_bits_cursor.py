"""The bitstream cursors of include/fsehip.h section 1c (BitStackReader,
BitStreamReader, BitStackWriter as O(1)-per-call C-ABI structs), driven one
call at a time exactly as the crate's own callers drive its readers.

Host logic (no GPU): checked against the oracle's restatements
(oracle/fse_oracle.c) and, for the alignment-dependent `available()`, a
line-by-line restatement of stack_reader.rs in this file."""
import numpy as np
import pytest

from oracle import oracle as O


@pytest.fixture(scope="module")
def M():
    import entropy_coders_amd as m

    return m


def at_offset(data: bytes, off: int) -> np.ndarray:
    """`data` in a buffer whose first byte sits at address % 8 == off."""
    raw = np.zeros(len(data) + 16, dtype=np.uint8)
    start = (off - raw.ctypes.data) % 8
    view = raw[start: start + len(data)]
    view[:] = np.frombuffer(data, dtype=np.uint8)
    assert view.ctypes.data % 8 == off
    return view


# ---------------------------------------------------------------- NormHistogram::read
def header_read_by_cursor(M, data):
    """NormHistogram::read (histogram.rs:436-505), restated with one cursor
    call per reader call: every peek/advance width depends on the values
    read before it."""
    r = M.BitStreamReader(data, len(data) * 8)
    log2 = r.read(4) + 5
    if log2 > 15:
        return "BAD_HEADER"
    table = [0] * 256
    symbol = 0
    threshold = 1 << log2
    remaining = threshold + 1
    nbits = log2 + 1
    previous0 = False
    try:
        while remaining > 1 and symbol < 256:
            if previous0:
                while True:
                    try:
                        v = r.peek(16)
                    except EOFError:
                        v = 0
                    if v != 0xFFFF:
                        break
                    r.advance_by(16)
                    symbol += 24
                while True:
                    try:
                        v = r.peek(2)
                    except EOFError:
                        v = 0
                    if v != 3:
                        break
                    r.advance_by(2)
                    symbol += 3
                symbol += r.read(2)
            if symbol >= 256:
                break
            mx = (2 * threshold - 1) - remaining
            try:
                raw = r.peek(nbits)
            except EOFError:
                raw = r.peek(nbits - 1)
            if (raw & (threshold - 1)) < mx:
                r.advance_by(nbits - 1)
                value = raw & (threshold - 1)
            else:
                r.advance_by(nbits)
                value = raw & (2 * threshold - 1)
                if value >= threshold:
                    value -= mx
            value -= 1
            remaining -= abs(value)
            table[symbol] = value
            symbol += 1
            previous0 = value == 0
            while remaining < threshold:
                nbits -= 1
                threshold >>= 1
    except EOFError:
        return "BAD_HEADER"
    if remaining != 1:
        return "BAD_HEADER"
    rest = r.finish_byte()
    return log2, table, symbol, len(data) - len(rest)


def _headers():
    rng = np.random.default_rng(5)
    out = []
    for kind, prob in ((0, 0.155), (0, 0.77), (1, 0.5), (2, 0.0), (0, 0.05)):
        blk = O.generate(kind, prob, 0x5EED0101, 0, 4096 + int(rng.integers(0, 60000)))
        comp, _ = O.compress2(blk)
        out.append(comp)  # header + payload (the reader stops at the header)
    for _ in range(20):  # sparse alphabets: long zero runs (the 0xFFFF / 3 markers)
        alpha = np.sort(rng.choice(256, size=int(rng.integers(2, 12)), replace=False)).astype(np.uint8)
        blk = alpha[rng.integers(0, len(alpha), int(rng.integers(64, 5000)))]
        try:
            comp, _ = O.compress2(blk, int(rng.integers(5, 16)))
        except O.OracleError:
            continue
        out.append(comp)
    return out


@pytest.mark.parametrize("i", range(20))
def test_header_read_driven_by_cursor(M, i):
    hs = _headers()
    data = hs[i % len(hs)]
    nh, used = O.header_read(data)
    got = header_read_by_cursor(M, data)
    assert got != "BAD_HEADER"
    log2, table, tl, consumed = got
    assert log2 == nh.log2 and tl == nh.table_len and consumed == used
    assert table[:tl] == list(nh.norm)[:tl]


def test_header_read_cursor_errors(M):
    data = _headers()[0]
    nh, used = O.header_read(data)
    # truncated headers: the cursor reports EOF where the oracle reports an error
    for cut in range(1, used):
        got = header_read_by_cursor(M, data[:cut])
        with pytest.raises(O.OracleError):
            O.header_read(data[:cut])
        assert got == "BAD_HEADER" or got[3] != used
    assert header_read_by_cursor(M, bytes([0xFF, 0xFF])) == "BAD_HEADER"  # table log 20


# ---------------------------------------------------------------- BitStackReader
class RefStackReader:
    """stack_reader.rs:17-226 on a 64-bit target, with the slice's real
    address (the restatement the C cursor must match, including available())."""

    def __init__(self, buf: np.ndarray):
        self.b = buf.tobytes()
        self.addr = buf.ctypes.data
        n = len(self.b)
        self.ok = n > 0
        if not n:
            return
        ptr = n - 1
        align = (-(self.addr + ptr)) % 4
        ptr = ptr + align - 4 if ptr > 4 - align else 0
        to_read = n - ptr
        self.buffer = int.from_bytes(self.b[ptr: ptr + min(to_read, 8)], "little")
        self.bits = to_read * 8
        self.finished = ptr == 0
        ptr = ptr - 4 if ptr >= 4 else 0
        self.ptr = ptr
        self.reload()
        if self.buffer == 0:
            self.ok = False
            return
        hb = self.buffer.bit_length() - 1
        if self.bits - hb > 8:
            self.ok = False
            return
        self.bits = hb
        self.reload()

    def reload(self):
        M64 = (1 << 64) - 1
        if self.finished:
            return
        if self.ptr == 0:
            to_read = 4 - ((self.addr + self.ptr) & 3)
            self.finished = self.bits <= 32
            if not self.finished:
                to_read = 0
            rd = int.from_bytes(self.b[self.ptr: self.ptr + to_read], "little")
            self.buffer = ((self.buffer << (8 * to_read)) | rd) & M64
            self.bits += 8 * to_read
            return
        will = self.bits <= 32
        rd = int.from_bytes(self.b[self.ptr: self.ptr + 4], "little")
        if will:
            self.buffer = ((self.buffer << 32) | rd) & M64
            self.bits += 32
        off = self.ptr
        self.ptr -= (4 if will else 0) if off >= 4 else (off if will else 0)

    def read(self, n):
        if n > self.bits:
            return None
        v = (self.buffer >> (self.bits - n)) & ((1 << n) - 1)
        self.bits -= n
        self.reload()
        return v


@pytest.mark.parametrize("off", range(8))
@pytest.mark.parametrize("seed", range(4))
def test_stack_reader_one_call_at_a_time(M, off, seed):
    rng = np.random.default_rng(100 + seed)
    count = int(rng.integers(1, 400))
    widths = rng.integers(0, 17, count).astype(np.uint8)
    vals = [int(rng.integers(0, 1 << int(w))) if w else 0 for w in widths]
    data, _ = O.bits_write(vals, widths, True)  # writer + marker bit (lib.rs:178-182)
    buf = at_offset(data, off)
    r = M.BitStackReader(buf)
    ref = RefStackReader(buf)
    assert ref.ok
    assert r.available() == ref.bits
    got = []
    for w in widths[::-1]:  # stack order, one read per call
        v = r.read(int(w))
        rv = ref.read(int(w))
        assert v == rv and r.available() == ref.bits
        got.append(v)
    assert got == vals[::-1]
    assert r.finish() and r.available() == 0
    assert r.read(1) is None and r.peek(1) is None and r.read(0) == 0


@pytest.mark.parametrize("off", range(8))
def test_stack_reader_peek_and_no_reload(M, off):
    rng = np.random.default_rng(7 + off)
    widths = rng.integers(1, 12, 300).astype(np.uint8)
    vals = [int(rng.integers(0, 1 << int(w))) for w in widths]
    data, _ = O.bits_write(vals, widths, True)
    r = M.BitStackReader(at_offset(data, off))
    out = []
    i = len(widths) - 1
    while i >= 1:  # the decoders' pattern: two reads, one reload (lib.rs:227-244)
        a, b = int(widths[i]), int(widths[i - 1])
        assert r.peek(a) == vals[i]
        out.append(r.read_no_reload(a))
        out.append(r.read(b))
        i -= 2
    assert out == [vals[j] for j in range(len(vals) - 1, i, -1)]
    before = r.available()
    r.advance_no_reload(0)
    assert r.available() == before


def test_stack_reader_none_cases(M):
    from entropy_coders_amd import FseError

    for bad in (b"", b"\x00", b"\x12\x00", bytes([1, 0, 0, 0, 0, 0, 0, 0, 0])):
        with pytest.raises(FseError) as e:
            M.BitStackReader(bad)
        assert e.value.code == "NO_MARKER"
    r = M.BitStackReader(b"\x01")  # the marker alone: nothing to read
    assert r.available() == 0 and r.finish() and r.read(1) is None
    with pytest.raises(FseError):
        r.advance_no_reload(1)  # past the buffer: the crate's debug assertion


# ---------------------------------------------------------------- BitStreamReader
@pytest.mark.parametrize("seed", range(6))
def test_stream_reader_ops_match_batched_form(M, seed):
    rng = np.random.default_rng(40 + seed)
    count = int(rng.integers(1, 200))
    widths = rng.integers(1, 33, count).astype(np.uint8)
    vals = [int(rng.integers(0, 1 << int(w))) for w in widths]
    data, bits = O.bits_write(vals, widths, False)
    total = int(bits) - int(rng.integers(0, 8)) if bits > 8 else int(bits)
    total = max(total, 1)
    data = data[: (total + 7) // 8]
    r = M.BitStreamReader(data, total)
    pos = 0
    for w, v in zip(widths, vals):
        w = int(w)
        if pos + w > total:
            with pytest.raises(EOFError):
                r.peek(w)
            with pytest.raises(EOFError):
                r.read(w)
            break
        assert r.peek(w) == (v if pos + w <= bits else v & ((1 << w) - 1))
        if rng.random() < 0.3:
            r.advance_by(w)
        else:
            assert r.read(w) == v
        pos += w
        assert r.available() == total - pos
    rest, rem, off = r.finish()
    assert rem == total - pos and off == pos % 8 and rest == data[pos // 8:]
    assert r.finish_byte() == data[(pos + 7) // 8:]


def test_stream_reader_asserts(M):
    from entropy_coders_amd import FseError

    for data, total in ((b"", 0), (b"\x01\x02", 8), (b"\x01", 9)):
        with pytest.raises(FseError) as e:
            M.BitStreamReader(data, total)
        assert e.value.code == "BAD_ARG"


# ---------------------------------------------------------------- BitStackWriter
@pytest.mark.parametrize("prefix", [b"", b"x", b"abc", b"12345678"])
@pytest.mark.parametrize("seed", range(4))
def test_writer_appends_one_field_per_call(M, prefix, seed):
    rng = np.random.default_rng(70 + seed)
    count = int(rng.integers(0, 500))
    widths = rng.integers(0, 17, count).astype(np.uint8)
    vals = [int(rng.integers(0, 1 << 20)) for _ in widths]  # unmasked values: stray high bits
    w = M.BitStackWriter(prefix)
    clean = []
    pending = 0
    for v, n in zip(vals, widths):
        n = int(n)
        cv = v & ((1 << n) - 1)
        clean.append(cv)
        mode = int(rng.integers(0, 4))
        if mode == 0:
            w.write_bits_unmasked(v, n)
        elif mode == 1:
            w.write_bits(cv, n)
        elif mode == 2:  # raw writes: flush at least every 32 bits (writer.rs:129-137)
            w.write_bits_raw_unmasked(v, n)
            pending += n
        else:
            w.write_bits_raw(cv, n)
            pending += n
        if pending > 16:
            w.flush()
            pending = 0
    out, bits = w.finish()
    want, wbits = O.bits_write(clean, widths, False)
    assert bits == wbits == int(widths.sum())
    assert out == prefix + want


def test_writer_capacity_is_sticky(M):
    import ctypes as C

    from entropy_coders_amd._lib import BitStackWriterState, load

    lib = load()
    dst = (C.c_uint8 * 3)()
    st = BitStackWriterState()
    assert lib.bitstack_writer_new(C.byref(st), dst, 3, 1) == 0
    assert lib.bitstack_writer_write_bits(C.byref(st), 0xABCD, 16) == 0
    assert lib.bitstack_writer_write_bits(C.byref(st), 1, 8) == -7  # DST_TOO_SMALL
    assert lib.bitstack_writer_write_bits(C.byref(st), 1, 1) == -7
    n, b = C.c_size_t(0), C.c_uint64(0)
    assert lib.bitstack_writer_finish(C.byref(st), C.byref(n), C.byref(b)) == -7


# ---------------------------------------------------------------- a whole decoder through the cursor
def test_decompress2_through_the_cursor(M):
    """fse_decompress2's loop (lib.rs:215-248) restated over the stack
    cursor and the oracle's DecodeTable: every width comes from the table
    entry of the state read before it."""
    src = O.generate(0, 0.2, 0x5EED0001, 0, 3001)
    comp, _ = O.compress2(src)
    L, ns, sym, nb, hdr = O.dtable(comp)
    r = M.BitStackReader(comp[hdr:])
    s0, s1 = r.read(L), r.read(L)
    out = []
    while True:
        e = s0
        v = r.read_no_reload(int(nb[e]))
        if v is None:
            out += [sym[s0], sym[s1]]
            break
        out.append(sym[e])
        s0 = int(ns[e]) + v
        e = s1
        v = r.read(int(nb[e]))
        if v is None:
            out += [sym[s1], sym[s0]]
            break
        out.append(sym[e])
        s1 = int(ns[e]) + v
    assert bytes(int(x) for x in out) == src.tobytes()
    assert r.finish()
