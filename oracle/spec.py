"""Pure-Python spec model of the reference FSE coder (second, independent restatement).

TEST INFRASTRUCTURE ONLY: used by tests/ and oracle/gen_golden.py to cross-check
the C oracle (oracle/fse_oracle.c) byte-for-byte.  It is deliberately written
differently from the C oracle -- bit lists instead of accumulators, Python big
integers with explicit u32/u64 wrapping -- so that a shared misreading of the
reference is less likely to pass unnoticed.  It is slow: use it on inputs of a
few KiB.

Each function cites the reference (Cognoscan/entropy_coders, /root/reference)
file:line it restates.  Integer semantics are those of a Rust release build.
"""
from __future__ import annotations

LOG_MIN, LOG_MAX, LOG_DEFAULT = 5, 15, 11  # lib.rs:9-12
M32 = (1 << 32) - 1
RTB = [0, 473195, 504333, 520860, 550000, 700000, 750000, 830000]  # histogram.rs:100


class SpecError(Exception):
    """A reference panic / None / Err, carried as a status name."""

    def __init__(self, code: str):
        super().__init__(code)
        self.code = code


def ilog2(x: int) -> int:
    if x <= 0:
        raise SpecError("ilog2(0)")
    return x.bit_length() - 1


# ---------------------------------------------------------------- bit I/O
class BitSink:
    """LSB-first bit appender (BitStackWriter semantics, writer.rs:140-222)."""

    def __init__(self):
        self.bits: list[int] = []

    def put(self, val: int, n: int) -> None:
        for i in range(n):
            self.bits.append((val >> i) & 1)

    def to_bytes(self) -> bytes:
        out = bytearray((len(self.bits) + 7) // 8)
        for i, b in enumerate(self.bits):
            if b:
                out[i >> 3] |= 1 << (i & 7)
        return bytes(out)


def stack_bits(payload: bytes) -> list[int]:
    """BitStackReader::new (stack_reader.rs:17-92): the bits below the marker."""
    if not payload or payload[-1] == 0:
        raise SpecError("NO_MARKER")
    total = (len(payload) - 1) * 8 + ilog2(payload[-1])
    return [(payload[i >> 3] >> (i & 7)) & 1 for i in range(total)]


class Stack:
    def __init__(self, payload: bytes):
        self.bits = stack_bits(payload)

    def pop(self, n: int):
        """peek/read (stack_reader.rs:176-215): None if fewer than n bits remain."""
        if n > len(self.bits):
            return None
        chunk = self.bits[len(self.bits) - n:]
        del self.bits[len(self.bits) - n:]
        return sum(b << i for i, b in enumerate(chunk))


def stream_steps(data: bytes, total_bits: int, widths, ops):
    """BitStreamReader (stream_reader.rs:16-119) driven by one call per
    field: op 0 = read (peek then advance_by, 56-60), 1 = peek (82-114), 2 =
    advance_by (67-75, no value: 0 here).  Bits are LSB-first, bytes past the
    slice read as zero, and any call with bits_read + bits > total_bits fails
    (UnexpectedEof), which ends the list.  Returns (values, calls that
    returned Ok, available() after them)."""
    if not data or (total_bits + 7) // 8 != len(data):
        raise SpecError("BAD_ARG")  # the constructor's asserts (17-21)
    v = int.from_bytes(data, "little")
    pos, out = 0, []
    for w, op in zip(widths, ops):
        if pos + w > total_bits:
            break
        out.append(0 if op == 2 else (v >> pos) & ((1 << w) - 1))
        if op != 1:
            pos += w
    return out, len(out), total_bits - pos


# ---------------------------------------------------------------- histogram
def histogram(data: bytes):
    """Histogram::new (histogram.rs:18-66) -> (counts, size, table_len)."""
    counts = [0] * 256
    for b in data:
        counts[b] += 1
    nz = [s for s in range(256) if counts[s]]
    table_len = (nz[-1] if nz else 0) + 1
    return counts, len(data), table_len


def optimal_log2(size: int, table_len: int) -> int:
    """histogram.rs:264-277 (release: (size-1).ilog2()-2 wraps as u32)."""
    min_src = ilog2(size) + 1
    min_sym = ilog2(table_len - 1) + 2
    max_bits = (ilog2(size - 1) - 2) & M32
    return max(LOG_MIN, min(LOG_MAX, max(min(LOG_DEFAULT, max_bits), min(min_src, min_sym))))


def normalize(counts, size, table_len, log2):
    """Histogram::normalize (histogram.rs:95-155) -> (norm, L, used_slow)."""
    L = max(min(max(log2, LOG_MIN), LOG_MAX), ilog2(table_len - 1) + 2)
    scale = 62 - L
    step = (1 << 62) // size
    v_step = 1 << (scale - 20)
    low_t = size >> L
    to_dist = 1 << L
    largest, largest_p = 0, 0
    norm = [0] * 256
    for i in range(table_len):
        t = counts[i]
        if t == size:
            norm[i] = to_dist
            return norm, L, False
        if t == 0:
            continue
        if t <= low_t:
            norm[i] = -1
            to_dist -= 1
            continue
        p = (t * step) >> scale
        if p < 8:
            p += 1 if (t * step - (p << scale)) > v_step * RTB[p] else 0
        if p > largest_p:
            largest_p, largest = p, i
        norm[i] = p
        to_dist -= p
    if to_dist != 0 and -to_dist >= (largest_p >> 1):
        return normalize_slow(counts, size, table_len, L), L, True
    norm[largest] += to_dist
    return norm, L, False


def normalize_slow(counts, size, table_len, L):
    """histogram.rs:157-261 (u32 arithmetic)."""
    UN = -2
    low_t = size >> L
    low_one = ((size * 3) & M32) >> (L + 1)
    norm = [0] * 256
    td = 1 << L
    total = size
    for s in range(table_len):
        t = counts[s]
        if t == 0:
            continue
        if t <= low_t:
            norm[s], td, total = -1, td - 1, total - t
        elif t <= low_one:
            norm[s], td, total = 1, td - 1, total - t
        else:
            norm[s] = UN
    if td == 0:
        return norm
    if total // td > low_one:
        low = ((total * 3) & M32) // ((td * 2) & M32)
        for s in range(table_len):
            if norm[s] == UN and counts[s] <= low:
                norm[s], td, total = 1, td - 1, total - counts[s]
    if (1 << L) - td == table_len:
        vmax, imax = 0, 0
        for s in range(256):
            if counts[s] > vmax:
                vmax, imax = counts[s], s
        norm[imax] += td
        return norm
    if total == 0:
        while td:
            moved = False
            for s in range(table_len):
                if norm[s] > 0:
                    norm[s] += 1
                    td -= 1
                    moved = True
                    if td == 0:
                        break
            if not moved:
                raise SpecError("CURSED")
        return norm
    vsl = 62 - L
    mid = (1 << (vsl - 1)) - 1
    r_step = ((1 << vsl) * td + mid) // total
    acc = mid
    for s in range(table_len):
        if norm[s] == UN:
            end = acc + counts[s] * r_step
            w = (end >> vsl) - (acc >> vsl)
            if w < 1:
                raise SpecError("CURSED")
            norm[s] = w
            acc = end
    return norm


def norm_table_len(norm) -> int:
    nz = [s for s in range(256) if norm[s] != 0]
    return (nz[-1] if nz else 0) + 1


# ---------------------------------------------------------------- header
def header_write(norm, L, table_len) -> bytes:
    """NormHistogram::write (histogram.rs:376-431)."""
    w = BitSink()
    w.put(L - LOG_MIN, 4)
    thr = 1 << L
    rem = thr + 1
    zc = 0
    nb = L + 1
    for s in norm[:table_len]:
        if rem <= 1:
            break
        if zc:
            if s == 0:
                zc += 1
                continue
            zc -= 1
            while zc >= 24:
                w.put(0xFFFF, 16)
                zc -= 24
            while zc >= 3:
                w.put(3, 2)
                zc -= 3
            w.put(zc, 2)
        mx = 2 * thr - 1 - rem
        rem -= abs(s)
        c = s + 1
        if c >= thr:
            c += mx
        w.put(c, nb - (1 if c < mx else 0))
        zc = 1 if c == 1 else 0
        if rem < 1:
            raise SpecError("BAD_TABLE")
        while rem < thr:
            nb -= 1
            thr >>= 1
    return w.to_bytes()


def header_read(data: bytes):
    """NormHistogram::read (histogram.rs:436-505) -> (norm, L, table_len, consumed)."""
    if not data:
        raise SpecError("EMPTY")
    bits = [(data[i >> 3] >> (i & 7)) & 1 for i in range(len(data) * 8)]
    pos = 0

    def peek(n):
        if pos + n > len(bits):
            return None
        return sum(bits[pos + i] << i for i in range(n))

    def adv(n):
        nonlocal pos
        if pos + n > len(bits):
            raise SpecError("BAD_HEADER")
        pos += n

    v = peek(4)
    if v is None:
        raise SpecError("BAD_HEADER")
    adv(4)
    L = v + LOG_MIN
    if L > LOG_MAX:
        raise SpecError("BAD_HEADER")
    norm = [0] * 256
    sym = 0
    thr = 1 << L
    rem = thr + 1
    nb = L + 1
    prev0 = False
    while rem > 1 and sym < 256:
        if prev0:
            while (peek(16) or 0) == 0xFFFF:
                adv(16)
                sym += 24
            while (peek(2) or 0) == 3:
                adv(2)
                sym += 3
            r2 = peek(2)
            if r2 is None:
                raise SpecError("BAD_HEADER")
            adv(2)
            sym += r2
        if sym >= 256:
            break
        mx = 2 * thr - 1 - rem
        raw = peek(nb)
        if raw is None:
            raw = peek(nb - 1)
        if raw is None:
            raise SpecError("BAD_HEADER")
        if (raw & (thr - 1)) < mx:
            adv(nb - 1)
            val = raw & (thr - 1)
        else:
            adv(nb)
            val = raw & (2 * thr - 1)
            if val >= thr:
                val -= mx
        val -= 1
        rem -= abs(val)
        norm[sym] = val
        sym += 1
        prev0 = val == 0
        while rem < thr:
            nb -= 1
            thr >>= 1
    if rem != 1:
        raise SpecError("BAD_HEADER")
    return norm, L, sym, (pos + 7) // 8


# ---------------------------------------------------------------- tables
def spread(norm, L, table_len):
    """Symbol spread (fse.rs:110-151, 294-326)."""
    size = 1 << L
    sym = [0] * size
    ht = size - 1
    for s in range(table_len):
        if norm[s] < 0:
            if ht >= 0:
                sym[ht] = s
            ht -= 1
    step = size * 5 // 8 + 3
    pos = 0
    for s in range(table_len):
        for _ in range(max(norm[s], 0)):
            sym[pos] = s
            pos = (pos + step) & (size - 1)
            while pos > ht:
                pos = (pos + step) & (size - 1)
    if pos != 0:
        raise SpecError("BAD_TABLE")
    return sym


def encode_table(norm, L, table_len):
    """EncodeTable::update (fse.rs:101-189) -> (st, dnb, dfs)."""
    size = 1 << L
    cumul = [0] * 256
    acc = 0
    for s in range(table_len):
        cumul[s] = acc
        acc += 1 if norm[s] == -1 else norm[s]
    sym = spread(norm, L, table_len)
    st = [0] * size
    for i, s in enumerate(sym):
        st[cumul[s]] = size + i
        cumul[s] += 1
    dnb, dfs = [0] * 256, [0] * 256
    total = 0
    for s in range(table_len):
        x = norm[s]
        if x == 0:
            dnb[s] = ((L + 1) << 16) - (1 << L)
        elif x in (-1, 1):
            dnb[s], dfs[s] = (L << 16) - (1 << L), total - 1
            total += 1
        else:
            mb = L - ilog2(x - 1)
            dnb[s], dfs[s] = (mb << 16) - (x << mb), total - x
            total += x
    return st, dnb, dfs


def decode_table(norm, L, table_len):
    """DecodeTable::update (fse.rs:280-338) -> list of (new_state, symbol, nb)."""
    size = 1 << L
    nxt = [0] * 256
    for s in range(table_len):
        nxt[s] = 1 if norm[s] <= -1 else norm[s]
    sym = spread(norm, L, table_len)
    dt = []
    for s in sym:
        ns = nxt[s]
        nxt[s] += 1
        nb = L - ilog2(ns)
        dt.append((((ns << nb) - size) & 0xFFFF, s, nb))
    return dt


# ---------------------------------------------------------------- codecs
class _Enc:
    """Encoder (fse.rs:196-251)."""

    def __init__(self, tab, first: int):
        # new_first_symbol (fse.rs:210-218): u32 wrapping, the index an i32
        # (wrapping add) turned usize, then a bounds-checked read that panics
        # outside the table (reachable at tableLog 15)
        self.st, self.dnb, self.dfs = tab
        b = self.dnb[first]
        bo = ((b + (1 << 15)) & M32) >> 16
        v = ((bo << 16) - b) & M32
        idx = ((v >> bo) + self.dfs[first]) & M32
        if idx >= 1 << 31:
            idx -= 1 << 32
        if not 0 <= idx < len(self.st):
            raise SpecError("ENCODER_INIT")
        self.x = self.st[idx]

    def step(self, s: int, sink: BitSink):
        bo = ((self.dnb[s] + self.x) & M32) >> 16
        sink.put(self.x & ((1 << bo) - 1), bo)
        self.x = self.st[(self.x >> bo) + self.dfs[s]]

    def finish(self, L: int, sink: BitSink):
        sink.put(self.x & ((1 << L) - 1), L)


def compress2(src: bytes, log2: int | None = None) -> tuple[bytes, int]:
    """fse_compress2 (lib.rs:146-183); log2=None uses NormHistogram::new."""
    counts, size, tl = histogram(src)
    if size == 0:
        raise SpecError("EMPTY")
    if tl == 1:
        raise SpecError("ALL_ZERO_SYMBOL0")
    if log2 is None:
        if size == 1:
            raise SpecError("TOO_SHORT")
        log2 = optimal_log2(size, tl)
    norm, L, _ = normalize(counts, size, tl, log2)
    if size < 2:
        raise SpecError("TOO_SHORT")
    head = header_write(norm, L, tl)
    tab = encode_table(norm, L, tl)
    sink = BitSink()
    n = len(src)
    if n % 2:
        e0, e1 = _Enc(tab, src[n - 1]), _Enc(tab, src[n - 2])
        e0.step(src[n - 3], sink)
        top = (n - 3) // 2
    else:
        e0, e1 = _Enc(tab, src[n - 2]), _Enc(tab, src[n - 1])
        top = n // 2 - 1
    for k in range(top - 1, -1, -1):
        e1.step(src[2 * k + 1], sink)
        e0.step(src[2 * k], sink)
    e1.finish(L, sink)
    e0.finish(L, sink)
    sink.put(1, 1)
    return head + sink.to_bytes(), len(sink.bits)


def compress_headerless(src: bytes):
    """The crate's test-module fse_compress (fse.rs:394-421): the 1-state
    stream of lib.rs:112-143 with no header in front (the caller keeps the
    NormHistogram).  Returns (norm, L, table_len, payload, payload bits)."""
    counts, size, tl = histogram(src)
    if size == 0:
        raise SpecError("EMPTY")
    if tl == 1:
        raise SpecError("ALL_ZERO_SYMBOL0")
    if size == 1:
        raise SpecError("TOO_SHORT")
    norm, L, _ = normalize(counts, size, tl, optimal_log2(size, tl))
    tab = encode_table(norm, L, tl)
    sink = BitSink()
    n = len(src)
    chunks = [src[i:i + 2] for i in range(0, n, 2)]
    first = chunks.pop()
    e = _Enc(tab, first[-1])
    if len(first) > 1:
        e.step(first[0], sink)
    for ch in reversed(chunks):
        e.step(ch[1], sink)
        e.step(ch[0], sink)
    e.finish(L, sink)
    sink.put(1, 1)
    return norm, L, tl, sink.to_bytes(), len(sink.bits)


def compress(src: bytes) -> tuple[bytes, int]:
    """fse_compress, one state (lib.rs:112-143): the header (hist.write) and,
    from the next byte on, the headerless stream."""
    norm, L, tl, payload, bits = compress_headerless(src)
    return header_write(norm, L, tl) + payload, bits


def _single_symbol(norm, L) -> bool:
    return any(v == (1 << L) for v in norm)


def decompress2(data: bytes, raw_len: int | None = None) -> bytes:
    """fse_decompress2 (lib.rs:215-248).  raw_len: container mode (exact length)."""
    norm, L, tl, used = header_read(data)
    stack = Stack(data[used:])
    dt = decode_table(norm, L, tl)
    if raw_len is None and _single_symbol(norm, L):
        raise SpecError("SINGLE_SYMBOL")
    s0 = stack.pop(L)
    s1 = stack.pop(L)
    if s0 is None or s1 is None:
        raise SpecError("TOO_SHORT")
    out = bytearray()

    def step(state):
        ns, sym, nb = dt[state]
        b = stack.pop(nb)
        if b is None:
            return None
        return (ns + b) & 0xFFFF, sym

    while True:
        if raw_len is not None and len(out) + 2 == raw_len:
            out += bytes([dt[s0][1], dt[s1][1]])
            break
        if raw_len is not None and len(out) + 1 == raw_len:
            out.append(dt[s0][1])
            break
        r = step(s0)
        if r is None:
            out += bytes([dt[s0][1], dt[s1][1]])
            break
        s0 = r[0]
        out.append(r[1])
        r = step(s1)
        if r is None:
            out += bytes([dt[s1][1], dt[s0][1]])
            break
        s1 = r[0]
        out.append(r[1])
    return bytes(out)


def decompress_headerless(norm, L, tl, payload: bytes) -> bytes:
    """The crate's test-module fse_decompress (fse.rs:424-434): the table from
    the caller's NormHistogram, then the lib.rs:187-211 loop."""
    stack = Stack(payload)
    dt = decode_table(norm, L, tl)
    if _single_symbol(norm, L):
        raise SpecError("SINGLE_SYMBOL")
    st = stack.pop(L)
    if st is None:
        raise SpecError("TOO_SHORT")
    out = bytearray()
    while True:
        ns, sym, nb = dt[st]
        b = stack.pop(nb)
        if b is None:
            break
        st = (ns + b) & 0xFFFF
        out.append(sym)
    out.append(dt[st][1])
    return bytes(out)


def decompress(data: bytes) -> bytes:
    """fse_decompress, one state (lib.rs:187-211)."""
    norm, L, tl, used = header_read(data)
    return decompress_headerless(norm, L, tl, data[used:])


# ---------------------------------------------------------------- generators
GOLDEN = 0x9E3779B97F4A7C15
M64 = (1 << 64) - 1


def splitmix64_mix(z: int) -> int:
    z &= M64
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & M64
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & M64
    return z ^ (z >> 31)


def build_lut(prob: float) -> bytes:
    """gen_sequence LUT (benches/fse_benchmark.rs:5-20)."""
    prob = min(max(prob, 0.005), 0.995)
    lut = bytearray()
    remaining, s = 4096, 0
    while remaining > 0:
        n = max(int(remaining * prob), 1)
        lut += bytes([s]) * n
        s = (s + 1) & 0xFF
        remaining -= n
    return bytes(lut)


def generate(kind: int, prob: float, seed: int, block_index: int, n: int) -> bytes:
    """Counter-based synthetic generator (same definition as fo_generate)."""
    lut = build_lut(prob) if kind == 0 else None
    sb = (seed ^ (block_index * GOLDEN)) & M64
    out = bytearray(n)
    for i in range(n):
        r = splitmix64_mix(sb + (i + 1) * GOLDEN)
        if kind == 0:
            out[i] = lut[r & 4095]
        elif kind == 1:
            x = r | (1 << 63)
            out[i] = min((x & -x).bit_length() - 1, 255)
        else:
            out[i] = ((r >> 32) * 240) >> 32
    return bytes(out)
