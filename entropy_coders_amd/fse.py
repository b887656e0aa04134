"""Python mirror of the reference crate's API for this path (tests, bench).

Reference-shaped calls (host bytes in, bytes out; lib.rs:146-248,
histogram.rs:18-66) and a batched device codec over torch tensors.  All
compute goes through libfsehip.so on the GPU.
"""
from __future__ import annotations

import ctypes as C
import threading

import numpy as np

from ._lib import (BitStackReaderState, BitStackWriterState, BitStreamReaderState, DecodeTable, EncodeTable, FseError,
                   Histogram, NormHistogram, Params, check, load)


def _buf(data) -> np.ndarray:
    if isinstance(data, np.ndarray):
        return np.ascontiguousarray(data, dtype=np.uint8)
    return np.frombuffer(bytes(data), dtype=np.uint8)


def _p(a: np.ndarray):
    return a.ctypes.data_as(C.c_void_p)


_tls = threading.local()


def _out(cap: int) -> np.ndarray:
    """A per-thread output buffer of >= cap bytes, reused across calls (the
    calls return copies): allocating a fresh 16 MiB array per call costs
    more than a small decode."""
    b = getattr(_tls, "out", None)
    if b is None or len(b) < cap:
        b = np.empty(max(cap, 1), dtype=np.uint8)
        _tls.out = b
    return b


def compress2(src) -> tuple[bytes, int]:
    """`fse_compress2(src, &mut dst) -> usize` (lib.rs:146): (bytes, payload bits)."""
    a = _buf(src)
    lib = load()
    cap = int(lib.fsehip_slot_bytes(max(len(a), 16), 12))
    dst = _out(cap)
    n = C.c_size_t(0)
    bits = C.c_uint64(0)
    check(lib.fse_compress2(_p(a), len(a), _p(dst), cap, C.byref(n), C.byref(bits)), "fse_compress2")
    return dst[: n.value].tobytes(), bits.value


def compress2_log(src, table_log: int) -> tuple[bytes, int]:
    """`Histogram::new(src).normalize(L)` + fse_compress2 body (histogram.rs:95)."""
    a = _buf(src)
    lib = load()
    cap = int(lib.fsehip_slot_bytes(max(len(a), 16), 12))
    dst = _out(cap)
    n = C.c_size_t(0)
    bits = C.c_uint64(0)
    check(lib.fse_compress2_log(_p(a), len(a), table_log, _p(dst), cap, C.byref(n), C.byref(bits)),
          "fse_compress2_log")
    return dst[: n.value].tobytes(), bits.value


def decompress2(src, cap: int = 1 << 24) -> bytes:
    """`fse_decompress2(src, &mut dst) -> Option<usize>` (lib.rs:215)."""
    a = _buf(src)
    lib = load()
    dst = _out(cap)
    n = C.c_size_t(0)
    check(lib.fse_decompress2(_p(a), len(a), _p(dst), cap, C.byref(n)), "fse_decompress2")
    return dst[: n.value].tobytes()


def compress(src) -> tuple[bytes, int]:
    """`fse_compress(src, &mut dst) -> (NormHistogram, usize)` (lib.rs:112): the
    1-state format; (bytes, payload bits).  The header in the bytes is the
    returned NormHistogram."""
    a = _buf(src)
    lib = load()
    cap = int(lib.fsehip_slot_bytes(max(len(a), 16), 12))
    dst = _out(cap)
    n = C.c_size_t(0)
    bits = C.c_uint64(0)
    check(lib.fse_compress(_p(a), len(a), _p(dst), cap, C.byref(n), C.byref(bits)), "fse_compress")
    return dst[: n.value].tobytes(), bits.value


def decompress(src, cap: int = 1 << 24) -> bytes:
    """`fse_decompress(src, &mut dst) -> Option<usize>` (lib.rs:187)."""
    a = _buf(src)
    lib = load()
    dst = _out(cap)
    n = C.c_size_t(0)
    check(lib.fse_decompress(_p(a), len(a), _p(dst), cap, C.byref(n)), "fse_decompress")
    return dst[: n.value].tobytes()


def decompress2_many(streams, dst_stride: int, nstates: int = 2, raw: bool = False, dst=None):
    """`fse_decompress2_many` / `fse_decompress_many` (nstates 1): many crate
    streams from host memory in one call, each decoded as `fse_decompress2`
    (lib.rs:215) would within dst_stride bytes.  Returns a list with, per
    stream, its bytes or the name of its status; with raw=True the call's own
    outputs instead: (dst, lengths, statuses) as numpy arrays (dst may be
    passed in, n * dst_stride bytes, to reuse one buffer across calls)."""
    from ._lib import STATUS

    if nstates not in (1, 2):
        raise ValueError(f"nstates must be 1 or 2, not {nstates!r}")
    lib = load()
    bufs = [_buf(x) for x in streams]
    n = len(bufs)
    ptrs = np.array([b.ctypes.data if len(b) else 0 for b in bufs] or [0], dtype=np.uintp)
    lens = np.array([len(b) for b in bufs] or [0], dtype=np.uintp)
    if dst is None:
        dst = np.empty(max(n, 1) * dst_stride, dtype=np.uint8)
    elif not (isinstance(dst, np.ndarray) and dst.dtype == np.uint8 and dst.flags.c_contiguous
              and dst.flags.writeable and dst.nbytes >= n * dst_stride):
        # the C call writes n * dst_stride bytes through the raw pointer
        raise ValueError(f"dst must be a writeable C-contiguous uint8 ndarray of >= {n * dst_stride} bytes")
    out_lens = np.zeros(max(n, 1), dtype=np.uintp)
    st = np.zeros(max(n, 1), dtype=np.int32)
    fn = lib.fse_decompress2_many if nstates == 2 else lib.fse_decompress_many
    check(fn(_p(ptrs), _p(lens), n, _p(dst), dst_stride, _p(out_lens), _p(st)), "fse_decompress2_many")
    if raw:
        return dst, out_lens[:n], st[:n]
    return [dst[i * dst_stride: i * dst_stride + int(out_lens[i])].tobytes() if st[i] == 0 else
            STATUS.get(int(st[i]), str(int(st[i]))) for i in range(n)]


def decompress_streams(streams, out_stride: int, nstates: int = 2, max_table_log: int = 11, device=None):
    """`fsehip_decompress_streams`: many crate streams (no sidecar, no raw
    length) decoded at once on the GPU, each as `fse_decompress2` (nstates 2)
    or `fse_decompress` (1) would, within out_stride bytes.  Returns a list
    with, per stream, its bytes or the name of its status."""
    import torch

    from ._lib import STATUS

    dev = torch.device(device or "cuda")
    stride = max(512, (max((len(x) for x in streams), default=1) + 255) // 256 * 256)
    host = np.zeros(len(streams) * stride, dtype=np.uint8)
    for i, x in enumerate(streams):
        host[i * stride: i * stride + len(x)] = np.frombuffer(bytes(x), dtype=np.uint8)
    d_in = torch.from_numpy(host).to(dev)
    lens = torch.tensor([len(x) for x in streams], dtype=torch.int32, device=dev)
    out = torch.empty(len(streams) * out_stride, dtype=torch.uint8, device=dev)
    out_len = torch.zeros(len(streams), dtype=torch.int32, device=dev)
    status = torch.zeros(len(streams), dtype=torch.int32, device=dev)
    check(load().fsehip_decompress_streams(nstates, max_table_log, C.c_void_p(d_in.data_ptr()), stride,
                                           C.c_void_p(lens.data_ptr()), len(streams), C.c_void_p(out.data_ptr()),
                                           out_stride, C.c_void_p(out_len.data_ptr()),
                                           C.c_void_p(status.data_ptr()),
                                           C.c_void_p(torch.cuda.current_stream(dev).cuda_stream)),
          "fsehip_decompress_streams")
    torch.cuda.synchronize(dev)
    host_out, ol, st = out.cpu().numpy(), out_len.cpu().numpy(), status.cpu().numpy()
    return [host_out[i * out_stride: i * out_stride + int(ol[i])].tobytes() if st[i] == 0 else
            STATUS.get(int(st[i]), str(int(st[i]))) for i in range(len(streams))]


def histogram_count(src) -> tuple[np.ndarray, int]:
    """`Histogram::new(data)` (histogram.rs:18-66): (counts[256], table_len)."""
    a = _buf(src)
    lib = load()
    counts = np.zeros(256, dtype=np.uint32)
    tl = C.c_uint32(0)
    check(lib.histogram_count(_p(a), len(a), _p(counts), C.byref(tl)), "histogram_count")
    return counts, tl.value


# ---------------------------------------------------------------- building blocks
def histogram_new(src) -> Histogram:
    """`Histogram::new(data)` (histogram.rs:18-66)."""
    a = _buf(src)
    h = Histogram()
    check(load().histogram_new(_p(a), len(a), C.byref(h)), "histogram_new")
    return h


def normalize(h: Histogram, log2: int) -> NormHistogram:
    """`Histogram::normalize(log2)` (histogram.rs:95-155)."""
    nh = NormHistogram()
    check(load().histogram_normalize(C.byref(h), log2, C.byref(nh)), "histogram_normalize")
    return nh


def normalize_optimal(h: Histogram) -> NormHistogram:
    """`Histogram::normalize_optimal` (histogram.rs:281-284)."""
    nh = NormHistogram()
    check(load().histogram_normalize_optimal(C.byref(h), C.byref(nh)), "histogram_normalize_optimal")
    return nh


def norm_histogram_new(src) -> NormHistogram:
    """`NormHistogram::new(data)` (histogram.rs:299-303)."""
    a = _buf(src)
    nh = NormHistogram()
    check(load().norm_histogram_new(_p(a), len(a), C.byref(nh)), "norm_histogram_new")
    return nh


def norm_histogram_write(nh: NormHistogram) -> tuple[bytes, int]:
    """`NormHistogram::write(&mut Vec)` (histogram.rs:376-431): (bytes, bits written)."""
    dst = np.zeros(1024, dtype=np.uint8)
    n = C.c_size_t(0)
    bits = C.c_uint64(0)
    check(load().norm_histogram_write(C.byref(nh), _p(dst), len(dst), C.byref(n), C.byref(bits)),
          "norm_histogram_write")
    return dst[: n.value].tobytes(), bits.value


def norm_histogram_read(data) -> tuple[NormHistogram, int]:
    """`NormHistogram::read(slice)` (histogram.rs:436-505): (histogram, bytes consumed)."""
    a = _buf(data)
    nh = NormHistogram()
    used = C.c_size_t(0)
    check(load().norm_histogram_read(_p(a), len(a), C.byref(nh), C.byref(used)), "norm_histogram_read")
    return nh, used.value


def encode_table_new(nh: NormHistogram) -> EncodeTable:
    """`EncodeTable::new(&hist)` (fse.rs:88-189) as plain data."""
    t = EncodeTable()
    check(load().encode_table_new(C.byref(nh), C.byref(t)), "encode_table_new")
    return t


def decode_table_new(nh: NormHistogram) -> DecodeTable:
    """`DecodeTable::new(&hist)` (fse.rs:269-338) as plain data."""
    t = DecodeTable()
    check(load().decode_table_new(C.byref(nh), C.byref(t)), "decode_table_new")
    return t


def compress_nh(src) -> tuple[bytes, int, NormHistogram]:
    """`fse_compress(src, &mut dst) -> (NormHistogram, usize)` (lib.rs:112) with
    the histogram returned: (bytes, payload bits, NormHistogram)."""
    a = _buf(src)
    lib = load()
    cap = int(lib.fsehip_slot_bytes(max(len(a), 16), 12))
    dst = _out(cap)
    n = C.c_size_t(0)
    bits = C.c_uint64(0)
    nh = NormHistogram()
    check(lib.fse_compress_nh(_p(a), len(a), _p(dst), cap, C.byref(n), C.byref(bits), C.byref(nh)), "fse_compress_nh")
    return dst[: n.value].tobytes(), bits.value, nh


# ---------------------------------------------------------------- bitstream
def bitstack_write(vals, widths, prefix: bytes = b"") -> tuple[bytes, int]:
    """BitStackWriter::new(&mut vec) over a vec holding `prefix`, then
    write_bits_unmasked per field + finish (writer.rs:14-222): (the vec's
    bytes, bits written)."""
    v = np.ascontiguousarray(vals, dtype=np.uint32)
    w = np.ascontiguousarray(widths, dtype=np.uint8)
    cap = len(prefix) + len(v) * 4 + 16
    dst = np.zeros(cap, dtype=np.uint8)
    dst[: len(prefix)] = np.frombuffer(bytes(prefix), dtype=np.uint8)
    n = C.c_size_t(len(prefix))
    bits = C.c_uint64(0)
    check(load().bitstack_write(_p(v), _p(w), len(v), _p(dst), cap, C.byref(n), C.byref(bits)), "bitstack_write")
    return dst[: n.value].tobytes(), bits.value


def bitstack_read(data, widths) -> tuple[list, int, bool]:
    """BitStackReader::new + read(width) per field, top down (stack_reader.rs):
    (values read, number of successful reads, finish())."""
    a = _buf(data)
    w = np.ascontiguousarray(widths, dtype=np.uint8)
    out = np.zeros(max(len(w), 1), dtype=np.uint32)
    nr = C.c_size_t(0)
    fin = C.c_int(0)
    check(load().bitstack_read(_p(a), len(a), _p(w), len(w), _p(out), C.byref(nr), C.byref(fin)), "bitstack_read")
    return [int(x) for x in out[: nr.value]], nr.value, bool(fin.value)


EOF_STATUS = -18  # FSE_ERR_EOF: the reference's None / Err(UnexpectedEof)


class BitStackReader:
    """BitStackReader (stack_reader.rs:5-227) over the C-ABI cursor
    (fsehip.h section 1c): one O(1) call per method.  `peek` / `read` /
    `read_no_reload` return None where the crate returns None."""

    def __init__(self, data):
        self._buf = _buf(data)  # the cursor points into this buffer
        self.state = BitStackReaderState()
        self._lib = load()
        check(self._lib.bitstack_reader_new(C.byref(self.state), _p(self._buf), len(self._buf)),
              "BitStackReader::new")

    def _val(self, fn, nbits):
        v = C.c_uint32(0)
        rc = fn(C.byref(self.state), nbits, C.byref(v))
        if rc == EOF_STATUS:
            return None
        check(rc, fn.__name__)
        return v.value

    def peek(self, nbits: int):
        return self._val(self._lib.bitstack_reader_peek, nbits)

    def read(self, nbits: int):
        return self._val(self._lib.bitstack_reader_read, nbits)

    def read_no_reload(self, nbits: int):
        return self._val(self._lib.bitstack_reader_read_no_reload, nbits)

    def advance_no_reload(self, nbits: int) -> None:
        check(self._lib.bitstack_reader_advance_no_reload(C.byref(self.state), nbits), "advance_no_reload")

    def reload(self) -> None:
        check(self._lib.bitstack_reader_reload(C.byref(self.state)), "reload")

    def available(self) -> int:
        return int(self._lib.bitstack_reader_available(C.byref(self.state)))

    def finish(self) -> bool:
        return bool(self._lib.bitstack_reader_finish(C.byref(self.state)))


class BitStreamReader:
    """BitStreamReader (stream_reader.rs:5-136) over the C-ABI cursor.
    `peek` / `read` / `advance_by` raise EOFError where the crate returns
    Err(UnexpectedEof)."""

    def __init__(self, data, total_bits: int):
        self._buf = _buf(data)
        self.state = BitStreamReaderState()
        self._lib = load()
        check(self._lib.bitstream_reader_new(C.byref(self.state), _p(self._buf), len(self._buf), total_bits),
              "BitStreamReader::new")

    def _rc(self, rc: int, what: str) -> None:
        if rc == EOF_STATUS:
            raise EOFError(what)
        check(rc, what)

    def peek(self, nbits: int) -> int:
        v = C.c_uint32(0)
        self._rc(self._lib.bitstream_reader_peek(C.byref(self.state), nbits, C.byref(v)), "peek")
        return v.value

    def read(self, nbits: int) -> int:
        v = C.c_uint32(0)
        self._rc(self._lib.bitstream_reader_read(C.byref(self.state), nbits, C.byref(v)), "read")
        return v.value

    def advance_by(self, nbits: int) -> None:
        self._rc(self._lib.bitstream_reader_advance_by(C.byref(self.state), nbits), "advance_by")

    def available(self) -> int:
        return int(self._lib.bitstream_reader_available(C.byref(self.state)))

    def finish(self) -> tuple[bytes, int, int]:
        b, rem, off = C.c_size_t(0), C.c_uint64(0), C.c_uint32(0)
        check(self._lib.bitstream_reader_finish(C.byref(self.state), C.byref(b), C.byref(rem), C.byref(off)), "finish")
        return self._buf[b.value:].tobytes(), rem.value, off.value

    def finish_byte(self) -> bytes:
        return self._buf[int(self._lib.bitstream_reader_finish_byte(C.byref(self.state))):].tobytes()


class BitStackWriter:
    """BitStackWriter (writer.rs:5-223) appending to a buffer that holds
    `prefix`, over the C-ABI cursor; `finish()` returns (the buffer's bytes,
    bits written)."""

    def __init__(self, prefix: bytes = b"", cap: int = 1 << 16):
        self._dst = np.zeros(len(prefix) + cap, dtype=np.uint8)
        self._dst[: len(prefix)] = np.frombuffer(bytes(prefix), dtype=np.uint8)
        self.state = BitStackWriterState()
        self._lib = load()
        check(self._lib.bitstack_writer_new(C.byref(self.state), _p(self._dst), len(self._dst), len(prefix)),
              "BitStackWriter::new")

    def write_bits(self, val: int, nbits: int) -> None:
        check(self._lib.bitstack_writer_write_bits(C.byref(self.state), val, nbits), "write_bits")

    def write_bits_unmasked(self, val: int, nbits: int) -> None:
        check(self._lib.bitstack_writer_write_bits_unmasked(C.byref(self.state), val, nbits), "write_bits_unmasked")

    def write_bits_raw(self, val: int, nbits: int) -> None:
        check(self._lib.bitstack_writer_write_bits_raw(C.byref(self.state), val, nbits), "write_bits_raw")

    def write_bits_raw_unmasked(self, val: int, nbits: int) -> None:
        check(self._lib.bitstack_writer_write_bits_raw_unmasked(C.byref(self.state), val, nbits),
              "write_bits_raw_unmasked")

    def flush(self) -> None:
        check(self._lib.bitstack_writer_flush(C.byref(self.state)), "flush")

    def finish(self) -> tuple[bytes, int]:
        n, bits = C.c_size_t(0), C.c_uint64(0)
        check(self._lib.bitstack_writer_finish(C.byref(self.state), C.byref(n), C.byref(bits)), "finish")
        return self._dst[: n.value].tobytes(), bits.value


BITS_READ, BITS_PEEK, BITS_ADVANCE = 0, 1, 2  # FSE_BITS_* (include/fsehip.h)


def bitstream_read(data, total_bits: int, widths, ops=None) -> tuple[list, int, int]:
    """BitStreamReader::new(slice, total_bits) and one call per field
    (stream_reader.rs:56-119): read(width), or with `ops` peek(width)
    (BITS_PEEK) / advance_by(width) (BITS_ADVANCE, value 0).  Returns (values
    of the steps that returned Ok, their number, available() after them)."""
    a = _buf(data)
    w = np.ascontiguousarray(widths, dtype=np.uint8)
    out = np.zeros(max(len(w), 1), dtype=np.uint32)
    nr = C.c_size_t(0)
    left = C.c_uint64(0)
    if ops is None:
        check(load().bitstream_read(_p(a), len(a), total_bits, _p(w), len(w), _p(out), C.byref(nr), C.byref(left)),
              "bitstream_read")
    else:
        o = np.ascontiguousarray(ops, dtype=np.uint8)
        if len(o) != len(w):
            raise ValueError("one op per field")
        check(load().bitstream_read_ops(_p(a), len(a), total_bits, _p(w), _p(o), len(w), _p(out), C.byref(nr),
                                        C.byref(left)), "bitstream_read_ops")
    return [int(x) for x in out[: nr.value]], nr.value, left.value


class BlockCodec:
    """Batched device codec: 64 KiB blocks (configurable) over torch tensors.

    compress(src) -> CompressedBlocks (slots, lengths, sidecar, status), all
    resident on the device; decompress(cb) -> uint8 tensor.  Work is queued
    on torch's current stream.
    """

    def __init__(self, block_size: int = 65536, table_log: int = 0, ckpt_interval: int = 128,
                 device=None, nstates: int = 2):
        import torch

        self.torch = torch
        self.device = torch.device(device or "cuda")
        self.block_size = block_size
        self.table_log = table_log
        self.ckpt_interval = ckpt_interval
        self.nstates = nstates  # 2: fse_compress2 blocks (lib.rs:146), 1: fse_compress (lib.rs:112)
        self.max_table_log = max(11, table_log) if table_log else 11
        self.lib = load()
        self.slot_bytes = int(self.lib.fsehip_slot_bytes(block_size, self.max_table_log))
        self.side_per_block = int(self.lib.fsehip_sidecar_per_block_ns(block_size, ckpt_interval, nstates))

    def params(self) -> Params:
        return Params(self.block_size, self.table_log, self.ckpt_interval, self.max_table_log, self.nstates)

    def _stream(self):
        return C.c_void_p(self.torch.cuda.current_stream(self.device).cuda_stream)

    def release_workspace(self) -> None:
        """`fsehip_release_workspace` for this codec's device and torch's
        current stream: frees the decode workspace (decode tables, and the
        deferred-symbol states: 2 bytes per output byte of the last
        sidecar-less batch) after the queued work."""
        check(self.lib.fsehip_release_workspace(self.device.index if self.device.index is not None else
                                                self.torch.cuda.current_device(), self._stream()),
              "fsehip_release_workspace")

    def rank_fallbacks(self, reset: bool = False) -> dict:
        """`fsehip_rank_fallbacks` on this codec's device: tables whose atomic
        ranks failed their self-check and were rebuilt with peer-mask ranks
        (batch encoder, decode-table builds, building-block table calls)."""
        import ctypes as C

        out = (C.c_uint32 * 3)()
        dev = self.device.index if self.device.index is not None else self.torch.cuda.current_device()
        check(self.lib.fsehip_rank_fallbacks(dev, C.byref(out), 1 if reset else 0), "fsehip_rank_fallbacks")
        return {"encode": int(out[0]), "decode_tables": int(out[1]), "table_calls": int(out[2])}

    def n_blocks(self, n_total: int) -> int:
        return (n_total + self.block_size - 1) // self.block_size

    def alloc(self, n_total: int) -> dict:
        t = self.torch
        nb = self.n_blocks(n_total)
        return {
            "n_total": n_total,
            "out": t.empty(nb * self.slot_bytes, dtype=t.uint8, device=self.device),
            "comp_len": t.zeros(nb, dtype=t.int32, device=self.device),
            "payload_bits": t.zeros(nb, dtype=t.int32, device=self.device),
            "sidecar": t.zeros(max(nb * self.side_per_block, 1), dtype=t.int64, device=self.device),
            "status": t.zeros(nb, dtype=t.int32, device=self.device),
        }

    def compress_into(self, src, cb: dict) -> None:
        p = self.params()
        rc = self.lib.fsehip_compress_blocks(
            C.byref(p), C.c_void_p(src.data_ptr()), cb["n_total"], C.c_void_p(cb["out"].data_ptr()),
            self.slot_bytes, C.c_void_p(cb["comp_len"].data_ptr()),
            C.c_void_p(cb["payload_bits"].data_ptr()),
            C.c_void_p(cb["sidecar"].data_ptr()) if self.ckpt_interval else None,
            C.c_void_p(cb["status"].data_ptr()), self._stream())
        check(rc, "fsehip_compress_blocks")

    def compress(self, src) -> dict:
        cb = self.alloc(src.numel())
        self.compress_into(src, cb)
        return cb

    def decompress_into(self, cb: dict, out, status, use_sidecar: bool = True) -> None:
        p = self.params()
        side = C.c_void_p(cb["sidecar"].data_ptr()) if (use_sidecar and self.ckpt_interval) else None
        rc = self.lib.fsehip_decompress_blocks(
            C.byref(p), C.c_void_p(cb["out"].data_ptr()), self.slot_bytes,
            C.c_void_p(cb["comp_len"].data_ptr()), side, C.c_void_p(out.data_ptr()), cb["n_total"],
            C.c_void_p(status.data_ptr()), self._stream())
        check(rc, "fsehip_decompress_blocks")

    def decompress(self, cb: dict, use_sidecar: bool = True):
        t = self.torch
        out = t.empty(cb["n_total"], dtype=t.uint8, device=self.device)
        status = t.zeros(self.n_blocks(cb["n_total"]), dtype=t.int32, device=self.device)
        self.decompress_into(cb, out, status, use_sidecar)
        return out, status

    def build_sidecar(self, cb: dict):
        """`fsehip_build_sidecar`: decode blocks that carry no sidecar (e.g.
        from the CPU crate) and record their sidecar.  Returns (out, sidecar,
        status) device tensors."""
        t = self.torch
        nb = self.n_blocks(cb["n_total"])
        out = t.empty(cb["n_total"], dtype=t.uint8, device=self.device)
        side = t.zeros(max(nb * self.side_per_block, 1), dtype=t.int64, device=self.device)
        status = t.zeros(nb, dtype=t.int32, device=self.device)
        p = self.params()
        check(self.lib.fsehip_build_sidecar(
            C.byref(p), C.c_void_p(cb["out"].data_ptr()), self.slot_bytes, C.c_void_p(cb["comp_len"].data_ptr()),
            C.c_void_p(out.data_ptr()), cb["n_total"], C.c_void_p(side.data_ptr()), C.c_void_p(status.data_ptr()),
            self._stream()), "fsehip_build_sidecar")
        return out, side, status

    def build_dtables(self, cb: dict) -> dict:
        """Decode tables for every block of `cb` (fsehip_build_dtables): the
        pre-built tables of decode-only workloads (C3)."""
        t = self.torch
        nb = self.n_blocks(cb["n_total"])
        per = int(self.lib.fsehip_dtable_bytes(self.max_table_log))
        tabs = {"dt": t.empty(nb * per // 4, dtype=t.int32, device=self.device),
                "info": t.empty(nb, dtype=t.int32, device=self.device)}
        self.build_dtables_into(cb, tabs)
        return tabs

    def build_dtables_into(self, cb: dict, tabs: dict) -> None:
        p = self.params()
        check(self.lib.fsehip_build_dtables(
            C.byref(p), C.c_void_p(cb["out"].data_ptr()), self.slot_bytes, C.c_void_p(cb["comp_len"].data_ptr()),
            self.n_blocks(cb["n_total"]), C.c_void_p(tabs["dt"].data_ptr()), C.c_void_p(tabs["info"].data_ptr()),
            self._stream()), "fsehip_build_dtables")

    def decompress_dt_into(self, cb: dict, tabs: dict, out, status, use_sidecar: bool = True) -> None:
        """Decode with pre-built tables (2-state needs the sidecar; 1-state
        without one runs the serial reference-order decoder)."""
        p = self.params()
        side = C.c_void_p(cb["sidecar"].data_ptr()) if (use_sidecar and self.ckpt_interval) else None
        check(self.lib.fsehip_decompress_blocks_dt(
            C.byref(p), C.c_void_p(cb["out"].data_ptr()), self.slot_bytes, C.c_void_p(cb["comp_len"].data_ptr()),
            side, C.c_void_p(tabs["dt"].data_ptr()),
            C.c_void_p(tabs["info"].data_ptr()), C.c_void_p(out.data_ptr()), cb["n_total"],
            C.c_void_p(status.data_ptr()), self._stream()), "fsehip_decompress_blocks_dt")

    def generate(self, kind: int, prob: float, seed: int, n_total: int):
        t = self.torch
        out = t.empty(n_total, dtype=t.uint8, device=self.device)
        check(self.lib.fsehip_generate(kind, prob, seed, self.block_size, C.c_void_p(out.data_ptr()),
                                       n_total, self._stream()), "fsehip_generate")
        return out

    def block_bytes(self, cb: dict, b: int) -> bytes:
        """Compressed bytes of block b (host copy) -- for parity checks."""
        ln = int(cb["comp_len"][b].item())
        s = b * self.slot_bytes
        return cb["out"][s: s + ln].cpu().numpy().tobytes()


__all__ = ["BITS_ADVANCE", "BITS_PEEK", "BITS_READ", "BitStackReader", "BitStackWriter", "BitStreamReader", "BlockCodec", "DecodeTable", "EncodeTable", "FseError",
           "Histogram", "NormHistogram", "bitstack_read", "bitstack_write", "bitstream_read", "compress", "compress2",
           "compress2_log", "compress_nh", "decode_table_new", "decompress", "decompress2", "decompress2_many",
           "decompress_streams",
           "encode_table_new",
           "histogram_count", "histogram_new", "norm_histogram_new", "norm_histogram_read", "norm_histogram_write",
           "normalize", "normalize_optimal"]
