"""ctypes binding of the C parity oracle (oracle/libfseoracle.so).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg, never by the product package.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "libfseoracle.so")

STATUS = {
    0: "OK", -1: "EMPTY", -2: "TOO_SHORT", -3: "ALL_ZERO_SYMBOL0", -4: "SINGLE_SYMBOL",
    -5: "BAD_HEADER", -6: "NO_MARKER", -7: "DST_TOO_SMALL", -8: "TABLELOG_RANGE",
    -9: "CURSED", -10: "BAD_TABLE", -11: "BAD_ARG", -12: "HIP", -13: "LENGTH_MISMATCH",
    -14: "UNSUPPORTED", -15: "NO_DEVICE", -16: "BAD_SIDECAR", -17: "ENCODER_INIT",
}


class OracleError(Exception):
    def __init__(self, rc: int):
        super().__init__(f"oracle status {rc} ({STATUS.get(rc, '?')})")
        self.rc = rc
        self.code = STATUS.get(rc, str(rc))


class Norm(C.Structure):
    _fields_ = [("norm", C.c_int32 * 256), ("log2", C.c_uint32), ("table_len", C.c_uint32)]


class Hist(C.Structure):
    _fields_ = [("counts", C.c_uint32 * 256), ("size", C.c_uint32), ("table_len", C.c_uint32)]


class CTable(C.Structure):
    _fields_ = [("log2", C.c_uint32), ("st", C.c_uint16 * 32768), ("dnb", C.c_uint32 * 256),
                ("dfs", C.c_int32 * 256), ("spread", C.c_uint8 * 32768)]


class DTable(C.Structure):
    _fields_ = [("log2", C.c_uint32), ("new_state", C.c_uint16 * 32768),
                ("sym", C.c_uint8 * 32768), ("nb", C.c_uint8 * 32768)]


_lib = None


def build() -> None:
    subprocess.run(["make", "-s", "-C", HERE], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        _lib = C.CDLL(LIB_PATH)
        P = C.c_void_p
        sz = C.c_size_t
        _lib.fo_generate.argtypes = [C.c_int, C.c_double, C.c_uint64, C.c_uint64, P, sz]
        _lib.fo_generate.restype = None
        for name in ("fo_compress2", "fo_compress"):
            getattr(_lib, name).argtypes = [P, sz, P, sz, C.POINTER(sz), C.POINTER(C.c_uint64)]
        _lib.fo_compress2_log.argtypes = [P, sz, C.c_uint32, P, sz, C.POINTER(sz),
                                          C.POINTER(C.c_uint64)]
        for name in ("fo_decompress2", "fo_decompress"):
            getattr(_lib, name).argtypes = [P, sz, P, sz, C.POINTER(sz)]
        _lib.fo_decompress2_n.argtypes = [P, sz, P, sz]
        _lib.fo_hist_count.argtypes = [P, sz, C.POINTER(Hist)]
        _lib.fo_optimal_log2.argtypes = [C.POINTER(Hist), C.POINTER(C.c_uint32)]
        _lib.fo_normalize.argtypes = [C.POINTER(Hist), C.c_uint32, C.POINTER(Norm),
                                      C.POINTER(C.c_int)]
        _lib.fo_norm_new.argtypes = [P, sz, C.POINTER(Norm)]
        _lib.fo_header_write.argtypes = [C.POINTER(Norm), P, sz, C.POINTER(sz)]
        _lib.fo_header_read.argtypes = [P, sz, C.POINTER(Norm), C.POINTER(sz)]
        _lib.fo_build_ctable.argtypes = [C.POINTER(Norm), C.POINTER(CTable)]
        _lib.fo_build_dtable.argtypes = [C.POINTER(Norm), C.POINTER(DTable)]
        _lib.fo_checkpoints2.argtypes = [P, sz, C.c_uint32, P, P, P, sz, C.POINTER(sz)]
        _lib.fo_checkpoints1.argtypes = [P, sz, C.c_uint32, P, P, sz, C.POINTER(sz)]
        _lib.fo_bits_write.argtypes = [P, P, sz, C.c_int, P, sz, C.POINTER(C.c_uint64)]
        _lib.fo_bits_write.restype = sz
        _lib.fo_bits_read_stack.argtypes = [P, sz, P, sz, P, C.POINTER(sz)]
        _lib.fo_compress2_blocks.argtypes = [P, sz, sz, P, sz, P, C.c_int]
        _lib.fo_decompress2_blocks.argtypes = [P, sz, P, sz, P, sz, sz, C.c_int]
    return _lib


def _ptr(a: np.ndarray):
    return a.ctypes.data_as(C.c_void_p)


def _u8(b) -> np.ndarray:
    return np.frombuffer(bytes(b), dtype=np.uint8).copy() if not isinstance(b, np.ndarray) else b


def _check(rc: int):
    if rc != 0:
        raise OracleError(rc)


def generate(kind: int, prob: float, seed: int, block_index: int, n: int) -> np.ndarray:
    out = np.empty(n, dtype=np.uint8)
    lib().fo_generate(kind, prob, seed, block_index, _ptr(out), n)
    return out


def compress_bound(n: int) -> int:
    """Worst case is L=15 bits per symbol plus a 512-byte header bound."""
    return 512 + (n * 15 + 7) // 8 + 16


def compress2(src, log2: int | None = None) -> tuple[bytes, int]:
    a = _u8(src)
    cap = compress_bound(len(a))
    dst = np.zeros(cap, dtype=np.uint8)
    out_len = C.c_size_t(0)
    bits = C.c_uint64(0)
    if log2 is None:
        rc = lib().fo_compress2(_ptr(a), len(a), _ptr(dst), cap, C.byref(out_len), C.byref(bits))
    else:
        rc = lib().fo_compress2_log(_ptr(a), len(a), log2, _ptr(dst), cap, C.byref(out_len),
                                    C.byref(bits))
    _check(rc)
    return dst[: out_len.value].tobytes(), bits.value


def compress(src) -> tuple[bytes, int]:
    a = _u8(src)
    cap = compress_bound(len(a))
    dst = np.zeros(cap, dtype=np.uint8)
    out_len = C.c_size_t(0)
    bits = C.c_uint64(0)
    _check(lib().fo_compress(_ptr(a), len(a), _ptr(dst), cap, C.byref(out_len), C.byref(bits)))
    return dst[: out_len.value].tobytes(), bits.value


def decompress2(data, cap: int = 1 << 22, raw_len: int | None = None) -> bytes:
    a = _u8(data)
    if raw_len is not None:
        dst = np.zeros(max(raw_len, 1), dtype=np.uint8)
        _check(lib().fo_decompress2_n(_ptr(a), len(a), _ptr(dst), raw_len))
        return dst[:raw_len].tobytes()
    dst = np.zeros(cap, dtype=np.uint8)
    out_len = C.c_size_t(0)
    _check(lib().fo_decompress2(_ptr(a), len(a), _ptr(dst), cap, C.byref(out_len)))
    return dst[: out_len.value].tobytes()


def decompress(data, cap: int = 1 << 22) -> bytes:
    a = _u8(data)
    dst = np.zeros(cap, dtype=np.uint8)
    out_len = C.c_size_t(0)
    _check(lib().fo_decompress(_ptr(a), len(a), _ptr(dst), cap, C.byref(out_len)))
    return dst[: out_len.value].tobytes()


def hist_count(src) -> Hist:
    a = _u8(src)
    h = Hist()
    _check(lib().fo_hist_count(_ptr(a), len(a), C.byref(h)))
    return h


def optimal_log2(h: Hist) -> int:
    L = C.c_uint32(0)
    _check(lib().fo_optimal_log2(C.byref(h), C.byref(L)))
    return L.value


def normalize(h: Hist, log2: int) -> tuple[Norm, bool]:
    nh = Norm()
    slow = C.c_int(0)
    _check(lib().fo_normalize(C.byref(h), log2, C.byref(nh), C.byref(slow)))
    return nh, bool(slow.value)


def norm_new(src) -> Norm:
    """NormHistogram::new (histogram.rs:299-303)."""
    a = _u8(src)
    nh = Norm()
    _check(lib().fo_norm_new(_ptr(a), len(a), C.byref(nh)))
    return nh


def ctable(nh: Norm):
    """EncodeTable::new (fse.rs:88-189): (log2, stateTable, deltaNbBits[256],
    deltaFindState[256], spread symbols)."""
    ct = CTable()
    _check(lib().fo_build_ctable(C.byref(nh), C.byref(ct)))
    size = 1 << ct.log2
    return (ct.log2, np.ctypeslib.as_array(ct.st)[:size].copy(), np.ctypeslib.as_array(ct.dnb).copy(),
            np.ctypeslib.as_array(ct.dfs).copy(), np.ctypeslib.as_array(ct.spread)[:size].copy())


def dtable_nh(nh: Norm):
    """DecodeTable::new (fse.rs:269-338): (log2, new_state[], sym[], nb[])."""
    dt = DTable()
    _check(lib().fo_build_dtable(C.byref(nh), C.byref(dt)))
    size = 1 << dt.log2
    return (dt.log2, np.ctypeslib.as_array(dt.new_state)[:size].copy(),
            np.ctypeslib.as_array(dt.sym)[:size].copy(), np.ctypeslib.as_array(dt.nb)[:size].copy())


def header_write(nh: Norm) -> bytes:
    dst = np.zeros(1024, dtype=np.uint8)
    n = C.c_size_t(0)
    _check(lib().fo_header_write(C.byref(nh), _ptr(dst), 1024, C.byref(n)))
    return dst[: n.value].tobytes()


def header_read(data) -> tuple[Norm, int]:
    a = _u8(data)
    nh = Norm()
    used = C.c_size_t(0)
    _check(lib().fo_header_read(_ptr(a), len(a), C.byref(nh), C.byref(used)))
    return nh, used.value


def dtable(data):
    """Decode table of a compressed block (NormHistogram::read +
    DecodeTable::new): (log2, new_state[], sym[], nb[], header_bytes)."""
    nh, used = header_read(data)
    dt = DTable()
    _check(lib().fo_build_dtable(C.byref(nh), C.byref(dt)))
    size = 1 << dt.log2
    return (dt.log2, np.ctypeslib.as_array(dt.new_state)[:size].copy(),
            np.ctypeslib.as_array(dt.sym)[:size].copy(), np.ctypeslib.as_array(dt.nb)[:size].copy(), used)


def checkpoints1(data, interval: int):
    """1-state decode checkpoints: (bitpos, state) before symbol p, every interval."""
    a = _u8(data)
    cap = 1 << 20
    bp = np.zeros(cap, np.uint32)
    s0 = np.zeros(cap, np.uint16)
    cnt = C.c_size_t(0)
    _check(lib().fo_checkpoints1(_ptr(a), len(a), interval, _ptr(bp), _ptr(s0), cap, C.byref(cnt)))
    return bp[: cnt.value], s0[: cnt.value]


def checkpoints2(data, interval: int):
    a = _u8(data)
    cap = 1 << 20
    bp = np.zeros(cap, np.uint32)
    s0 = np.zeros(cap, np.uint16)
    s1 = np.zeros(cap, np.uint16)
    cnt = C.c_size_t(0)
    _check(lib().fo_checkpoints2(_ptr(a), len(a), interval, _ptr(bp), _ptr(s0), _ptr(s1), cap,
                                 C.byref(cnt)))
    c = cnt.value
    return bp[:c].copy(), s0[:c].copy(), s1[:c].copy()


def bits_write(vals, widths, mark: bool) -> tuple[bytes, int]:
    v = np.asarray(vals, dtype=np.uint64)
    w = np.asarray(widths, dtype=np.uint8)
    cap = (int(w.sum()) + 8) // 8 + 8
    dst = np.zeros(cap, dtype=np.uint8)
    wb = C.c_uint64(0)
    n = lib().fo_bits_write(_ptr(v), _ptr(w), len(v), int(mark), _ptr(dst), cap, C.byref(wb))
    return dst[:n].tobytes(), wb.value


def bits_read_stack(data, widths) -> tuple[list[int], int]:
    a = _u8(data)
    w = np.asarray(widths, dtype=np.uint8)
    out = np.zeros(len(w), dtype=np.uint64)
    left = C.c_size_t(0)
    _check(lib().fo_bits_read_stack(_ptr(a), len(a), _ptr(w), len(w), _ptr(out), C.byref(left)))
    return [int(x) for x in out], left.value


def compress2_blocks(src: np.ndarray, block: int, threads: int, dst: np.ndarray = None, lens: np.ndarray = None):
    """`dst` / `lens`: reused output buffers (already faulted in), or None."""
    n_blocks = (len(src) + block - 1) // block
    slot = compress_bound(block)
    if dst is None:
        dst = np.empty(n_blocks * slot, dtype=np.uint8)
    if lens is None:
        lens = np.zeros(n_blocks, dtype=np.uint32)
    assert len(dst) >= n_blocks * slot and len(lens) >= n_blocks
    _check(lib().fo_compress2_blocks(_ptr(src), len(src), block, _ptr(dst), slot, _ptr(lens),
                                     threads))
    return dst, lens, slot


def decompress2_blocks(comp: np.ndarray, slot: int, lens: np.ndarray, block: int, n_total: int,
                       threads: int, out: np.ndarray = None) -> np.ndarray:
    if out is None:
        out = np.empty(n_total, dtype=np.uint8)
    assert len(out) >= n_total
    _check(lib().fo_decompress2_blocks(_ptr(comp), slot, _ptr(lens), len(lens), _ptr(out), block,
                                       n_total, threads))
    return out
