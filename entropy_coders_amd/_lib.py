"""Loader for the in-tree HIP library libfsehip.so (the product).

There is no CPU fallback: if the library is missing or no HIP device is
usable, calls raise.  Build with ``make -C entropy_coders_amd`` or
``__graft_entry__.build()``.
"""
from __future__ import annotations

import ctypes as C
import os

HERE = os.path.dirname(os.path.abspath(__file__))
# FSEHIP_LIB: an alternative in-tree build of the same library for the
# diagnostics in tools/ -- libfsehip_diag.so (`make diag`: the environment
# knobs compiled in) or an A/B variant libfsehip_NAME.so
# (tools/variant_build.sh).  Only a bare libfsehip_*.so name beside this file
# is accepted; the product is libfsehip.so, which reads no environment.
_LIB_NAME = os.environ.get("FSEHIP_LIB", "libfsehip.so")
if _LIB_NAME != "libfsehip.so" and not (
        _LIB_NAME.startswith("libfsehip_") and _LIB_NAME.endswith(".so") and os.sep not in _LIB_NAME):
    raise RuntimeError(f"FSEHIP_LIB={_LIB_NAME!r}: expected libfsehip_NAME.so (an in-tree variant build)")
LIB_PATH = os.path.join(HERE, _LIB_NAME)

# every symbol include/fsehip.h declares (checked by tests/test_abi.py)
EXPORTS = (
    "fse_compress2", "fse_compress2_log", "fse_decompress2", "histogram_count",
    "fsehip_slot_bytes", "fsehip_sidecar_per_block", "fsehip_compress_blocks",
    "fsehip_decompress_blocks", "fsehip_build_sidecar", "fsehip_decompress_streams", "fsehip_histogram_blocks",
    "fsehip_generate", "fsehip_device_count", "fsehip_version",
    "fsehip_pack_blocks", "fsehip_unpack_blocks",
    "fsehip_dtable_bytes", "fsehip_build_dtables", "fsehip_decompress_blocks_dt",
    "fse_compress", "fse_decompress", "fsehip_sidecar_per_block_ns", "fse_decompress2_many", "fse_decompress_many",
    "fsehip_copy_blocks", "fsehip_release_workspace", "fsehip_rank_fallbacks",
    "histogram_new", "histogram_normalize", "histogram_normalize_optimal", "norm_histogram_new",
    "norm_histogram_write", "norm_histogram_read", "encode_table_new", "decode_table_new", "fse_compress_nh",
    "bitstack_write", "bitstack_read", "bitstream_read", "bitstream_read_ops",
    "fsehip_bitstack_write", "fsehip_bitstack_read", "fsehip_bitstream_read", "fsehip_bitstream_read_ops",
    "bitstack_reader_new", "bitstack_reader_reload", "bitstack_reader_peek", "bitstack_reader_read_no_reload",
    "bitstack_reader_advance_no_reload", "bitstack_reader_read", "bitstack_reader_available", "bitstack_reader_finish",
    "bitstream_reader_new", "bitstream_reader_read", "bitstream_reader_advance_by", "bitstream_reader_peek",
    "bitstream_reader_available", "bitstream_reader_finish", "bitstream_reader_finish_byte",
    "bitstack_writer_new", "bitstack_writer_flush", "bitstack_writer_write_bits_raw",
    "bitstack_writer_write_bits_raw_unmasked", "bitstack_writer_write_bits", "bitstack_writer_write_bits_unmasked",
    "bitstack_writer_finish",
)

STATUS = {
    0: "OK", -1: "EMPTY", -2: "TOO_SHORT", -3: "ALL_ZERO_SYMBOL0", -4: "SINGLE_SYMBOL",
    -5: "BAD_HEADER", -6: "NO_MARKER", -7: "DST_TOO_SMALL", -8: "TABLELOG_RANGE",
    -9: "CURSED", -10: "BAD_TABLE", -11: "BAD_ARG", -12: "HIP", -13: "LENGTH_MISMATCH",
    -14: "UNSUPPORTED", -15: "NO_DEVICE", -16: "BAD_SIDECAR", -17: "ENCODER_INIT",
    -18: "EOF",
}


class FseError(Exception):
    """A negative status from the C ABI (a reference panic/None/Err)."""

    def __init__(self, rc: int, what: str = ""):
        self.rc = rc
        self.code = STATUS.get(rc, str(rc))
        super().__init__(f"{what}: status {rc} ({self.code})" if what else f"status {rc} ({self.code})")


class Params(C.Structure):
    _fields_ = [("block_size", C.c_uint32), ("table_log", C.c_uint32),
                ("ckpt_interval", C.c_uint32), ("max_table_log", C.c_uint32),
                ("nstates", C.c_uint32)]


class Histogram(C.Structure):
    """fse_histogram = Histogram (histogram.rs:9-14)."""
    _fields_ = [("counts", C.c_uint32 * 256), ("size", C.c_uint32), ("table_len", C.c_uint32)]


class NormHistogram(C.Structure):
    """fse_norm_histogram = NormHistogram (histogram.rs:289-294)."""
    _fields_ = [("norm", C.c_int32 * 256), ("log2", C.c_uint32), ("table_len", C.c_uint32)]


class SymbolTransform(C.Structure):
    _fields_ = [("bits", C.c_uint32), ("find_state", C.c_int32)]


class EncodeTable(C.Structure):
    """fse_encode_table = EncodeTable (fse.rs:72-84)."""
    _fields_ = [("table_log", C.c_uint32), ("table", C.c_uint16 * 32768), ("symbols", C.c_uint8 * 32768),
                ("symbol_tt", SymbolTransform * 256)]


class DecodeTransform(C.Structure):
    _fields_ = [("new_state", C.c_uint16), ("symbol", C.c_uint8), ("num_bits", C.c_uint8)]


class DecodeTable(C.Structure):
    """fse_decode_table = DecodeTable (fse.rs:253-265)."""
    _fields_ = [("table_log", C.c_uint32), ("fast_mode", C.c_uint32), ("table", DecodeTransform * 32768)]


class BitStackReaderState(C.Structure):
    """fse_bitstack_reader = BitStackReader (stack_reader.rs:5-11)."""
    _fields_ = [("base", C.c_void_p), ("ptr", C.c_void_p), ("buffer", C.c_uint64), ("bits", C.c_uint64),
                ("finished", C.c_int32), ("reserved", C.c_int32)]


class BitStreamReaderState(C.Structure):
    """fse_bitstream_reader = BitStreamReader (stream_reader.rs:5-11)."""
    _fields_ = [("src", C.c_void_p), ("n", C.c_uint64), ("total_bits", C.c_uint64), ("bits_read", C.c_uint64)]


class BitStackWriterState(C.Structure):
    """fse_bitstack_writer = BitStackWriter (writer.rs:5-12)."""
    _fields_ = [("dst", C.c_void_p), ("cap", C.c_uint64), ("len", C.c_uint64), ("initial_len", C.c_uint64),
                ("storage", C.c_uint64), ("bits", C.c_uint32), ("status", C.c_int32)]


_lib = None


def load() -> C.CDLL:
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(f"{LIB_PATH} is missing: build the HIP extension first "
                           "(make -C entropy_coders_amd); there is no CPU fallback")
    # One HIP runtime per process: PyTorch ships its own libamdhip64.so.7 /
    # libhsa-runtime64.so.1 and loads them by path; loaded first, the
    # library's DT_NEEDED entries (same sonames) resolve to torch's copies.
    # Loaded the other way round, /opt/rocm's runtime comes in first and torch
    # then finds no GPU ("No HIP GPUs are available", seen when a test called
    # the library before touching torch).  So torch, when installed, goes first.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    lib = C.CDLL(LIB_PATH)
    P, sz, u32, u64, i32 = C.c_void_p, C.c_size_t, C.c_uint32, C.c_uint64, C.c_int32
    lib.fse_compress2.argtypes = [P, sz, P, sz, C.POINTER(sz), C.POINTER(u64)]
    lib.fse_compress2_log.argtypes = [P, sz, u32, P, sz, C.POINTER(sz), C.POINTER(u64)]
    lib.fse_decompress2.argtypes = [P, sz, P, sz, C.POINTER(sz)]
    lib.fse_compress.argtypes = [P, sz, P, sz, C.POINTER(sz), C.POINTER(u64)]
    lib.fse_decompress.argtypes = [P, sz, P, sz, C.POINTER(sz)]
    lib.fse_decompress2_many.argtypes = [P, P, sz, P, sz, P, P]
    lib.fse_decompress_many.argtypes = [P, P, sz, P, sz, P, P]
    lib.histogram_count.argtypes = [P, sz, P, C.POINTER(u32)]
    lib.fsehip_slot_bytes.argtypes = [u32, u32]
    lib.fsehip_slot_bytes.restype = u64
    lib.fsehip_sidecar_per_block.argtypes = [u32, u32]
    lib.fsehip_sidecar_per_block.restype = u32
    lib.fsehip_sidecar_per_block_ns.argtypes = [u32, u32, u32]
    lib.fsehip_sidecar_per_block_ns.restype = u32
    lib.fsehip_compress_blocks.argtypes = [C.POINTER(Params), P, u64, P, u64, P, P, P, P, P]
    lib.fsehip_decompress_blocks.argtypes = [C.POINTER(Params), P, u64, P, P, P, u64, P, P]
    lib.fsehip_build_sidecar.argtypes = [C.POINTER(Params), P, u64, P, P, u64, P, P, P]
    lib.fsehip_decompress_streams.argtypes = [C.c_uint32, C.c_uint32, P, u64, P, C.c_uint32, P, C.c_uint32, P, P, P]
    lib.fsehip_dtable_bytes.argtypes = [u32]
    lib.fsehip_dtable_bytes.restype = u64
    lib.fsehip_build_dtables.argtypes = [C.POINTER(Params), P, u64, P, u32, P, P, P]
    lib.fsehip_decompress_blocks_dt.argtypes = [C.POINTER(Params), P, u64, P, P, P, P, P, u64, P, P]
    lib.fsehip_histogram_blocks.argtypes = [P, u64, u32, P, P, P]
    lib.fsehip_generate.argtypes = [C.c_int, C.c_double, u64, u32, P, u64, P]
    lib.fsehip_pack_blocks.argtypes = [P, u64, P, P, u32, P, P]
    lib.fsehip_unpack_blocks.argtypes = [P, P, P, u32, P, u64, P]
    lib.fsehip_copy_blocks.argtypes = [P, P, P, u32, P, P, P]
    lib.fsehip_release_workspace.argtypes = [C.c_int, P]
    lib.fsehip_rank_fallbacks.argtypes = [C.c_int, C.POINTER(u32 * 3), C.c_int]
    H, NH = C.POINTER(Histogram), C.POINTER(NormHistogram)
    lib.histogram_new.argtypes = [P, sz, H]
    lib.histogram_normalize.argtypes = [H, u32, NH]
    lib.histogram_normalize_optimal.argtypes = [H, NH]
    lib.norm_histogram_new.argtypes = [P, sz, NH]
    lib.norm_histogram_write.argtypes = [NH, P, sz, C.POINTER(sz), C.POINTER(u64)]
    lib.norm_histogram_read.argtypes = [P, sz, NH, C.POINTER(sz)]
    lib.encode_table_new.argtypes = [NH, C.POINTER(EncodeTable)]
    lib.decode_table_new.argtypes = [NH, C.POINTER(DecodeTable)]
    lib.fse_compress_nh.argtypes = [P, sz, P, sz, C.POINTER(sz), C.POINTER(u64), NH]
    lib.bitstack_write.argtypes = [P, P, sz, P, sz, C.POINTER(sz), C.POINTER(u64)]
    lib.bitstack_read.argtypes = [P, sz, P, sz, P, C.POINTER(sz), C.POINTER(C.c_int)]
    lib.bitstream_read.argtypes = [P, sz, u64, P, sz, P, C.POINTER(sz), C.POINTER(u64)]
    lib.bitstream_read_ops.argtypes = [P, sz, u64, P, P, sz, P, C.POINTER(sz), C.POINTER(u64)]
    lib.fsehip_bitstack_write.argtypes = [P, P, u64, P, u64, P, P]
    lib.fsehip_bitstack_read.argtypes = [P, u64, P, u64, P, P, P]
    lib.fsehip_bitstream_read.argtypes = [P, u64, u64, P, u64, P, P, P]
    lib.fsehip_bitstream_read_ops.argtypes = [P, u64, u64, P, P, u64, P, P, P]
    SR, TR, SW = C.POINTER(BitStackReaderState), C.POINTER(BitStreamReaderState), C.POINTER(BitStackWriterState)
    pu32 = C.POINTER(u32)
    lib.bitstack_reader_new.argtypes = [SR, P, sz]
    lib.bitstack_reader_reload.argtypes = [SR]
    for f in ("peek", "read_no_reload", "read"):
        getattr(lib, "bitstack_reader_" + f).argtypes = [SR, u32, pu32]
    lib.bitstack_reader_advance_no_reload.argtypes = [SR, u32]
    lib.bitstack_reader_available.argtypes = [SR]
    lib.bitstack_reader_available.restype = u64
    lib.bitstack_reader_finish.argtypes = [SR]
    lib.bitstream_reader_new.argtypes = [TR, P, sz, u64]
    lib.bitstream_reader_read.argtypes = [TR, u32, pu32]
    lib.bitstream_reader_peek.argtypes = [TR, u32, pu32]
    lib.bitstream_reader_advance_by.argtypes = [TR, u32]
    lib.bitstream_reader_available.argtypes = [TR]
    lib.bitstream_reader_available.restype = u64
    lib.bitstream_reader_finish.argtypes = [TR, C.POINTER(sz), C.POINTER(u64), pu32]
    lib.bitstream_reader_finish_byte.argtypes = [TR]
    lib.bitstream_reader_finish_byte.restype = sz
    lib.bitstack_writer_new.argtypes = [SW, P, sz, sz]
    lib.bitstack_writer_flush.argtypes = [SW]
    for f in ("write_bits_raw", "write_bits_raw_unmasked", "write_bits", "write_bits_unmasked"):
        getattr(lib, "bitstack_writer_" + f).argtypes = [SW, u32, u32]
    lib.bitstack_writer_finish.argtypes = [SW, C.POINTER(sz), C.POINTER(u64)]
    lib.fsehip_device_count.argtypes = []
    lib.fsehip_version.restype = C.c_char_p
    for name in EXPORTS:
        if getattr(lib, name, None) is None:
            raise RuntimeError(f"libfsehip.so lacks {name}")
    _lib = lib
    return lib


def check(rc: int, what: str = "") -> None:
    if rc != 0:
        raise FseError(rc, what)
