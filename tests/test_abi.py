"""CPU-side checks of the product boundary: the HIP library builds, loads
without a GPU, and exports every symbol include/fsehip.h declares."""
import os
import re

import pytest

from entropy_coders_amd import _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_header_declares_exports():
    src = open(os.path.join(ROOT, "include", "fsehip.h")).read()
    declared = set(re.findall(r"^\w[\w\s\*]*?\b(\w+)\(", src, flags=re.M))
    declared = {d for d in declared if d.startswith(("fse", "histogram", "norm_histogram", "encode_table",
                                                     "decode_table", "bitstack", "bitstream"))}
    assert declared == set(_lib.EXPORTS), declared ^ set(_lib.EXPORTS)


def test_library_loads_and_exports():
    lib = _lib.load()
    for name in _lib.EXPORTS:
        assert getattr(lib, name) is not None
    assert lib.fsehip_version().startswith(b"fsehip")


def test_layout_helpers():
    lib = _lib.load()
    slot = lib.fsehip_slot_bytes(65536, 11)
    assert slot % 256 == 0 and slot >= 65536 * 11 // 8 + 512
    assert lib.fsehip_sidecar_per_block(65536, 512) == 65536 // 2 // 512 + 2
    assert lib.fsehip_sidecar_per_block(65536, 0) == 0


def test_no_cpu_fallback_without_gpu():
    import torch

    if torch.cuda.is_available():
        pytest.skip("GPU present")
    from entropy_coders_amd import FseError, compress2

    with pytest.raises(FseError) as e:
        compress2(b"abcabcabd" * 10)
    assert e.value.code == "NO_DEVICE"


def test_pod_layouts():
    """The plain-data twins of the Rust types have the C header's layout."""
    import ctypes as C

    assert C.sizeof(_lib.Histogram) == 256 * 4 + 8
    assert C.sizeof(_lib.NormHistogram) == 256 * 4 + 8
    assert C.sizeof(_lib.EncodeTable) == 4 + 2 * 32768 + 32768 + 256 * 8
    assert C.sizeof(_lib.DecodeTransform) == 4
    assert C.sizeof(_lib.DecodeTable) == 8 + 4 * 32768
    assert _lib.EncodeTable.symbol_tt.offset == 4 + 2 * 32768 + 32768


def test_block_size_limit_rejected_before_any_gpu_work():
    """Blocks above 2^28 bytes would overflow the kernels' u32 bit counts:
    both batched entry points refuse them (UNSUPPORTED) up front."""
    import ctypes as C

    lib = _lib.load()
    p = _lib.Params(1 << 29, 0, 128, 11, 2)
    fake = C.c_void_p(16)
    rc = lib.fsehip_compress_blocks(C.byref(p), fake, 1 << 29, fake, 1 << 30, fake, fake, None, fake, None)
    assert _lib.STATUS[rc] == "UNSUPPORTED"
    rc = lib.fsehip_decompress_blocks(C.byref(p), fake, 1 << 30, fake, None, fake, 1 << 29, fake, None)
    assert _lib.STATUS[rc] == "UNSUPPORTED"


def test_building_blocks_fail_loudly_without_gpu():
    import torch

    if torch.cuda.is_available():
        pytest.skip("GPU present")
    from entropy_coders_amd import (FseError, bitstack_write, histogram_new, norm_histogram_new,
                                    norm_histogram_read)

    for call in (lambda: histogram_new(b"abc"), lambda: norm_histogram_new(b"abcabd"),
                 lambda: norm_histogram_read(b"\x06\x10"), lambda: bitstack_write([1, 2], [3, 4])):
        with pytest.raises(FseError) as e:
            call()
        assert e.value.code == "NO_DEVICE"


def test_decoder_alignment_rejected_before_any_gpu_work():
    """The decoders read whole 16/32-byte chunks of a slot and store 16-byte
    output groups: misaligned strides or buffers are BAD_ARG up front
    (fsehip.h), never misaligned vector accesses."""
    import ctypes as C

    lib = _lib.load()
    ok, odd = C.c_void_p(4096), C.c_void_p(4096 + 8)
    stat = C.c_void_p(8192)
    # fsehip_decompress_streams: out_stride 24008 is not a multiple of 16; d_out off by 8
    assert _lib.STATUS[lib.fsehip_decompress_streams(2, 11, ok, 256, ok, 4, ok, 24008, stat, stat, None)] == "BAD_ARG"
    assert _lib.STATUS[lib.fsehip_decompress_streams(2, 11, ok, 256, ok, 4, odd, 24000, stat, stat, None)] == "BAD_ARG"
    # fsehip_decompress_blocks_dt: slot not a multiple of 32, d_in or d_out misaligned
    p = _lib.Params(65536, 0, 0, 12, 2)
    for d_in, slot, d_out in ((ok, 90880 + 16, ok), (odd, 90880, ok), (ok, 90880, odd)):
        rc = lib.fsehip_decompress_blocks_dt(C.byref(p), d_in, slot, ok, None, ok, ok, d_out, 65536, stat, None)
        assert _lib.STATUS[rc] == "BAD_ARG", (d_in, slot, d_out)


def test_product_library_reads_no_environment():
    """The product libfsehip.so has no environment knobs: it does not import
    getenv and holds none of the diagnostics variables' names (those live in
    libfsehip_diag.so, `make diag`).  A drop-in must not change its output
    because of a variable in the caller's environment (lib.rs:146-248 are
    pure functions)."""
    import subprocess

    path = os.path.join(ROOT, "entropy_coders_amd", "libfsehip.so")
    dyn = subprocess.run(["nm", "-D", path], capture_output=True, text=True, check=True).stdout
    assert not re.search(r"\bU (secure_)?getenv\b", dyn), "product library imports getenv"
    blob = open(path, "rb").read()
    for knob in (b"FSEHIP_DEBUG", b"FSEHIP_ENC_LANES", b"FSEHIP_SERIAL_DEFER", b"FSEHIP_SERIAL_DW",
                 b"FSEHIP_STAMPS", b"FSEHIP_ENC_XLDS", b"FSEHIP_DT_XLDS", b"FSEHIP_RANK_INJECT"):
        assert knob not in blob, knob


def test_lib_variant_name_is_checked():
    """FSEHIP_LIB (tools only) accepts nothing but an in-tree libfsehip_*.so name."""
    import subprocess
    import sys

    for bad in ("../../tmp/x.so", "/tmp/libfsehip_x.so", "libother.so"):
        r = subprocess.run([sys.executable, "-c", "import entropy_coders_amd"], cwd=ROOT,
                           env=dict(os.environ, FSEHIP_LIB=bad, PYTHONPATH=ROOT), capture_output=True, text=True)
        assert r.returncode != 0 and "FSEHIP_LIB" in r.stderr, bad
