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
    declared = {d for d in declared if d.startswith(("fse", "histogram"))}
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
