"""Resident workgroups per CU of the main kernels on this device (the
library's fsehipx_occupancy diagnostics export; FSEHIP_LIB picks a build)."""
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from entropy_coders_amd import _lib  # noqa: E402

lib = _lib.load()
buf = C.create_string_buffer(4096)
lib.fsehipx_occupancy.restype = C.c_int
n = lib.fsehipx_occupancy(buf, 4096)
print(buf.value[:n].decode())
