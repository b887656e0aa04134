"""entropy_coders_amd -- MI355X-native FSE (tANS) entropy coder.

Drop-in for the hot path of Cognoscan/entropy_coders: `fse_compress2`,
`fse_decompress2`, the 1-state `fse_compress` / `fse_decompress`, the
histogram / normalisation / header / table building blocks and the
bitstream run as hand-written HIP kernels for gfx950 behind a C ABI
(include/fsehip.h).  See DESIGN.md.
"""
from ._lib import STATUS, FseError, load  # noqa: F401
from .fse import *  # noqa: F401,F403
from .fse import __all__ as _fse_all

__all__ = ["FseError", "STATUS", "load", *_fse_all]
