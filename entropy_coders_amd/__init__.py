"""entropy_coders_amd -- MI355X-native FSE (tANS) entropy coder.

Drop-in for the hot path of Cognoscan/entropy_coders: `fse_compress2`,
`fse_decompress2`, the 1-state `fse_compress` / `fse_decompress` and
`Histogram::new` run as hand-written HIP kernels for
gfx950 behind a C ABI (include/fsehip.h).  See DESIGN.md.
"""
from ._lib import FseError, STATUS, load  # noqa: F401
from .fse import (  # noqa: F401
    BlockCodec, compress, compress2, compress2_log, decompress, decompress2, histogram_count,
)

__all__ = ["FseError", "STATUS", "load", "BlockCodec", "compress", "compress2", "compress2_log",
           "decompress", "decompress2", "histogram_count"]
