"""Resource guard for the product kernels (CPU test, no GPU needed).

Both hot kernels are latency-bound and their speed follows the workgroups a CU
keeps resident: the encoder needs 11 per CU, the
512-thread segment decoder 3, the one-wave table kernel 21.  LDS is allocated
in whole granules, so a few hundred bytes more can cost a workgroup per CU
(round 5: 53,296 -> 54,324 B took the decoder from 3 to 2 workgroups per CU and
cost C2 decode 11 %).  This test reads the AMDGPU metadata note of the gfx950
code objects inside libfsehip.so (LDS bytes, VGPRs) and fails the build, not
the bench, when such a regression appears."""
import os
import struct

import msgpack
import pytest

from entropy_coders_amd import _lib

LDS_BYTES = 160 * 1024  # per CU (MI355X_MICROARCH.md)
LDS_GRANULE = 512       # fits every occupancy measured on gfx950 (3 x 53,296 fits, 3 x 54,324 does not)
VGPRS = 512             # per SIMD lane
VGPR_GRANULE = 8


def _bundles(data):
    i = data.find(b"__CLANG_OFFLOAD_BUNDLE__")
    while i >= 0:
        (n,) = struct.unpack_from("<Q", data, i + 24)
        p = i + 32
        for _ in range(n):
            off, size, tl = struct.unpack_from("<QQQ", data, p)
            p += 24
            triple = data[p:p + tl].decode()
            p += tl
            yield triple, data[i + off:i + off + size]
        i = data.find(b"__CLANG_OFFLOAD_BUNDLE__", i + 24)


def _notes(elf):
    (shoff,) = struct.unpack_from("<Q", elf, 0x28)
    shentsize, shnum = struct.unpack_from("<HH", elf, 0x3A)
    for k in range(shnum):
        sh = shoff + k * shentsize
        (typ,) = struct.unpack_from("<I", elf, sh + 4)
        off, size = struct.unpack_from("<QQ", elf, sh + 0x18)
        if typ != 7:  # SHT_NOTE
            continue
        q = off
        while q < off + size:
            nsz, dsz, nt = struct.unpack_from("<III", elf, q)
            q += 12
            name = elf[q:q + nsz].rstrip(b"\0")
            q += (nsz + 3) & ~3
            desc = elf[q:q + dsz]
            q += (dsz + 3) & ~3
            yield name, nt, desc


def kernel_metadata(path):
    """{kernel name: metadata dict} of the gfx950 code objects in `path`."""
    data = open(path, "rb").read()
    out = {}
    for triple, co in _bundles(data):
        if "gfx950" not in triple or co[:4] != b"\x7fELF":
            continue
        for name, nt, desc in _notes(co):
            if name == b"AMDGPU" and nt == 32:  # NT_AMDGPU_METADATA
                for k in msgpack.unpackb(desc, raw=False)["amdhsa.kernels"]:
                    out[k[".name"]] = k
    return out


def workgroups_per_cu(md, lds_extra=0):
    lds = md[".group_segment_fixed_size"] + lds_extra
    gran = -(-lds // LDS_GRANULE) * LDS_GRANULE
    by_lds = LDS_BYTES // gran if gran else 64
    waves = -(-md[".max_flat_workgroup_size"] // 64)
    vg = -(-(md[".vgpr_count"] + md.get(".agpr_count", 0)) // VGPR_GRANULE) * VGPR_GRANULE
    by_vgpr = (VGPRS // vg) * 4 // waves  # waves per SIMD x 4 SIMDs
    return min(by_lds, by_vgpr)


@pytest.fixture(scope="module")
def meta():
    path = _lib.LIB_PATH
    if not os.path.exists(path):
        pytest.skip("libfsehip.so not built")
    return kernel_metadata(path)


def _find(meta, prefix):
    hits = [k for k in meta if k.startswith(prefix)]
    assert len(hits) == 1, (prefix, hits)
    return meta[hits[0]]


# (kernel, LDS bytes today, workgroups per CU it must keep)
GUARDS = [
    ("_ZN6fsehip20encode_blocks_kernelILi11ELi64ELi2EE", 14768, 11),   # C2 encode (fse_compress2, L <= 11)
    ("_ZN6fsehip20encode_blocks_kernelILi11ELi64ELi1EE", 14768, 11),   # 1-state encode
    ("_ZN6fsehip17decode_pre_kernelILi11ELj45056ELi2ELi1ELj512EE", 53296, 3),  # C2/C3 segment decode
    ("_ZN6fsehip17decode_pre_kernelILi11ELj45056ELi2ELi1ELj256EE", 53280, 3),  # 128-pair checkpoints
    ("_ZN6fsehip17decode_pre_kernelILi11ELj45056ELi1ELi1ELj512EE", 53296, 3),  # 1-state segment decode
    ("_ZN6fsehip20dtable_blocks_kernelILi11EE", 7168, 22),             # decode tables
    ("_ZN6fsehip18serial_ring_kernelILi11ELj8ELi2ELb1ELj1EE", 37088, 4),  # sidecar-less decode
    ("_ZN6fsehip17decode_pre_kernelILi11ELj67584ELi2ELi2ELj512EE", 75888, 2),  # list pass (near-uniform blocks)
    ("_ZN6fsehip17decode_pre_kernelILi12ELj65392ELi2ELi2ELj512EE", 81920, 2),  # the same at L = 12
]


def test_metadata_parses(meta):
    assert len(meta) > 40
    assert any("encode_blocks_kernel" in k for k in meta)


@pytest.mark.parametrize("prefix,lds,wgs", GUARDS)
def test_product_kernel_occupancy(meta, prefix, lds, wgs):
    md = _find(meta, prefix)
    assert md[".group_segment_fixed_size"] <= lds, (prefix, md[".group_segment_fixed_size"])
    assert workgroups_per_cu(md) >= wgs, (prefix, md[".group_segment_fixed_size"], md[".vgpr_count"])
    assert md.get(".private_segment_fixed_size", 0) == 0, "register spills to scratch"


def test_granule_model_matches_round5_regression():
    """The model reproduces the measured regression: 54,324 B is 2 per CU."""
    md = {".group_segment_fixed_size": 54324, ".max_flat_workgroup_size": 512, ".vgpr_count": 64}
    assert workgroups_per_cu(md) == 2
    md[".group_segment_fixed_size"] = 53296
    assert workgroups_per_cu(md) == 3
