"""Segment decode with the decode tables built inside the decode workgroups
(fsehipx_dec_inwg(1): fsehip_decompress_blocks with a sidecar, 2-state, table
log <= 11, batches of >= 256 blocks: hdr_parse_kernel, then each decode
workgroup builds its block's table in LDS while staging its image; a measured
negative, compiled only into -DFSEHIP_DEC_INWG=1 builds: skipped otherwise) against the route on prebuilt tables
(fsehip_build_dtables + fsehip_decompress_blocks_dt) and the source: same
output bytes and the same per-block statuses, also for damaged headers and
damaged markers (NormHistogram::read errors, NO_MARKER, BAD_TABLE)."""
import numpy as np
import pytest

from oracle import oracle as O

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch_cuda():
    import ctypes as C

    import torch

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from entropy_coders_amd._lib import load
    f = load().fsehipx_dec_inwg
    f.argtypes = [C.c_int]
    f.restype = C.c_int
    if f(1) < 0:
        pytest.skip("in-workgroup tables not built into this library (FSEHIP_DEC_INWG)")
    yield torch
    f(0)


def _both_routes(torch, codec, cb, n):
    out_a = torch.empty(n, dtype=torch.uint8, device="cuda")
    st_a = torch.zeros(codec.n_blocks(n), dtype=torch.int32, device="cuda")
    codec.decompress_into(cb, out_a, st_a)  # in-workgroup tables (>= 256 blocks, L <= 11)
    tabs = codec.build_dtables(cb)
    out_b = torch.empty(n, dtype=torch.uint8, device="cuda")
    st_b = torch.zeros_like(st_a)
    codec.decompress_dt_into(cb, tabs, out_b, st_b)  # prebuilt tables
    torch.cuda.synchronize()
    return out_a.cpu().numpy(), st_a.cpu().numpy(), out_b.cpu().numpy(), st_b.cpu().numpy()


@pytest.mark.parametrize("kind,prob,log2", [(0, 0.155, 0), (0, 0.77, 9), (1, 0.5, 0), (2, 0.0, 11), (0, 0.05, 10),
                                            (0, 0.155, 5), (0, 0.3, 7)])
def test_inwg_tables_roundtrip(torch_cuda, kind, prob, log2):
    torch = torch_cuda
    from entropy_coders_amd import BlockCodec

    codec = BlockCodec(block_size=65536, table_log=log2, ckpt_interval=64)
    n = 300 * 65536 + 4321  # 301 blocks, a short last one
    src = codec.generate(kind, prob, 0x5EED0021, n)
    cb = codec.compress(src)
    torch.cuda.synchronize()
    assert int(cb["status"].abs().max()) == 0
    a, sa, b, sb = _both_routes(torch, codec, cb, n)
    assert (sa == 0).all() and (sb == 0).all()
    ref = src.cpu().numpy()
    assert np.array_equal(a, ref)
    assert np.array_equal(b, ref)


def test_inwg_tables_damaged(torch_cuda):
    torch = torch_cuda
    from entropy_coders_amd import BlockCodec

    rng = np.random.default_rng(0x1A6)
    nb, bs = 320, 4096
    codec = BlockCodec(block_size=bs, ckpt_interval=64)
    host = np.concatenate([O.generate(int(rng.integers(0, 3)), float(rng.uniform(0.05, 0.8)), int(rng.integers(1 << 30)),
                                      b, bs) for b in range(nb)])
    cb = codec.compress(torch.from_numpy(host).cuda())
    torch.cuda.synchronize()
    assert int(cb["status"].abs().max()) == 0
    slots = cb["out"].cpu().numpy().copy()
    lens = cb["comp_len"].cpu().numpy()
    sl = codec.slot_bytes
    for b in range(nb):
        r = rng.random()
        if r < 0.4:  # header bytes
            for _ in range(int(rng.integers(1, 4))):
                i = int(rng.integers(0, min(int(lens[b]) - 1, 40)))
                slots[b * sl + i] ^= np.uint8(1 << int(rng.integers(0, 8)))
        elif r < 0.5:  # the marker byte
            slots[b * sl + int(lens[b]) - 1] = 0
    cb["out"] = torch.from_numpy(slots).cuda()
    a, sa, b_, sb = _both_routes(torch, codec, cb, nb * bs)
    assert np.array_equal(sa, sb)
    assert (sa != 0).sum() > 0
    for b in range(nb):  # blocks both routes decoded agree byte for byte
        if sa[b] == 0:
            assert np.array_equal(a[b * bs:(b + 1) * bs], b_[b * bs:(b + 1) * bs]), b
