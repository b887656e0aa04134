"""The table builds rank positions with one LDS atomic per 64 positions
(fse_device.hpp wave_build_spread), which relies on same-address
ds_add_rtn_u32 results coming back in ascending lane order.  The library
checks that once per device before its first table build and falls back to
peer-mask ranks if it fails; this test runs the same check kernel and
requires the property to hold here, so that the fast path is the one the
other GPU tests exercise."""
import ctypes as C

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def test_lds_atomic_lane_order():
    from entropy_coders_amd._lib import load
    lib = load()
    f = lib.fsehipx_rank_order_check
    f.argtypes = [C.POINTER(C.c_uint32), C.POINTER(C.c_uint64)]
    f.restype = C.c_int
    bad, total = C.c_uint32(123), C.c_uint64(0)
    assert f(C.byref(bad), C.byref(total)) == 0
    assert total.value > 1_000_000
    assert bad.value == 0


@pytest.fixture()
def rank_mode():
    from entropy_coders_amd._lib import load
    f = load().fsehipx_rank_mode
    f.argtypes = [C.c_int]
    f.restype = C.c_int
    yield f
    f(-1)


@pytest.mark.parametrize("kind,prob,log2,nstates", [(0, 0.155, 0, 2), (0, 0.77, 9, 2), (2, 0.0, 12, 2),
                                                    (1, 0.5, 13, 2), (0, 0.155, 14, 2), (0, 0.155, 0, 1),
                                                    (0, 0.05, 10, 2)])
def test_peer_rank_fallback_matches_atomic(rank_mode, kind, prob, log2, nstates):
    """The fallback (peer-mask ranks) and the atomic ranks build the same
    tables: identical compressed blocks, sidecars and decode tables."""
    import torch

    from entropy_coders_amd import BlockCodec

    codec = BlockCodec(block_size=16384, table_log=log2, ckpt_interval=64, nstates=nstates)
    n = 40 * 16384 + 333
    src = codec.generate(kind, prob, 0x5EED0011, n)
    out = {}
    for mode in (0, 1):
        rank_mode(mode)
        cb = codec.compress(src)
        tabs = codec.build_dtables(cb)
        torch.cuda.synchronize()
        assert int(cb["status"].abs().max()) == 0
        nb = codec.n_blocks(n)
        lens = cb["comp_len"].cpu().numpy()
        blocks = cb["out"].view(nb, -1).cpu().numpy()
        info = tabs["info"].cpu().numpy()
        per = int(codec.lib.fsehip_dtable_bytes(codec.max_table_log)) // 4
        dt = tabs["dt"].cpu().numpy().view(np.uint32).reshape(nb, per)
        assert (info >= 0).all()
        tables = [dt[b, :1 << ((int(info[b]) >> 16) & 0xFF)].tobytes() for b in range(nb)]  # a table's 2^L entries
        out[mode] = ([bytes(blocks[b, :lens[b]]) for b in range(nb)], cb["sidecar"].cpu().numpy().tobytes(), tables,
                     info.tobytes())
    assert out[0] == out[1]
