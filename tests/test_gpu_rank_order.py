"""The table builds rank positions with one LDS atomic per 64 positions
(fse_device.hpp wave_build_spread), which relies on same-address
ds_add_rtn_u32 results coming back in ascending lane order.  Every table
checks its own ranks and is rebuilt with the peer-mask ranks when the check
fails (fsehip_rank_fallbacks counts those).  These tests: the lane-order probe
holds on this GPU; both rank methods build identical tables; the check raises
no false alarm; and a fault injected into the ranks is caught and the output
stays exact."""
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


def _fallbacks(reset=False):
    import ctypes as C

    from entropy_coders_amd._lib import load
    import torch

    out = (C.c_uint32 * 3)()
    assert load().fsehip_rank_fallbacks(torch.cuda.current_device(), C.byref(out), 1 if reset else 0) == 0
    return list(out)


@pytest.mark.parametrize("kind,prob,log2,nstates", [(0, 0.155, 0, 2), (0, 0.77, 9, 2), (2, 0.0, 12, 2),
                                                    (1, 0.5, 13, 2), (0, 0.155, 14, 2), (0, 0.155, 5, 1),
                                                    (0, 0.05, 10, 2)])
def test_rank_self_check_no_false_alarm(kind, prob, log2, nstates):
    """Every table checks its atomic ranks (fse_device.hpp wave_build_spread):
    on a GPU whose LDS atomics keep lane order (checked above) no table may
    fail the check, at any table log, either check mode (the encoder's
    stateTable check, the decode tables' inverse check) or format."""
    import torch

    from entropy_coders_amd import BlockCodec

    _fallbacks(reset=True)
    codec = BlockCodec(block_size=16384, table_log=log2, ckpt_interval=64, nstates=nstates)
    n = 64 * 16384 + 77
    src = codec.generate(kind, prob, 0x5EED0101, n)
    cb = codec.compress(src)
    tabs = codec.build_dtables(cb)
    out, st = codec.decompress(cb)
    torch.cuda.synchronize()
    assert int(cb["status"].abs().max()) == 0 and int(st.abs().max()) == 0
    assert torch.equal(out, src)
    assert (tabs["info"].cpu().numpy() >= 0).all()
    assert _fallbacks() == [0, 0, 0]


_INJECT_CHILD = r"""
import ctypes as C, numpy as np, torch
from entropy_coders_amd import BlockCodec
from entropy_coders_amd._lib import load
from oracle import oracle as O
lib = load()
assert b"diagnostics" in lib.fsehip_version()
cnt = (C.c_uint32 * 3)()
assert lib.fsehip_rank_fallbacks(0, C.byref(cnt), 1) == 0
codec = BlockCodec(block_size=65536, ckpt_interval=64)
nb = 24
src = codec.generate(0, 0.155, 0x5EED0202, nb * 65536 - 1000)
cb = codec.compress(src)
tabs = codec.build_dtables(cb)
out, st = codec.decompress(cb)
out2, st2 = codec.decompress(cb, use_sidecar=False)
torch.cuda.synchronize()
assert int(cb["status"].abs().max()) == 0 and int(st.abs().max()) == 0 and int(st2.abs().max()) == 0
assert torch.equal(out, src) and torch.equal(out2, src)
host = src.cpu().numpy()
for b in range(nb):
    assert codec.block_bytes(cb, b) == O.compress2(host[b * 65536:(b + 1) * 65536])[0], b
assert lib.fsehip_rank_fallbacks(0, C.byref(cnt), 0) == 0
print("fallbacks", list(cnt))
assert cnt[0] == nb, list(cnt)        # every encoder table caught and rebuilt
assert cnt[1] >= 2 * nb, list(cnt)    # decode tables: build_dtables + each decode's build
print("child-ok")
"""


def test_rank_fault_injection_caught():
    """Fault injection (diagnostics build, FSEHIP_RANK_INJECT=1): the first 64
    positions of every table get their ranks in descending lane order, as a
    GPU whose LDS atomics broke the lane order would give them.  Every table
    must fail its check and be rebuilt with the peer-mask ranks, so the
    bytes still equal the oracle's and every decode route round-trips."""
    import os
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    if not os.path.exists(os.path.join(root, "entropy_coders_amd", "libfsehip_diag.so")):
        pytest.skip("diagnostics build missing")
    env = dict(os.environ, PYTHONPATH=root, FSEHIP_LIB="libfsehip_diag.so", FSEHIP_RANK_INJECT="1")
    r = subprocess.run([sys.executable, "-c", _INJECT_CHILD], cwd=root, env=env, capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0 and "child-ok" in r.stdout, (r.stdout[-2000:], r.stderr[-4000:])
