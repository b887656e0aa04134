"""C3 at full size (BASELINE.json configs[2]): 32,768 x 64 KiB
blocks of C2 data (LUT p=0.155, ~1 GiB compressed, 2 GiB raw), decode
tables pre-built by `fsehip_build_dtables`, decoded by
`fsehip_decompress_blocks_dt` -- exactly the bench's decode-only line.

Checks: every block's status, an exact round trip of all 2 GiB on the
device, the decode tables' info words, and the compressed bytes of sampled
blocks against the oracle's `fse_compress2` (lib.rs:146-183).  Both the
sidecar route and the reference-order route (no sidecar) are run."""
import numpy as np
import pytest

from oracle import oracle as O

pytestmark = pytest.mark.gpu

BLOCKS = 32768
BLOCK = 65536


# 64 pairs: the bench's own checkpoint interval (512 segments per block,
# decoded by the 512-thread decode_pre_kernel); 128: 256-thread workgroups
@pytest.fixture(scope="module", params=[64, 128])
def c3(request):
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from entropy_coders_amd import BlockCodec

    codec = BlockCodec(block_size=BLOCK, ckpt_interval=request.param)
    n = BLOCKS * BLOCK
    src = codec.generate(0, 0.155, 0x5EED0003, n)
    cb = codec.compress(src)
    tabs = codec.build_dtables(cb)
    torch.cuda.synchronize()
    yield torch, codec, n, src, cb, tabs
    del src, cb, tabs
    torch.cuda.empty_cache()


def test_c3_encode_statuses_and_sampled_bytes(c3):
    torch, codec, n, src, cb, tabs = c3
    assert int(cb["status"].abs().max()) == 0
    lens = cb["comp_len"].cpu().numpy()
    assert lens.min() > 0 and lens.max() <= codec.slot_bytes
    # ~1 GiB compressed, as the config says
    assert 0.45 < lens.sum() / n < 0.55
    rng = np.random.default_rng(3)
    sample = sorted(set([0, 1, BLOCKS // 2, BLOCKS - 1] + rng.integers(0, BLOCKS, 28).tolist()))
    host = src.view(BLOCKS, BLOCK)[sample].cpu().numpy()
    bits = cb["payload_bits"].cpu().numpy()
    side = cb["sidecar"].cpu().numpy().view(np.uint64)
    for i, b in enumerate(sample):
        want, wbits = O.compress2(host[i])
        assert codec.block_bytes(cb, b) == want, b
        assert bits[b] == wbits, b
        bp, s0, s1 = O.checkpoints2(want, codec.ckpt_interval)
        mine = side[b * codec.side_per_block: b * codec.side_per_block + len(bp)]
        assert np.array_equal(mine & 0xFFFFFFFF, bp.astype(np.uint64)), b
        assert np.array_equal((mine >> 32) & 0xFFFF, s0.astype(np.uint64)), b
        assert np.array_equal(mine >> 48, s1.astype(np.uint64)), b


def test_c3_dtable_info(c3):
    torch, codec, n, src, cb, tabs = c3
    info = tabs["info"].cpu().numpy()
    assert (info >= 0).all()
    assert ((info >> 16) == 11).all()  # optimal_log2 gives 11 for every 64 KiB block
    for b in (0, BLOCKS - 1):
        L, _, _, _, used = O.dtable(codec.block_bytes(cb, b))
        assert info[b] >> 16 == L and info[b] & 0xFFFF == used


@pytest.mark.parametrize("use_sidecar", [True, False])
def test_c3_decode_prebuilt_roundtrip(c3, use_sidecar):
    torch, codec, n, src, cb, tabs = c3
    out = torch.full((n,), 0xA5, dtype=torch.uint8, device=src.device)
    st = torch.full((BLOCKS,), 12345, dtype=torch.int32, device=src.device)
    codec.decompress_dt_into(cb, tabs, out, st, use_sidecar=use_sidecar)
    torch.cuda.synchronize()
    assert int(st.abs().max()) == 0
    assert torch.equal(out, src)
