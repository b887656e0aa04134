"""GPU parity for the decode stage split (decode_pre_kernel
"Oversized blocks"): blocks whose compressed image exceeds the 44 KiB LDS
stage are deferred by the first launch and decoded by the 66 KiB-stage list
pass; blocks above that use the global-memory reader. A batch that mixes
every kind (including blocks just below and above the stage sizes) must
still decode every block bit-exact, in both formats, and the encoded bytes
must equal the oracle's (lib.rs:112-143, lib.rs:148-185).
"""
import numpy as np
import pytest

from oracle import oracle as O

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch_cuda():
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch


def _mixed_src(torch, codec, layout, seed=0x5EED0777):
    """One block per (kind, prob) in `layout`, each from its own generator."""
    parts = []
    for i, (kind, prob) in enumerate(layout):
        blk = codec.generate(kind, prob, seed + i, codec.block_size)
        parts.append(blk)
    return torch.cat(parts)


def _check(torch, codec, src, n_check):
    cb = codec.compress(src)
    outs = [codec.decompress(cb), codec.decompress(cb, use_sidecar=False)]
    tabs = codec.build_dtables(cb)
    out3 = torch.empty_like(src)
    st3 = torch.zeros(codec.n_blocks(src.numel()), dtype=torch.int32, device=codec.device)
    codec.decompress_dt_into(cb, tabs, out3, st3)
    outs.append((out3, st3))
    torch.cuda.synchronize()
    assert int(cb["status"].abs().max()) == 0
    for out, st in outs:
        assert int(st.abs().max()) == 0, st.cpu().numpy()
        assert torch.equal(out, src)
    host = src.cpu().numpy()
    bs = codec.block_size
    comp = O.compress2 if codec.nstates == 2 else O.compress
    lens = cb["comp_len"].cpu().numpy()
    for b in range(n_check):
        want, wbits = comp(host[b * bs:(b + 1) * bs])
        assert codec.block_bytes(cb, b) == want, f"block {b}"
        assert int(cb["payload_bits"][b]) == wbits
    return lens


# uniform (~65 KB compressed: list pass), skewed (~8 KB), C2 (~33 KB) and
# LUT p = 0.1 (~38.6 KB): first pass
LAYOUT = [(2, 0.0), (0, 0.77), (0, 0.155), (2, 0.0), (0, 0.1), (2, 0.0), (0, 0.155), (1, 0.5), (2, 0.0)]
MID = (34560, 44 << 10)


@pytest.mark.parametrize("nstates", [2, 1])
def test_mixed_stage_batch(torch_cuda, nstates):
    from entropy_coders_amd import BlockCodec

    codec = BlockCodec(block_size=65536, ckpt_interval=128 if nstates == 2 else 64, nstates=nstates)
    src = _mixed_src(torch_cuda, codec, LAYOUT * 4)
    lens = _check(torch_cuda, codec, src, len(LAYOUT))
    assert (lens > 44 << 10).any() and (lens < 34560).any()
    assert ((lens > MID[0]) & (lens <= MID[1])).any()


@pytest.mark.parametrize("nstates", [2, 1])
def test_blocks_above_big_stage(torch_cuda, nstates):
    """128 KiB blocks: uniform ones exceed even the 66 KiB stage (global
    reader), skewed ones fit the 44 KiB stage."""
    from entropy_coders_amd import BlockCodec

    codec = BlockCodec(block_size=131072, ckpt_interval=128 if nstates == 2 else 64, nstates=nstates)
    src = _mixed_src(torch_cuda, codec, [(2, 0.0), (0, 0.77), (0, 0.155), (2, 0.0)])
    lens = _check(torch_cuda, codec, src, 4)
    assert lens.max() > 66 << 10
    assert np.count_nonzero(lens > 66 << 10) == 2


def test_deferred_pass_many_blocks(torch_cuda):
    """More blocks than the deferred pass has workgroups (2 per CU, ~512):
    each of its workgroups collects and decodes several deferred blocks of
    the strided set it scans, interleaved with blocks the first pass did."""
    from entropy_coders_amd import BlockCodec

    codec = BlockCodec(block_size=65536, ckpt_interval=128)
    src = _mixed_src(torch_cuda, codec, LAYOUT * 140)  # 1260 blocks, 700 deferred
    lens = _check(torch_cuda, codec, src, 3)
    assert np.count_nonzero(lens > 44 << 10) == 560
    assert np.count_nonzero((lens > MID[0]) & (lens <= MID[1])) == 140


@pytest.mark.parametrize("ckpt", [64, 32])
def test_wide_workgroups_fine_checkpoints(torch_cuda, ckpt):
    """More than 256 segments per block (64 KiB blocks, checkpoints every 64
    or 32 pairs): the segment decoder runs 512-thread workgroups, one segment
    per thread at 64, two interleaved per thread at 32, on both stages; every
    route must give the source back and the sidecar must be the oracle's."""
    from entropy_coders_amd import BlockCodec

    codec = BlockCodec(block_size=65536, ckpt_interval=ckpt)
    src = _mixed_src(torch_cuda, codec, LAYOUT * 2)
    _check(torch_cuda, codec, src, 4)
    cb = codec.compress(src)
    host = src.cpu().numpy()
    side = cb["sidecar"].cpu().numpy().view(np.uint64)
    per = codec.side_per_block
    for b in (0, 2, 4):  # uniform, C2, p = 0.1
        comp, _ = O.compress2(host[b * 65536:(b + 1) * 65536])
        bp, s0, s1 = O.checkpoints2(comp, ckpt)
        got = side[b * per: b * per + len(bp)]
        assert np.array_equal(got & 0xFFFFFFFF, bp.astype(np.uint64)), b
        assert np.array_equal((got >> 32) & 0xFFFF, s0.astype(np.uint64)), b
        assert np.array_equal(got >> 48, s1.astype(np.uint64)), b
