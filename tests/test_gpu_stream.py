"""GPU tests of the host-streaming pipeline: chunked,
stream-overlapped compress/decompress of host-resident data must give the
same blocks as the device codec (and the oracle) and exact round trips."""
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


@pytest.mark.parametrize("nstates,ckpt,chunk", [(2, 128, 4), (2, 0, 3), (1, 64, 5)])
def test_host_pipeline_roundtrip(torch_cuda, nstates, ckpt, chunk):
    torch = torch_cuda
    from entropy_coders_amd import BlockCodec
    from entropy_coders_amd.stream import HostPipeline

    block = 65536
    n = 13 * block + 4321  # 14 blocks, ragged tail, 4 chunks
    codec = BlockCodec(block_size=block, ckpt_interval=ckpt, nstates=nstates)
    src_dev = codec.generate(0, 0.155, 0x5EED0F04, n)
    host = src_dev.cpu().pin_memory()
    pipe = HostPipeline(codec, chunk_blocks=chunk)
    stream, lens, side, status = pipe.compress(host)
    assert int(status.abs().max()) == 0
    # same blocks as the device codec, and as the oracle on a sample
    cb = codec.compress(src_dev)
    torch.cuda.synchronize()
    assert torch.equal(lens, cb["comp_len"].cpu())
    offs = np.concatenate([[0], np.cumsum(lens.numpy().astype(np.int64))])
    raw = host.numpy()
    for b in range(codec.n_blocks(n)):
        got = stream[offs[b]:offs[b + 1]].numpy().tobytes()
        assert got == codec.block_bytes(cb, b), f"block {b}"
        if b in (0, 5, codec.n_blocks(n) - 1):
            s = raw[b * block:(b + 1) * block]
            want = O.compress2(s)[0] if nstates == 2 else O.compress(s)[0]
            assert got == want, f"block {b}"
    if ckpt:  # valid entries of each block (the rest of a block's sidecar row is unspecified)
        spb = codec.side_per_block
        want_side = cb["sidecar"].cpu()
        for b in range(codec.n_blocks(n)):
            nb_ = min(block, n - b * block)
            pm = ((nb_ - 3) // 2 if nb_ & 1 else nb_ // 2 - 1) if nstates == 2 else nb_ - 1
            k = pm // ckpt + 1
            assert torch.equal(side[b * spb: b * spb + k], want_side[b * spb: b * spb + k]), f"sidecar {b}"
    out, dstat = pipe.decompress(stream, lens, side, n)
    assert int(dstat.abs().max()) == 0
    assert torch.equal(out, host)


@pytest.mark.parametrize("ckpt", [64, 128, 512])
def test_build_sidecar_matches_encoder(torch_cuda, ckpt):
    """Blocks compressed without a sidecar (as from the CPU crate): the
    serial decoder restores them and records the same sidecar the encoder
    would have written; the parallel decoder then uses it."""
    torch = torch_cuda
    from entropy_coders_amd import BlockCodec

    n = 9 * 65536 + 1001
    ref = BlockCodec(ckpt_interval=ckpt)
    src = ref.generate(1, 0.5, 0x5EED0F05, n)
    cb_ref = ref.compress(src)
    bare = BlockCodec(ckpt_interval=0)
    cb = bare.compress(src)  # no sidecar
    torch.cuda.synchronize()
    out, side, st = ref.build_sidecar(cb)
    torch.cuda.synchronize()
    assert int(st.abs().max()) == 0
    assert torch.equal(out, src)
    spb = ref.side_per_block
    want = cb_ref["sidecar"].cpu()
    got = side.cpu()
    for b in range(ref.n_blocks(n)):
        nb_ = min(65536, n - b * 65536)
        pm = (nb_ - 3) // 2 if nb_ & 1 else nb_ // 2 - 1
        k = pm // ckpt + 1
        assert torch.equal(got[b * spb: b * spb + k], want[b * spb: b * spb + k]), f"block {b}"
    cb["sidecar"] = side
    out2, st2 = ref.decompress(cb)
    torch.cuda.synchronize()
    assert int(st2.abs().max()) == 0 and torch.equal(out2, src)
