"""Decode tables on the GPU (fsehip_build_dtables, C3's pre-built dtables)
against the oracle's DecodeTable (fse.rs:280-338), and the three decode
routes (segment-parallel, serial, pre-built tables) against the
source."""
import os

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


@pytest.mark.parametrize("kind,prob,log2", [(0, 0.155, 0), (2, 0.0, 12), (0, 0.77, 9), (1, 0.5, 0),
                                            (1, 0.5, 13), (0, 0.155, 14)])
def test_dtables_match_oracle(torch_cuda, kind, prob, log2):
    torch = torch_cuda
    from entropy_coders_amd import BlockCodec

    codec = BlockCodec(block_size=16384, table_log=log2, ckpt_interval=64)
    n = 24 * 16384 + 777
    src = codec.generate(kind, prob, 0x5EED0007, n)
    cb = codec.compress(src)
    tabs = codec.build_dtables(cb)
    torch.cuda.synchronize()
    assert int(cb["status"].abs().max()) == 0
    info = tabs["info"].cpu().numpy()
    per = int(codec.lib.fsehip_dtable_bytes(codec.max_table_log)) // 4
    dt = tabs["dt"].cpu().numpy().view(np.uint32)
    for b in range(codec.n_blocks(n)):
        blk = codec.block_bytes(cb, b)
        L, ns, sym, nb, used = O.dtable(blk)
        assert info[b] >= 0, (b, info[b])
        assert info[b] >> 16 == L and info[b] & 0xFFFF == used, b
        e = dt[b * per: b * per + (1 << L)]
        assert np.array_equal(e & 0xFF, nb), b
        assert np.array_equal((e >> 8) & 0xFF, sym), b
        sh = 17 if codec.max_table_log >= 15 else 18  # newState field (fsehip.h, fsehip_build_dtables)
        assert np.array_equal(e >> sh, ns), b


def test_decode_routes_agree(torch_cuda):
    """Every decode route gives the source back: segment-parallel with the
    sidecar (tables built inside), serial without it, prebuilt tables with
    and without the sidecar, and the sidecar recorded by the serial decoder
    equal to the encoder's."""
    torch = torch_cuda
    from entropy_coders_amd import BlockCodec

    codec = BlockCodec(block_size=65536, ckpt_interval=128)
    n = 48 * 65536 + 4321
    src = codec.generate(0, 0.2, 0x5EED0008, n)
    cb = codec.compress(src)
    for side in (True, False):
        out, st = codec.decompress(cb, use_sidecar=side)
        torch.cuda.synchronize()
        assert int(st.abs().max()) == 0 and torch.equal(out, src), side
    tabs = codec.build_dtables(cb)
    for side in (True, False):
        out = torch.empty_like(src)
        st = torch.zeros(codec.n_blocks(n), dtype=torch.int32, device=src.device)
        codec.decompress_dt_into(cb, tabs, out, st, use_sidecar=side)
        torch.cuda.synchronize()
        assert int(st.abs().max()) == 0 and torch.equal(out, src), side
    out, side, st = codec.build_sidecar(cb)
    torch.cuda.synchronize()
    assert int(st.abs().max()) == 0 and torch.equal(out, src)
    nb = codec.n_blocks(n)
    assert torch.equal(side[: nb * codec.side_per_block], cb["sidecar"][: nb * codec.side_per_block])


def test_dtables_error_blocks(torch_cuda):
    """Blocks the encoder rejected (comp_len 0) and corrupted headers report
    the header-read status in dtinfo and in the decode status."""
    torch = torch_cuda
    from entropy_coders_amd import BlockCodec
    from entropy_coders_amd._lib import STATUS

    codec = BlockCodec(block_size=4096, ckpt_interval=64)
    host = np.concatenate([O.generate(0, 0.3, 3, 0, 4096), np.zeros(4096, np.uint8),
                           O.generate(0, 0.3, 3, 2, 4096)])
    src = torch.from_numpy(host).cuda()
    cb = codec.compress(src)
    # corrupt block 2's marker byte
    ln = int(cb["comp_len"][2])
    cb["out"][2 * codec.slot_bytes + ln - 1] = 0
    tabs = codec.build_dtables(cb)
    out = torch.empty_like(src)
    st = torch.zeros(3, dtype=torch.int32, device=src.device)
    codec.decompress_dt_into(cb, tabs, out, st)
    torch.cuda.synchronize()
    info = tabs["info"].cpu().numpy()
    stat = st.cpu().numpy()
    assert info[0] >= 0 and stat[0] == 0
    assert STATUS[int(info[1])] == "EMPTY" and stat[1] == info[1]
    assert STATUS[int(info[2])] == "NO_MARKER" and stat[2] == info[2]
    assert np.array_equal(out[:4096].cpu().numpy(), host[:4096])


@pytest.mark.parametrize("ckpt", [64, 32])
def test_dual_chain_segments(torch_cuda, ckpt):
    """Checkpoints every <= 64 pairs give a 64 KiB block more segments than
    the decoder's 256 lanes: each lane then decodes two segments
    interleaved.  Exact against the source and the oracle's bytes, on the
    prebuilt-table and the built-inside routes, with a ragged last block,
    and a corrupted checkpoint is reported on the dual path."""
    torch = torch_cuda
    from entropy_coders_amd import BlockCodec
    from entropy_coders_amd._lib import STATUS

    codec = BlockCodec(block_size=65536, ckpt_interval=ckpt)
    n = 40 * 65536 + 33333
    src = codec.generate(0, 0.155, 0x5EED0009 + ckpt, n)
    cb = codec.compress(src)
    torch.cuda.synchronize()
    assert int(cb["status"].abs().max()) == 0
    host = src.cpu().numpy()
    for b in (0, 17, 40):
        assert codec.block_bytes(cb, b) == O.compress2(host[b * 65536:(b + 1) * 65536])[0]
    out, st = codec.decompress(cb)
    torch.cuda.synchronize()
    assert int(st.abs().max()) == 0 and torch.equal(out, src)
    tabs = codec.build_dtables(cb)
    out2 = torch.empty_like(src)
    st2 = torch.zeros(codec.n_blocks(n), dtype=torch.int32, device=src.device)
    codec.decompress_dt_into(cb, tabs, out2, st2)
    torch.cuda.synchronize()
    assert int(st2.abs().max()) == 0 and torch.equal(out2, src)
    # a wrong state in a checkpoint of block 5's second half (a B-chain segment)
    spb = codec.side_per_block
    k = 5 * spb + (32767 // ckpt + 1) * 3 // 4
    cb["sidecar"][k] ^= 1 << 33
    codec.decompress_dt_into(cb, tabs, out2, st2)
    torch.cuda.synchronize()
    stat = st2.cpu().numpy()
    assert STATUS[int(stat[5])] == "BAD_SIDECAR"
    assert (np.delete(stat, 5) == 0).all()


@pytest.mark.parametrize("n_blocks", [320, 40])
def test_dtables_damaged_headers(torch_cuda, n_blocks):
    """Header parse at batch sizes on both sides of the lane-parallel parse
    (hdr_parse_kernel, batches of >= 256 blocks; smaller ones parse on the
    scalar unit inside the table kernel): blocks with damaged header bytes get
    the oracle's NormHistogram::read status, the others its table, entry for
    entry."""
    torch = torch_cuda
    from entropy_coders_amd import BlockCodec
    from entropy_coders_amd._lib import STATUS

    rng = np.random.default_rng(0xD7AB + n_blocks)
    codec = BlockCodec(block_size=4096, ckpt_interval=64)
    host = np.concatenate([O.generate(int(rng.integers(0, 3)), float(rng.uniform(0.05, 0.8)), int(rng.integers(1 << 30)),
                                      b, 4096) for b in range(n_blocks)])
    cb = codec.compress(torch.from_numpy(host).cuda())
    torch.cuda.synchronize()
    assert int(cb["status"].abs().max()) == 0
    slots = cb["out"].cpu().numpy().copy()
    lens = cb["comp_len"].cpu().numpy()
    sb = codec.slot_bytes
    for b in range(n_blocks):
        if rng.random() < 0.5:
            for _ in range(int(rng.integers(1, 4))):  # header bytes only: the marker stays
                i = int(rng.integers(0, min(int(lens[b]) - 1, 40)))
                slots[b * sb + i] ^= np.uint8(1 << int(rng.integers(0, 8)))
    cb["out"] = torch.from_numpy(slots).cuda()
    tabs = codec.build_dtables(cb)
    torch.cuda.synchronize()
    info = tabs["info"].cpu().numpy()
    per = int(codec.lib.fsehip_dtable_bytes(codec.max_table_log)) // 4
    dt = tabs["dt"].cpu().numpy().view(np.uint32)
    bad = 0
    for b in range(n_blocks):
        blk = slots[b * sb: b * sb + int(lens[b])].tobytes()
        try:
            L, ns, sym, nb, used = O.dtable(blk)
        except O.OracleError as e:
            assert info[b] == e.rc, (b, info[b], e.code)
            bad += 1
            continue
        if L > codec.max_table_log:  # a valid header beyond this codec's tables (max_table_log 11)
            assert STATUS[int(info[b])] == "UNSUPPORTED", (b, info[b])
            bad += 1
            continue
        if used >= len(blk):  # the header ran into the marker byte: NO_MARKER (lib.rs:222)
            assert info[b] < 0, b
            continue
        assert info[b] >= 0 and info[b] >> 16 == L and info[b] & 0xFFFF == used, (b, info[b])
        e = dt[b * per: b * per + (1 << L)]
        assert np.array_equal(e & 0xFF, nb) and np.array_equal((e >> 8) & 0xFF, sym), b
        assert np.array_equal(e >> 18, ns), b
    # (damaged headers often still parse: the oracle then gives the same other table)


@pytest.mark.parametrize("log2", [0, 5, 6, 8, 10, 11])
def test_dtables_parallel_build_match_oracle(torch_cuda, log2):
    """Batches of >= 256 blocks at L <= 11 build their tables from the
    lane-parallel header parse (hdr_parse_kernel -> dtable_blocks_kernel):
    every block's table against the oracle's DecodeTable entry for entry,
    over skewed / near-uniform (table_len > 64) / sparse / geometric blocks,
    so -1 symbols, long zero runs and wide alphabets all occur.  (The same
    test passed on the 4-wave dtable_par_kernel of the diagnostics build.)"""
    torch = torch_cuda
    from entropy_coders_amd import BlockCodec

    rng = np.random.default_rng(0x9A2 + log2)
    nb_, bs = 288, 4096
    blocks = []
    for b in range(nb_):
        k = b % 4
        if k == 0:
            blocks.append(O.generate(0, float(rng.uniform(0.05, 0.8)), int(rng.integers(1 << 30)), b, bs))
        elif k == 1:
            blocks.append(O.generate(2, 0.0, int(rng.integers(1 << 30)), b, bs))
        elif k == 2:
            alpha = np.sort(rng.choice(256, size=int(rng.integers(2, 120)), replace=False)).astype(np.uint8)
            w = rng.random(len(alpha)) ** 4 + 1e-4
            blocks.append(alpha[rng.choice(len(alpha), size=bs, p=w / w.sum())])
        else:
            blocks.append(np.minimum(rng.geometric(float(rng.uniform(0.2, 0.8)), bs) - 1, 255).astype(np.uint8))
    host = np.concatenate(blocks)
    codec = BlockCodec(block_size=bs, table_log=log2, ckpt_interval=64)
    cb = codec.compress(torch.from_numpy(host).cuda())
    tabs = codec.build_dtables(cb)
    torch.cuda.synchronize()
    st = cb["status"].cpu().numpy()
    info = tabs["info"].cpu().numpy()
    per = int(codec.lib.fsehip_dtable_bytes(codec.max_table_log)) // 4
    dt = tabs["dt"].cpu().numpy().view(np.uint32)
    checked = wide = 0
    for b in range(nb_):
        if st[b] != 0:  # e.g. a single-symbol block at a forced log
            continue
        blk = codec.block_bytes(cb, b)
        L, ns, sym, nb, used = O.dtable(blk)
        assert info[b] >= 0 and info[b] >> 16 == L and info[b] & 0xFFFF == used, (b, info[b])
        e = dt[b * per: b * per + (1 << L)]
        assert np.array_equal(e & 0xFF, nb), b
        assert np.array_equal((e >> 8) & 0xFF, sym), b
        assert np.array_equal(e >> 18, ns), b
        checked += 1
        wide += int(sym.max()) >= 64
    assert checked >= nb_ * 3 // 4 and wide > 0, (checked, wide)
