"""GPU edge cases against the oracle: sparse alphabets (zero runs in the
NCount header), ragged/degenerate blocks inside one batch, per-block error
statuses, and the pack/unpack compaction used by the multi-GPU gather."""
import numpy as np
import pytest

from oracle import oracle as O

pytestmark = pytest.mark.gpu

BLOCK = 4096


@pytest.fixture(scope="module")
def torch_cuda():
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch


def _sparse(rng, syms, n, weights=None):
    syms = np.asarray(syms, dtype=np.uint8)
    p = None if weights is None else np.asarray(weights, float) / np.sum(weights)
    return syms[rng.choice(len(syms), size=n, p=p)]


def _edge_blocks():
    rng = np.random.default_rng(1234)
    blocks = [
        _sparse(rng, [5, 200, 255], BLOCK),                        # long zero runs in the header
        _sparse(rng, [0, 255], BLOCK, [1, 3]),                     # 254-symbol zero run
        _sparse(rng, [1, 2], BLOCK, [1, 1000]),                    # one very rare symbol
        _sparse(rng, list(range(0, 256, 17)), BLOCK),              # periodic gaps
        _sparse(rng, list(range(256)), BLOCK),                     # full alphabet
        _sparse(rng, [0, 3, 4, 5, 6, 7, 8, 200], BLOCK, [50, 1, 1, 1, 1, 1, 1, 5]),  # repeat flags
        np.full(BLOCK, 9, np.uint8),                               # single symbol (container mode)
        np.zeros(BLOCK, np.uint8),                                 # ALL_ZERO_SYMBOL0 (reference panic)
        (np.arange(BLOCK) % 256).astype(np.uint8),                 # flat
        _sparse(rng, [7, 8], BLOCK, [1, 1]),
    ]
    return blocks


def test_sparse_host_api(torch_cuda):
    from entropy_coders_amd import compress2, decompress2

    for i, s in enumerate(_edge_blocks()):
        try:
            want, wbits = O.compress2(s)
        except O.OracleError as e:
            from entropy_coders_amd import FseError
            with pytest.raises(FseError) as g:
                compress2(s)
            assert g.value.code == e.code
            continue
        got, bits = compress2(s)
        assert got == want and bits == wbits, i
        if len(set(s.tolist())) > 1:
            assert decompress2(got) == s.tobytes(), i
    for L in (9, 10, 12):
        s = _edge_blocks()[0]
        assert compress2_log_eq(s, L)


def compress2_log_eq(s, L):
    from entropy_coders_amd import compress2_log

    return compress2_log(s, L)[0] == O.compress2(s, L)[0]


@pytest.mark.parametrize("ckpt", [0, 64, 128])
def test_edge_batch(torch_cuda, ckpt):
    torch = torch_cuda
    from entropy_coders_amd import BlockCodec
    from entropy_coders_amd._lib import STATUS

    blocks = _edge_blocks()
    tail = blocks[0][:1000]
    host = np.concatenate(blocks + [tail])
    codec = BlockCodec(block_size=BLOCK, ckpt_interval=ckpt)
    src = torch.from_numpy(host).cuda()
    cb = codec.compress(src)
    out, st = codec.decompress(cb)
    torch.cuda.synchronize()
    est = cb["status"].cpu().numpy()
    dst = st.cpu().numpy()
    outh = out.cpu().numpy()
    for b, s in enumerate(blocks + [tail]):
        try:
            want, wbits = O.compress2(s)
        except O.OracleError as e:
            assert STATUS.get(int(est[b])) == e.code, b
            assert dst[b] != 0, b
            continue
        assert est[b] == 0, b
        assert codec.block_bytes(cb, b) == want, b
        assert int(cb["payload_bits"][b]) == wbits, b
        assert dst[b] == 0, (b, dst[b])
        assert np.array_equal(outh[b * BLOCK: b * BLOCK + len(s)], s), b


def test_pack_unpack(torch_cuda):
    torch = torch_cuda
    from entropy_coders_amd import BlockCodec
    from entropy_coders_amd.dist import pack_device, pack_host

    codec = BlockCodec(block_size=65536, ckpt_interval=128)
    n = 37 * 65536 + 999
    src = codec.generate(0, 0.3, 99, n)
    cb = codec.compress(src)
    stream, offs = pack_device(cb["out"], codec.slot_bytes, cb["comp_len"])
    torch.cuda.synchronize()
    ref, roffs = pack_host(cb["out"].cpu(), codec.slot_bytes, cb["comp_len"].cpu())
    assert torch.equal(stream.cpu(), ref) and torch.equal(offs.cpu(), roffs)
    nb = codec.n_blocks(n)
    for b in (0, 17, nb - 1):
        o = int(offs[b])
        assert stream[o: o + int(cb["comp_len"][b])].cpu().numpy().tobytes() == codec.block_bytes(cb, b)
    # unpack into fresh slots, then decode from them
    import ctypes as C
    from entropy_coders_amd._lib import check, load

    lib = load()
    cb2 = codec.alloc(n)
    cb2["comp_len"].copy_(cb["comp_len"])
    cb2["sidecar"].copy_(cb["sidecar"])
    hs = C.c_void_p(torch.cuda.current_stream().cuda_stream)
    check(lib.fsehip_unpack_blocks(C.c_void_p(stream.data_ptr()), C.c_void_p(offs.data_ptr()),
                                   C.c_void_p(cb["comp_len"].data_ptr()), nb, C.c_void_p(cb2["out"].data_ptr()),
                                   codec.slot_bytes, hs))
    out, st = codec.decompress(cb2)
    torch.cuda.synchronize()
    assert int(st.abs().max()) == 0 and torch.equal(out, src)


@pytest.mark.parametrize("use_sidecar", [True, False])
def test_corrupt_blocks_fail_cleanly(torch_cuda, use_sidecar):
    """Damaged blocks (flipped payload bytes, broken headers, truncated
    lengths, a bad sidecar entry) must come back as per-block statuses or
    garbage bytes -- never a fault, a hang or a write outside the block."""
    torch = torch_cuda
    from entropy_coders_amd import BlockCodec

    block = 65536
    nb = 12
    codec = BlockCodec(block_size=block, ckpt_interval=128)
    src = codec.generate(0, 0.155, 0x5EED0F06, nb * block)
    cb = codec.compress(src)
    torch.cuda.synchronize()
    rng = np.random.default_rng(7)
    slots = cb["out"].cpu().numpy().copy()
    lens = cb["comp_len"].cpu().numpy().copy()
    side = cb["sidecar"].cpu().numpy().copy()
    sb = codec.slot_bytes
    for b in range(nb):
        base, ln = b * sb, int(lens[b])
        kind = b % 6
        if kind == 1:  # flipped payload bytes
            for i in rng.integers(64, ln - 1, 20):
                slots[base + i] ^= 0xA5
        elif kind == 2:  # broken header bytes
            slots[base: base + 8] = rng.integers(0, 256, 8, dtype=np.uint8)
        elif kind == 3:  # truncated (last byte may become 0: no marker)
            lens[b] = ln // 2
        elif kind == 4:  # marker byte cleared
            slots[base + ln - 1] = 0
        elif kind == 5:  # a sidecar entry pointing past the block
            side[b * codec.side_per_block + 3] = np.int64(0x7FFFFFF0)
    cb["out"] = torch.from_numpy(slots).to(codec.device)
    cb["comp_len"] = torch.from_numpy(lens).to(codec.device)
    cb["sidecar"] = torch.from_numpy(side).to(codec.device)
    # a guard region after the output catches writes past the last block
    buf = torch.full((nb * block + 4096,), 0x5A, dtype=torch.uint8, device=codec.device)
    st = torch.zeros(nb, dtype=torch.int32, device=codec.device)
    codec.decompress_into(cb, buf[: nb * block], st, use_sidecar=use_sidecar)
    torch.cuda.synchronize()
    status = st.cpu().numpy()
    assert bool((buf[nb * block:] == 0x5A).all()), "write past the output"
    for b in range(nb):
        if b % 6 == 0:
            assert status[b] == 0 and torch.equal(buf[b * block:(b + 1) * block], src[b * block:(b + 1) * block])
    for b in (3, 4, 9, 10):  # truncated / marker cleared: always detected
        assert status[b] != 0, (b, status)


@pytest.mark.parametrize("table_log,n_blocks", [(0, 1), (0, 3), (0, 5), (11, 7), (12, 1), (12, 3)])
def test_sidecar_less_partial_groups(torch_cuda, table_log, n_blocks):
    """The sidecar-less decoder packs K blocks into one workgroup (5 at
    L <= 11, 2 at L = 12), one decode lane each: block counts that leave a
    group part-empty, and a ragged last block, must decode exactly and
    rebuild the encoder's sidecar."""
    torch = torch_cuda
    from entropy_coders_amd import BlockCodec

    block = 65536
    codec = BlockCodec(block_size=block, table_log=table_log, ckpt_interval=128)
    n = n_blocks * block - 777
    src = codec.generate(0, 0.155, 0x5EED0A00 + n_blocks, n)
    cb = codec.compress(src)
    out = torch.full((n,), 0xA5, dtype=torch.uint8, device=codec.device)
    st = torch.full((n_blocks,), -99, dtype=torch.int32, device=codec.device)
    codec.decompress_into(cb, out, st, use_sidecar=False)
    o2, side2, st2 = codec.build_sidecar(cb)
    torch.cuda.synchronize()
    assert int(st.abs().max()) == 0 and int(st2.abs().max()) == 0
    assert torch.equal(out, src) and torch.equal(o2, src)
    assert torch.equal(side2, cb["sidecar"])


@pytest.mark.parametrize("nstates", [2, 1])
def test_sidecar_less_bulk_tail_boundary(torch_cuda, nstates):
    """The sidecar-less decoder's bulk loop runs 32 state words (64 symbols)
    between end checks and leaves the rest to the checked tail: lengths and
    capacities on either side of that boundary, in container mode (raw
    length known, ragged last blocks) and in the crate's own termination
    (fsehip_decompress_streams at several strides), against the oracle."""
    torch = torch_cuda
    from entropy_coders_amd import BlockCodec, decompress_streams

    rng = np.random.default_rng(0xB0B0 + nstates)
    for block in (64, 80, 128, 144, 192, 4096 + 64):  # multiples of 16 (several blocks)
        sizes = [block] * 5 + [int(rng.integers(2, block + 1))]
        host = np.concatenate([O.generate(0, float(rng.uniform(0.05, 0.6)), int(rng.integers(1 << 30)), 0, m)
                               for m in sizes])
        codec = BlockCodec(block_size=block, ckpt_interval=0, nstates=nstates)
        src = torch.from_numpy(host).cuda()
        cb = codec.compress(src)
        out, st = codec.decompress(cb, use_sidecar=False)
        torch.cuda.synchronize()
        for b, m in enumerate(sizes):
            lo = b * block
            seg = host[lo: lo + m]
            try:
                (O.compress2 if nstates == 2 else O.compress)(seg)
            except O.OracleError:
                assert int(st[b]) != 0, (block, b)
                continue
            assert int(st[b]) == 0, (block, b, int(st[b]))
            assert np.array_equal(out[lo: lo + m].cpu().numpy(), seg), (block, b)
    comp = (lambda x: O.compress2(x, None)[0]) if nstates == 2 else (lambda x: O.compress(x)[0])
    dec = O.decompress2 if nstates == 2 else O.decompress
    lens = list(range(3, 80)) + list(range(124, 140)) + [4096 + 60, 4096 + 66, 4096 + 70]
    streams = []
    for m in lens:
        x = O.generate(0, float(rng.uniform(0.05, 0.6)), int(rng.integers(1 << 30)), 0, m)
        if len(set(x.tolist())) < 2:
            continue
        try:
            streams.append(comp(x))
        except O.OracleError:
            continue
    for stride in (64, 80, 128, 144, 4096 + 64, 8192):  # multiples of 16 (the ABI)
        got = decompress_streams(streams, stride, nstates=nstates, max_table_log=11)
        for i, (x, g) in enumerate(zip(streams, got)):
            try:
                want = dec(x, stride)
            except O.OracleError as e:
                assert g == e.code, (stride, i, e.code, g)
                continue
            assert g == want, (stride, i)


@pytest.mark.parametrize("seed", range(6))
@pytest.mark.parametrize("nstates", [2, 1])
def test_random_corruption_never_hangs(torch_cuda, seed, nstates):
    """Random damage (payload bytes, header bytes, lengths up to the slot,
    the marker byte) on 40 blocks at once, decoded by every route: each block
    ends with a status or garbage bytes inside its own output; no fault, no
    hang (the serial decoder's loader wave and decode lanes must always
    release each other), no write past the output."""
    torch = torch_cuda
    from entropy_coders_amd import BlockCodec

    rng = np.random.default_rng(0xC0DE + seed)
    block, nb = 4096, 40
    codec = BlockCodec(block_size=block, ckpt_interval=64, nstates=nstates)
    src = codec.generate(0, float(rng.uniform(0.05, 0.8)), int(rng.integers(1 << 30)), nb * block)
    cb = codec.compress(src)
    torch.cuda.synchronize()
    slots = cb["out"].cpu().numpy().copy()
    lens = cb["comp_len"].cpu().numpy().copy()
    side = cb["sidecar"].cpu().numpy().copy()
    sb = codec.slot_bytes
    for b in range(nb):
        base, ln = b * sb, int(lens[b])
        for _ in range(int(rng.integers(0, 4))):
            what = int(rng.integers(0, 5))
            if what == 0:
                slots[base + int(rng.integers(0, ln))] ^= np.uint8(1 << int(rng.integers(0, 8)))
            elif what == 1:
                slots[base: base + 4] = rng.integers(0, 256, 4, dtype=np.uint8)
            elif what == 2:
                lens[b] = int(rng.integers(1, sb + 1))
            elif what == 3:
                slots[base + ln - 1] = np.uint8(rng.integers(0, 256))
            else:
                side[b * codec.side_per_block + int(rng.integers(0, codec.side_per_block))] ^= np.int64(
                    int(rng.integers(1, 1 << 40)))
    cb["out"] = torch.from_numpy(slots).to(codec.device)
    cb["comp_len"] = torch.from_numpy(lens).to(codec.device)
    cb["sidecar"] = torch.from_numpy(side).to(codec.device)
    for use_sidecar in (True, False):
        buf = torch.full((nb * block + 4096,), 0x5A, dtype=torch.uint8, device=codec.device)
        st = torch.full((nb,), 7, dtype=torch.int32, device=codec.device)
        codec.decompress_into(cb, buf[: nb * block], st, use_sidecar=use_sidecar)
        torch.cuda.synchronize()
        assert bool((buf[nb * block:] == 0x5A).all()), "write past the output"
        assert int(st.max()) <= 0, "a block without a status"
    out, side2, st2 = codec.build_sidecar(cb)
    torch.cuda.synchronize()
    assert int(st2.max()) <= 0


def test_large_single_blocks(torch_cuda):
    """Blocks of megabytes (the reference compresses a whole buffer as one
    block, lib.rs:146-183): the host entry points on a 3 MiB + 17 and a 16 MiB
    buffer, and a batch of 8 MiB blocks (ragged last) through every decode
    route: sidecar segments (many rounds per workgroup, payload through the
    global window), sidecar-less serial, and the rebuilt sidecar."""
    torch = torch_cuda
    from entropy_coders_amd import BlockCodec, compress2, decompress2

    for n, p, seed in ((3 * 2**20 + 17, 0.155, 0x1A96E01), (16 * 2**20, 0.5, 0x1A96E02)):
        s = O.generate(0, p, seed, 0, n)
        want, wbits = O.compress2(s)
        got, bits = compress2(s)
        assert got == want and bits == wbits, n
        assert decompress2(got) == s.tobytes(), n
    B = 8 * 2**20
    blocks = [O.generate(0, 0.155, 0x1A96E03, 0, B), O.generate(2, 0.0, 0x1A96E04, 0, B),
              O.generate(0, 0.77, 0x1A96E05, 0, 3 * 2**20 + 5)]
    host = np.concatenate(blocks)
    for ckpt in (64, 256):
        codec = BlockCodec(block_size=B, ckpt_interval=ckpt)
        cb = codec.compress(torch.from_numpy(host).cuda())
        routes = [codec.decompress(cb), codec.decompress(cb, use_sidecar=False)]
        rebuilt = codec.build_sidecar(cb)
        routes.append(rebuilt[::2])
        torch.cuda.synchronize()
        spb = codec.side_per_block
        for b, s in enumerate(blocks):
            want, wbits = O.compress2(s)
            assert int(cb["status"][b]) == 0, (ckpt, b)
            assert codec.block_bytes(cb, b) == want, (ckpt, b)
            assert int(cb["payload_bits"][b]) == wbits, (ckpt, b)
            assert torch.equal(rebuilt[1][b * spb: (b + 1) * spb], cb["sidecar"][b * spb: (b + 1) * spb]), (ckpt, b)
            for r, (out, st) in enumerate(routes):
                assert int(st[b]) == 0, (ckpt, b, r)
                assert torch.equal(out[b * B: b * B + len(s)].cpu(), torch.from_numpy(s)), (ckpt, b, r)


def test_max_block_size(torch_cuda):
    """The largest block the batched path takes (2^28 bytes: bit positions are
    32-bit, fsehip.h), exact against the oracle and decoded through its
    sidecar; one byte-group more is UNSUPPORTED, not a wrong result."""
    torch = torch_cuda
    from entropy_coders_amd import BlockCodec, FseError
    from entropy_coders_amd._lib import STATUS

    B = 1 << 28
    s = O.generate(0, 0.155, 0x1A96E06, 0, B)
    want, wbits = O.compress2(s)
    codec = BlockCodec(block_size=B, ckpt_interval=256)
    src = torch.from_numpy(s).cuda()
    cb = codec.compress(src)
    out, st = codec.decompress(cb)
    torch.cuda.synchronize()
    assert int(cb["status"][0]) == 0 and int(st[0]) == 0
    assert int(cb["payload_bits"][0]) == wbits
    assert codec.block_bytes(cb, 0) == want
    assert torch.equal(out, src)
    with pytest.raises(FseError) as g:
        BlockCodec(block_size=B + 16, ckpt_interval=256).compress(src[:4096])
    assert g.value.code == "UNSUPPORTED"
    # an incompressible 2^28-byte block encodes exactly, but its compressed
    # stream (> 2^28 bytes) is beyond the decoders' 32-bit bit positions:
    # UNSUPPORTED, on every route, never wrong bytes
    del out, src, cb
    s = np.random.default_rng(7).integers(0, 256, B, dtype=np.uint8)
    want, wbits = O.compress2(s)
    assert len(want) > B
    cb = codec.compress(torch.from_numpy(s).cuda())
    assert int(cb["status"][0]) == 0 and codec.block_bytes(cb, 0) == want
    for use_sidecar in (True, False):
        _, st = codec.decompress(cb, use_sidecar=use_sidecar)
        assert STATUS.get(int(st[0])) == "UNSUPPORTED", use_sidecar


def test_large_blocks_one_state(torch_cuda):
    """The 1-state format (fse_compress, lib.rs:112-143) on megabyte blocks:
    the host calls on 5 MiB, and 8 MiB batch blocks through every route."""
    torch = torch_cuda
    from entropy_coders_amd import BlockCodec, compress, decompress

    s = O.generate(0, 0.3, 0x1A96E07, 0, 5 * 2**20 + 3)
    want, wbits = O.compress(s)
    got, bits = compress(s)
    assert got == want and bits == wbits
    assert decompress(got) == s.tobytes()
    B = 8 * 2**20
    blocks = [O.generate(0, 0.155, 0x1A96E08, 0, B), O.generate(0, 0.6, 0x1A96E09, 0, 2**20 + 9)]
    host = np.concatenate(blocks)
    codec = BlockCodec(block_size=B, ckpt_interval=128, nstates=1)
    cb = codec.compress(torch.from_numpy(host).cuda())
    routes = [codec.decompress(cb), codec.decompress(cb, use_sidecar=False)]
    rebuilt = codec.build_sidecar(cb)
    routes.append(rebuilt[::2])
    torch.cuda.synchronize()
    spb = codec.side_per_block
    for b, s in enumerate(blocks):
        want, wbits = O.compress(s)
        assert int(cb["status"][b]) == 0, b
        assert codec.block_bytes(cb, b) == want, b
        assert int(cb["payload_bits"][b]) == wbits, b
        assert torch.equal(rebuilt[1][b * spb: (b + 1) * spb], cb["sidecar"][b * spb: (b + 1) * spb]), b
        for r, (out, st) in enumerate(routes):
            assert int(st[b]) == 0, (b, r)
            assert torch.equal(out[b * B: b * B + len(s)].cpu(), torch.from_numpy(s)), (b, r)
