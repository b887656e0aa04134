"""GPU parity for the 1-state format (`fse_compress` / `fse_decompress`,
lib.rs:112-143 / lib.rs:187-212): bytes equal to the oracle's, round trips
through both decoders (serial reference-order, and the sidecar segment
decoder), and the sidecar equal to the oracle's decode checkpoints.
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


def test_compress_golden(torch_cuda, golden):
    from entropy_coders_amd import compress, decompress

    manifest, arrays = golden
    seen = 0
    for case in manifest["cases"]:
        if case["format"] != 1:
            continue
        src = arrays[case["name"] + "__src"]
        want = arrays[case["name"] + "__comp"].tobytes()
        got, bits = compress(src)
        assert got == want, case["name"]
        assert bits == case["payload_bits"], case["name"]
        assert decompress(want) == src.tobytes(), case["name"]
        seen += 1
    assert seen >= 2


@pytest.mark.parametrize("n", [2, 3, 4, 5, 15, 16, 17, 18, 31, 32, 33, 47, 63, 64, 65, 127, 255, 256,
                               257, 1000, 1001, 4095, 4097, 65535, 65536, 65537, 200003])
def test_compress_lengths(torch_cuda, n):
    from entropy_coders_amd import compress, decompress

    src = O.generate(0, 0.2, 91, n, n)
    if len(set(src.tolist())) == 1:
        src[0] ^= 1
    want, wbits = O.compress(src)
    got, bits = compress(src)
    assert got == want and bits == wbits
    assert decompress(got) == src.tobytes()


@pytest.mark.parametrize("kind,prob", [(1, 0.5), (2, 0.0), (0, 0.77), (0, 0.02)])
def test_compress_distributions(torch_cuda, kind, prob):
    from entropy_coders_amd import compress, decompress

    src = O.generate(kind, prob, 7, 3, 50001)
    want, wbits = O.compress(src)
    got, bits = compress(src)
    assert got == want and bits == wbits
    assert decompress(got) == src.tobytes()


def test_edge_inputs_match_oracle(torch_cuda):
    """Every edge input either encodes to the oracle's bytes or fails with
    the oracle's status (a reference panic / None)."""
    from entropy_coders_amd import FseError, compress, decompress

    cases = [b"", b"\x07", b"\x07\x08", b"\x08\x07", bytes(100), b"\x09" * 100, b"\x00" * 99 + b"\x01",
             bytes(range(256)), b"\xff\x00" * 8]
    for data in cases:
        try:
            want = O.compress(data)
        except O.OracleError as e:
            with pytest.raises(FseError) as g:
                compress(data)
            assert g.value.code == e.code, data[:8]
            continue
        got = compress(data)
        assert got == want, data[:8]
        try:
            wdec = O.decompress(want[0])
        except O.OracleError as e:
            with pytest.raises(FseError) as g:
                decompress(want[0])
            assert g.value.code == e.code, data[:8]
            continue
        assert decompress(want[0]) == wdec, data[:8]


def test_decompress_errors(torch_cuda):
    from entropy_coders_amd import FseError, compress, decompress

    comp, _ = compress(b"\x09" * 100)
    with pytest.raises(FseError) as e:
        decompress(comp)
    assert e.value.code == "SINGLE_SYMBOL"
    src = O.generate(0, 0.3, 1, 0, 3000)
    comp, _ = compress(src)
    for bad in (comp[:-1] + b"\x00", b"\x00"):
        try:
            O.decompress(bad)
            want = None
        except O.OracleError as oe:
            want = oe.code
        if want is None:
            assert decompress(bad) == O.decompress(bad)
        else:
            with pytest.raises(FseError) as g:
                decompress(bad)
            assert g.value.code == want
    with pytest.raises(FseError) as e:
        decompress(comp, cap=100)
    assert e.value.code == "DST_TOO_SMALL"


def _batched(torch, kind, prob, n_total, block=65536, seed=0x5EED1001, ckpt=64, check_all=True):
    from entropy_coders_amd import BlockCodec

    codec = BlockCodec(block_size=block, ckpt_interval=ckpt, nstates=1)
    src = codec.generate(kind, prob, seed, n_total)
    cb = codec.compress(src)
    out, st = codec.decompress(cb)  # sidecar segment decoder
    out2, st2 = codec.decompress(cb, use_sidecar=False)  # serial, reference order
    out3, side3, st3 = codec.build_sidecar(cb)  # serial, recording the checkpoints
    torch.cuda.synchronize()
    assert int(cb["status"].abs().max()) == 0, cb["status"].cpu().numpy()[:8]
    assert int(st.abs().max()) == 0, st.cpu().numpy()[:8]
    assert int(st2.abs().max()) == 0, st2.cpu().numpy()[:8]
    assert int(st3.abs().max()) == 0, st3.cpu().numpy()[:8]
    assert torch.equal(out, src)
    assert torch.equal(out2, src)
    assert torch.equal(out3, src)
    nb = codec.n_blocks(n_total)
    spb = codec.side_per_block
    assert torch.equal(side3[: nb * spb], cb["sidecar"][: nb * spb]), "rebuilt sidecar != encoder sidecar"
    host = src.cpu().numpy()
    blocks = range(nb) if check_all else sorted({0, nb // 2, nb - 1})
    for b in blocks:
        s = host[b * block: (b + 1) * block]
        want, wbits = O.compress(s)
        assert codec.block_bytes(cb, b) == want, f"block {b}"
        assert int(cb["payload_bits"][b]) == wbits
        bp, s0 = O.checkpoints1(want, ckpt)
        side = cb["sidecar"][b * codec.side_per_block: b * codec.side_per_block + len(bp)].cpu().numpy()
        side = side.view(np.uint64)
        assert np.array_equal(side & 0xFFFFFFFF, bp.astype(np.uint64)), f"bitpos block {b}"
        assert np.array_equal((side >> 32) & 0xFFFF, s0.astype(np.uint64)), f"state block {b}"
        assert np.all((side >> 48) == 0)
    return codec, cb


def test_batched_onestate_c2(torch_cuda):
    _batched(torch_cuda, 0, 0.155, 16 * 65536 + 12345)


@pytest.mark.parametrize("ckpt", [16, 128, 1024])
def test_batched_onestate_ckpt(torch_cuda, ckpt):
    _batched(torch_cuda, 1, 0.5, 4 * 65536 + 777, ckpt=ckpt)


def test_batched_onestate_small_blocks(torch_cuda):
    _batched(torch_cuda, 0, 0.3, 64 * 4096 + 33, block=4096, ckpt=16)


def test_batched_onestate_prebuilt_tables(torch_cuda):
    torch = torch_cuda
    codec, cb = _batched(torch, 2, 0.0, 8 * 65536, check_all=False)
    tabs = codec.build_dtables(cb)
    for use_side in (True, False):
        out = torch.empty(cb["n_total"], dtype=torch.uint8, device=codec.device)
        st = torch.zeros(codec.n_blocks(cb["n_total"]), dtype=torch.int32, device=codec.device)
        codec.decompress_dt_into(cb, tabs, out, st, use_sidecar=use_side)
        torch.cuda.synchronize()
        assert int(st.abs().max()) == 0
        src = codec.generate(2, 0.0, 0x5EED1001, cb["n_total"])
        assert torch.equal(out, src)


def test_headerless_variant(torch_cuda):
    """The crate's test-module 1-state codec (fse.rs:394-434) writes the
    fse_compress stream without a header: the GPU fse_compress bytes after the
    header are exactly that stream, and a headerless stream decodes once its
    NormHistogram is written in front of it (norm_histogram_write)."""
    from oracle import spec as S
    from entropy_coders_amd import compress_nh, decompress, norm_histogram_write

    for prob, n in ((0.2, 1 << 15), (0.5, 333), (0.05, 4096)):
        src = O.generate(0, prob, 0x5EED0001, 0, n).tobytes()
        norm, L, tl, payload, bits = S.compress_headerless(src)
        comp, cbits, nh = compress_nh(src)
        head, _ = norm_histogram_write(nh)
        assert comp == head + payload and cbits == bits
        assert decompress(head + payload) == src
