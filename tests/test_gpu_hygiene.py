"""Product hygiene at the boundary (GPU): the product library ignores the
diagnostics environment knobs (an ablation variable in the caller's
environment cannot change a block's bytes), and the decode workspace can be
released and re-grown."""
import os
import subprocess
import sys

import numpy as np
import pytest

from oracle import oracle as O

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def torch_cuda():
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch


_CHILD = r"""
import numpy as np, torch
from oracle import oracle as O
from entropy_coders_amd import BlockCodec, compress2, decompress2
import entropy_coders_amd._lib as L
assert L.LIB_PATH.endswith("/libfsehip.so"), L.LIB_PATH
src = np.concatenate([O.generate(0, 0.155, 0x5EED0002, b, 65536) for b in range(6)] + [O.generate(0, 0.77, 7, 0, 40001)])
codec = BlockCodec(ckpt_interval=64)
d = torch.from_numpy(src).cuda()
cb = codec.compress(d)
out, st = codec.decompress(cb)
out2, st2 = codec.decompress(cb, use_sidecar=False)
torch.cuda.synchronize()
assert int(cb["status"].abs().max()) == 0 and int(st.abs().max()) == 0 and int(st2.abs().max()) == 0
assert torch.equal(out[: len(src)], d) and torch.equal(out2[: len(src)], d)
for b in range(7):
    blk = src[b * 65536:(b + 1) * 65536]
    assert codec.block_bytes(cb, b) == O.compress2(blk)[0], b
bp, s0, s1 = O.checkpoints2(O.compress2(src[:65536])[0], 64)
side = cb["sidecar"][: len(bp)].cpu().numpy().view(np.uint64)
assert np.array_equal(side & 0xFFFFFFFF, bp.astype(np.uint64))
assert np.array_equal((side >> 32) & 0xFFFF, s0.astype(np.uint64)) and np.array_equal(side >> 48, s1.astype(np.uint64))
comp, bits = compress2(src[:65536])
assert (comp, bits) == O.compress2(src[:65536]) and decompress2(comp) == src[:65536].tobytes()
print("child-ok")
"""


def test_product_ignores_diagnostic_knobs(torch_cuda):
    """Every knob the diagnostics build reads, set in a child process's
    environment to its output-changing value (FSEHIP_DEBUG=16 skips the
    encoder's repair rounds, 4 drops its payload stores, 2 forces the
    too-small path; FSEHIP_ENC_LANES=32, FSEHIP_SERIAL_DEFER=0,
    FSEHIP_SERIAL_DW=2, the occupancy paddings): the product library still
    writes the oracle's bytes, sidecar and round trips."""
    env = dict(os.environ, PYTHONPATH=ROOT, FSEHIP_DEBUG="30", FSEHIP_ENC_LANES="32", FSEHIP_SERIAL_DEFER="0",
               FSEHIP_SERIAL_DW="2", FSEHIP_ENC_XLDS="60000", FSEHIP_DT_XLDS="60000", FSEHIP_STAMPS="1",
               FSEHIP_RANK_INJECT="1")
    env.pop("FSEHIP_LIB", None)
    r = subprocess.run([sys.executable, "-c", _CHILD], cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and "child-ok" in r.stdout, (r.stdout[-2000:], r.stderr[-4000:])
    assert "[stamps]" not in r.stderr


def test_release_workspace_and_decode_again(torch_cuda):
    """fsehip_release_workspace frees the stream's decode workspace (tables,
    deferred-symbol states); the next sidecar-less and sidecar decodes
    allocate again and are exact.  Releasing twice, and for every device, is
    fine."""
    torch = torch_cuda
    from entropy_coders_amd import BlockCodec
    from entropy_coders_amd._lib import load

    codec = BlockCodec(ckpt_interval=64)
    src = codec.generate(0, 0.155, 0x5EED0042, 48 * 65536 + 999)
    cb = codec.compress(src)
    for rep in range(3):
        out, st = codec.decompress(cb, use_sidecar=False)
        torch.cuda.synchronize()
        assert int(st.abs().max()) == 0 and torch.equal(out, src), rep
        codec.release_workspace()
        codec.release_workspace()
        out, st = codec.decompress(cb)
        torch.cuda.synchronize()
        assert int(st.abs().max()) == 0 and torch.equal(out, src), rep
    assert load().fsehip_release_workspace(-1, None) == 0
    out, st = codec.decompress(cb, use_sidecar=False)
    torch.cuda.synchronize()
    assert torch.equal(out, src)
    assert codec.block_bytes(cb, 3) == O.compress2(src[3 * 65536: 4 * 65536].cpu().numpy())[0]


def test_reference_kats_through_hip_normalize(torch_cuda):
    """The crate's known-answer tests uniform_dist_256 and exp_dist
    (histogram.rs:595-656) through the HIP Histogram::new (histogram_new),
    Histogram::normalize (histogram_normalize) and NormHistogram::write/read,
    beside the oracle: a flat histogram normalises to 2^(L-8) per symbol at
    L = max(log2, 9); the exponential one to 2^L >> (1 + j) below log2 - 1
    and -1 for its two unit counts; then hist_verify's properties
    (histogram.rs:553-587: sum of |norm| = 2^L, the zero pattern, the header
    round trip leaving trailing bytes untouched)."""
    from entropy_coders_amd import histogram_new, norm_histogram_read, norm_histogram_write, normalize

    def verify(h, nh, log2):
        norm = list(nh.norm)
        onh, _ = O.normalize(O.hist_count(bytes(data)), log2)
        assert norm == list(onh.norm) and nh.log2 == onh.log2
        assert sum(abs(v) for v in norm) == 1 << nh.log2
        assert all((c == 0) == (v == 0) for c, v in zip(h.counts, norm))
        hdr, _ = norm_histogram_write(nh)
        assert hdr == O.header_write(onh)
        test = b"I am a test"
        back, used = norm_histogram_read(hdr + test)
        assert (hdr + test)[used:] == test
        assert list(back.norm) == norm and back.log2 == nh.log2 and back.table_len == nh.table_len

    for log2 in range(8, 16):  # uniform_dist_256 (histogram.rs:595-619)
        data = b"".join(bytes([x]) * (1 << (log2 - 8)) for x in range(256))
        h = histogram_new(data)
        assert list(h.counts) == [1 << (log2 - 8)] * 256 and h.table_len == 256
        nh = normalize(h, log2)
        L = max(log2, 9)
        assert nh.log2 == L and list(nh.norm) == [1 << (L - 8)] * 256, log2
        verify(h, nh, log2)
    for log2 in range(8, 16):  # exp_dist (histogram.rs:621-656)
        size = 1 << log2
        rem, data, sym = size, [], 0
        while True:
            data += [sym] * (rem >> 1)
            rem -= rem >> 1
            sym += 1
            if rem == 1:
                data.append(sym)
                break
        data = bytes(data)
        h = histogram_new(data)
        assert list(h.counts) == [(size >> (1 + j)) if j < log2 else (1 if j == log2 else 0) for j in range(256)]
        nh = normalize(h, log2)
        assert list(nh.norm)[: log2 + 1] == [size >> (1 + j) for j in range(log2 - 1)] + [-1, -1], log2
        assert all(v == 0 for v in list(nh.norm)[log2 + 1:])
        verify(h, nh, log2)


@pytest.mark.parametrize("nstates", [2, 1])
def test_host_calls_past_the_pinned_window(torch_cuda, nstates):
    """Per-call entry points whose compressed and decoded bytes exceed the 4 MiB
    pinned return window (fse_capi.cpp kPinOut): the head comes back through
    pinned memory, the rest by a device-to-host copy; bytes equal the oracle's
    and the stream decodes back exactly (near-uniform data, ~1 B per byte)."""
    from entropy_coders_amd import compress, compress2, decompress, decompress2

    src = O.generate(2, 0.0, 0x5EED0007, 0, (6 << 20) + 12345)
    if nstates == 2:
        comp, bits = compress2(src)
        assert (comp, bits) == O.compress2(src)
        assert len(comp) > (4 << 20)
        assert decompress2(comp, cap=len(src) + 64) == src.tobytes()
    else:
        comp, bits = compress(src)
        assert (comp, bits) == O.compress(src)
        assert len(comp) > (4 << 20)
        assert decompress(comp, cap=len(src) + 64) == src.tobytes()
