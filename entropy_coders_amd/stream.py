"""Host-streaming pipeline: inputs that live in host
memory, not HBM.

The data is cut into chunks of `chunk_blocks` blocks.  Three HIP streams
overlap the PCIe copies with the kernels: while chunk i is encoded (or
decoded), chunk i+1 is copied in and chunk i-1 is copied out.  Every
buffer is double-buffered and reuse is ordered by events, so the host
thread never waits for the GPU except to learn a chunk's compressed size
(compress only), and by then the next chunk's work is already queued.

Wire format of a compressed stream (the same as `dist.pack_device`):
blocks back to back (each an exact `fse_compress2` block), plus the
per-block lengths and the per-block sidecar (decode checkpoints; see
DESIGN.md "sidecar").  `compress` returns host tensors; `decompress` takes
them back.  Host buffers should be pinned for the copies to overlap; the
class pins its own outputs.

The pipeline drives the same C ABI as everything else (libfsehip.so); it
adds no compute of its own.
"""
from __future__ import annotations

import ctypes as C

import torch

from ._lib import check
from .fse import BlockCodec


def _ptr(t: torch.Tensor) -> C.c_void_p:
    return C.c_void_p(t.data_ptr())


class HostPipeline:
    """Chunked, stream-overlapped compress/decompress of host-resident data."""

    def __init__(self, codec: BlockCodec, chunk_blocks: int = 1024):
        self.codec = codec
        self.torch = torch
        self.dev = codec.device
        self.cbk = chunk_blocks
        self.chunk_bytes = chunk_blocks * codec.block_size
        self.s_in = torch.cuda.Stream(self.dev)
        self.s_comp = torch.cuda.Stream(self.dev)
        self.s_out = torch.cuda.Stream(self.dev)
        spb = max(codec.side_per_block, 1)
        t = torch
        self.sets = []
        for _ in range(2):
            cb = codec.alloc(self.chunk_bytes)
            self.sets.append({
                "raw": t.empty(self.chunk_bytes, dtype=t.uint8, device=self.dev),
                "cb": cb,
                "packed": t.empty(chunk_blocks * codec.slot_bytes, dtype=t.uint8, device=self.dev),
                "offsets": t.zeros(chunk_blocks, dtype=t.int64, device=self.dev),
                "total": t.zeros(1, dtype=t.int64, device=self.dev),
                "h_total": t.zeros(1, dtype=t.int64, pin_memory=True),
                "status": t.zeros(chunk_blocks, dtype=t.int32, device=self.dev),
                "side_n": spb,
                "ev_in": torch.cuda.Event(),
                "ev_comp": torch.cuda.Event(),
                "ev_out": torch.cuda.Event(),
            })

    # -- helpers ----------------------------------------------------------
    def _chunks(self, n_total: int):
        nb = self.codec.n_blocks(n_total)
        for i, b0 in enumerate(range(0, nb, self.cbk)):
            b1 = min(b0 + self.cbk, nb)
            r0 = b0 * self.codec.block_size
            r1 = min(b1 * self.codec.block_size, n_total)
            yield i, b0, b1, r0, r1

    def _pack(self, st: dict, nblk: int) -> None:
        """Slots -> packed bytes on the compute stream; total length on the device."""
        codec = self.codec
        lens = st["cb"]["comp_len"][:nblk].to(torch.int64)
        off = st["offsets"][:nblk]
        off.zero_()
        if nblk > 1:
            torch.cumsum(lens[:-1], 0, out=off[1:])
        st["total"].copy_(off[nblk - 1:nblk] + lens[nblk - 1:nblk])
        hs = C.c_void_p(torch.cuda.current_stream(self.dev).cuda_stream)
        check(codec.lib.fsehip_pack_blocks(_ptr(st["cb"]["out"]), codec.slot_bytes, _ptr(st["cb"]["comp_len"]),
                                           _ptr(off), nblk, _ptr(st["packed"]), hs), "fsehip_pack_blocks")

    # -- compress ---------------------------------------------------------
    def alloc_compress_out(self, n_total: int) -> dict:
        """Pinned host outputs for `compress` of n_total bytes (pinning is
        slow: allocate once, reuse)."""
        codec, t = self.codec, torch
        nb = codec.n_blocks(n_total)
        spb = max(codec.side_per_block, 1)
        return {"stream": t.empty(max(nb * codec.slot_bytes, 1), dtype=t.uint8, pin_memory=True),
                "lens": t.empty(nb, dtype=t.int32, pin_memory=True),
                "side": t.empty(nb * spb, dtype=t.int64, pin_memory=True),
                "status": t.empty(nb, dtype=t.int32, pin_memory=True)}

    def compress(self, host_src: torch.Tensor, out: dict | None = None):
        """host_src: 1-D uint8 CPU tensor (pinned for overlap).  Returns
        (stream, lens, sidecar, status) host tensors (views of `out` when
        given); stream holds the blocks back to back."""
        codec = self.codec
        n = host_src.numel()
        spb = max(codec.side_per_block, 1)
        out = out or self.alloc_compress_out(n)
        out_stream, out_lens, out_side, out_status = out["stream"], out["lens"], out["side"], out["status"]
        pos = 0
        pending = None  # (set, b0, b1) whose output is not yet queued

        def drain(item):
            nonlocal pos
            st, b0, b1 = item
            st["ev_comp"].synchronize()  # the next chunk's work is already queued
            total = int(st["h_total"][0])
            with torch.cuda.stream(self.s_out):
                self.s_out.wait_event(st["ev_comp"])
                nblk = b1 - b0
                out_stream[pos:pos + total].copy_(st["packed"][:total], non_blocking=True)
                out_lens[b0:b1].copy_(st["cb"]["comp_len"][:nblk], non_blocking=True)
                if codec.side_per_block:
                    out_side[b0 * spb:b1 * spb].copy_(st["cb"]["sidecar"][:nblk * spb], non_blocking=True)
                out_status[b0:b1].copy_(st["cb"]["status"][:nblk], non_blocking=True)
                st["ev_out"].record(self.s_out)
            pos += total

        for i, b0, b1, r0, r1 in self._chunks(n):
            st = self.sets[i & 1]
            nblk = b1 - b0
            with torch.cuda.stream(self.s_in):
                self.s_in.wait_event(st["ev_comp"])  # chunk i-2's kernels are done with raw
                st["raw"][:r1 - r0].copy_(host_src[r0:r1], non_blocking=True)
                st["ev_in"].record(self.s_in)
            with torch.cuda.stream(self.s_comp):
                self.s_comp.wait_event(st["ev_in"])
                self.s_comp.wait_event(st["ev_out"])  # chunk i-2's results have left
                cb = st["cb"]
                cb["n_total"] = r1 - r0
                codec.compress_into(st["raw"], cb)
                self._pack(st, nblk)
                st["h_total"].copy_(st["total"], non_blocking=True)
                st["ev_comp"].record(self.s_comp)
            if pending is not None:
                drain(pending)
            pending = (st, b0, b1)
        if pending is not None:
            drain(pending)
        self.s_out.synchronize()
        nb = codec.n_blocks(n)
        return out_stream[:pos], out_lens[:nb], out_side[:nb * spb], out_status[:nb]

    # -- decompress -------------------------------------------------------
    def alloc_decompress_out(self, n_total: int) -> dict:
        t = torch
        return {"raw": t.empty(max(n_total, 1), dtype=t.uint8, pin_memory=True),
                "status": t.empty(max(self.codec.n_blocks(n_total), 1), dtype=t.int32, pin_memory=True)}

    def decompress(self, stream: torch.Tensor, lens: torch.Tensor, side: torch.Tensor, n_total: int,
                   out: dict | None = None):
        """Inverse of `compress`: (stream, lens, sidecar) host tensors ->
        (raw, status) host tensors (views of `out` when given)."""
        codec = self.codec
        spb = max(codec.side_per_block, 1)
        t = torch
        lens64 = lens.to(t.int64)
        offs = t.zeros_like(lens64)
        if len(lens64) > 1:
            offs[1:] = t.cumsum(lens64, 0)[:-1]
        o = out or self.alloc_decompress_out(n_total)
        out, status = o["raw"][:n_total], o["status"][:codec.n_blocks(n_total)]
        for i, b0, b1, r0, r1 in self._chunks(n_total):
            st = self.sets[i & 1]
            nblk = b1 - b0
            c0 = int(offs[b0])
            c1 = int(offs[b1 - 1] + lens64[b1 - 1])
            cb = st["cb"]
            with torch.cuda.stream(self.s_in):
                self.s_in.wait_event(st["ev_comp"])  # chunk i-2's kernels are done with these buffers
                st["packed"][:c1 - c0].copy_(stream[c0:c1], non_blocking=True)
                cb["comp_len"][:nblk].copy_(lens[b0:b1], non_blocking=True)
                if codec.side_per_block:
                    cb["sidecar"][:nblk * spb].copy_(side[b0 * spb:b1 * spb], non_blocking=True)
                st["offsets"][:nblk].copy_(offs[b0:b1] - c0, non_blocking=True)
                st["ev_in"].record(self.s_in)
            with torch.cuda.stream(self.s_comp):
                self.s_comp.wait_event(st["ev_in"])
                self.s_comp.wait_event(st["ev_out"])  # chunk i-2's raw output has left
                hs = C.c_void_p(self.s_comp.cuda_stream)
                check(codec.lib.fsehip_unpack_blocks(_ptr(st["packed"]), _ptr(st["offsets"]), _ptr(cb["comp_len"]),
                                                     nblk, _ptr(cb["out"]), codec.slot_bytes, hs),
                      "fsehip_unpack_blocks")
                cb["n_total"] = r1 - r0
                codec.decompress_into(cb, st["raw"], st["status"])
                st["ev_comp"].record(self.s_comp)
            with torch.cuda.stream(self.s_out):
                self.s_out.wait_event(st["ev_comp"])
                out[r0:r1].copy_(st["raw"][:r1 - r0], non_blocking=True)
                status[b0:b1].copy_(st["status"][:nblk], non_blocking=True)
                st["ev_out"].record(self.s_out)
        self.s_out.synchronize()
        return out, status


__all__ = ["HostPipeline"]
