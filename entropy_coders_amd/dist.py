"""Multi-GPU sharding of independent blocks (one process per GPU).

Blocks of the reference format carry no cross-block state (lib.rs:146-183
compresses one slice into one self-contained block), so the data path needs
no collective: each rank compresses / decompresses its own shard of blocks.
The exchanges are around the data path:

- gather_stream: every rank's packed compressed shard (plus block lengths and
  the sidecar) to one rank.  A gatherv: an all_gather of the sizes, then one
  batch of point-to-point sends/receives of exactly those sizes
  (dist.batch_isend_irecv; ncclGroupStart + ncclSend/ncclRecv under RCCL),
  no padding to the largest rank.
- scatter_stream: the reverse, for distributed decode: one rank holds a
  packed stream of every block, each rank receives its blocks.

Both are timed separately from the throughput metric.  Everything here is
backend-agnostic torch.distributed code over tensors: RCCL ("nccl") with
device tensors on MI355X, gloo with CPU tensors in the CPU tests.
"""
from __future__ import annotations

import torch
import torch.distributed as dist

# message tags (gloo matches point-to-point messages by tag; RCCL ignores them)
_TAG_LENS, _TAG_DATA, _TAG_SIDE = 11, 12, 13


def rank_blocks(n_blocks: int, rank: int, world: int, scheme: str = "contiguous") -> range:
    """Global block indices owned by `rank`.

    contiguous: rank r owns [r*q + min(r, m), ...) (q, m = divmod(n, world));
    round_robin: rank r owns r, r + world, r + 2*world, ... (C4: block b on GPU b mod 8)
    """
    if scheme == "round_robin":
        return range(rank, n_blocks, world)
    if scheme != "contiguous":
        raise ValueError(f"unknown scheme {scheme!r}")
    q, m = divmod(n_blocks, world)
    start = rank * q + min(rank, m)
    return range(start, start + q + (1 if rank < m else 0))


def exclusive_offsets(comp_len: torch.Tensor) -> torch.Tensor:
    """Byte offsets of blocks packed back to back (exclusive scan, int64)."""
    lens = comp_len.to(torch.int64)
    offsets = torch.zeros_like(lens)
    if len(lens) > 1:
        offsets[1:] = torch.cumsum(lens, 0)[:-1]
    return offsets


def pack_host(slots: torch.Tensor, slot_bytes: int, comp_len: torch.Tensor):
    """Reference (torch) packer: slot layout -> (stream, offsets).  Used on
    CPU tensors in tests; on the GPU use `pack_device` (HIP kernel)."""
    offsets = exclusive_offsets(comp_len)
    lens = comp_len.to(torch.int64)
    stream = torch.empty(int(lens.sum()), dtype=torch.uint8, device=slots.device)
    for b in range(len(lens)):
        n = int(lens[b])
        o = int(offsets[b])
        stream[o:o + n] = slots[b * slot_bytes: b * slot_bytes + n]
    return stream, offsets


def _hip():
    import ctypes as C

    from ._lib import check, load

    return C, check, load()


def pack_device(slots: torch.Tensor, slot_bytes: int, comp_len: torch.Tensor):
    """Slot layout -> contiguous stream on the GPU (fsehip_pack_blocks)."""
    C, check, lib = _hip()
    offsets = exclusive_offsets(comp_len)
    total = int(comp_len.to(torch.int64).sum())
    stream = torch.empty(max(total, 1), dtype=torch.uint8, device=slots.device)
    hs = C.c_void_p(torch.cuda.current_stream(slots.device).cuda_stream)
    check(lib.fsehip_pack_blocks(C.c_void_p(slots.data_ptr()), slot_bytes,
                                 C.c_void_p(comp_len.data_ptr()), C.c_void_p(offsets.data_ptr()),
                                 len(comp_len), C.c_void_p(stream.data_ptr()), hs), "fsehip_pack_blocks")
    return stream[:total], offsets


def unpack_device(stream: torch.Tensor, comp_len: torch.Tensor, slot_bytes: int) -> torch.Tensor:
    """Packed stream -> slot layout on the GPU (fsehip_unpack_blocks), ready
    for fsehip_decompress_blocks."""
    C, check, lib = _hip()
    lens = comp_len.to(device=stream.device, dtype=torch.int32).contiguous()
    offsets = exclusive_offsets(lens)
    slots = torch.zeros(max(len(lens), 1) * slot_bytes, dtype=torch.uint8, device=stream.device)
    hs = C.c_void_p(torch.cuda.current_stream(stream.device).cuda_stream)
    check(lib.fsehip_unpack_blocks(C.c_void_p(stream.data_ptr()), C.c_void_p(offsets.data_ptr()),
                                   C.c_void_p(lens.data_ptr()), len(lens), C.c_void_p(slots.data_ptr()),
                                   slot_bytes, hs), "fsehip_unpack_blocks")
    return slots


def select_blocks(stream: torch.Tensor, offsets: torch.Tensor, comp_len: torch.Tensor, idx) -> torch.Tensor:
    """The bytes of blocks `idx` (in that order) out of a packed stream, packed
    back to back.  Device tensors: one fsehip_copy_blocks launch; CPU tensors
    (gloo tests): slicing."""
    idx_t = torch.as_tensor(list(idx) if not isinstance(idx, torch.Tensor) else idx, dtype=torch.int64)
    lens = comp_len.to(torch.int64).cpu()[idx_t]
    total = int(lens.sum())
    out = torch.empty(max(total, 1), dtype=torch.uint8, device=stream.device)
    if len(idx_t) == 0:
        return out[:0]
    if stream.is_cuda:
        C, check, lib = _hip()
        dev = stream.device
        src_off = offsets.to(dev, torch.int64)[idx_t.to(dev)].contiguous()
        dst_off = exclusive_offsets(lens).to(dev)
        l32 = lens.to(device=dev, dtype=torch.int32)
        hs = C.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
        check(lib.fsehip_copy_blocks(C.c_void_p(stream.data_ptr()), C.c_void_p(src_off.data_ptr()),
                                     C.c_void_p(l32.data_ptr()), len(idx_t), C.c_void_p(out.data_ptr()),
                                     C.c_void_p(dst_off.data_ptr()), hs), "fsehip_copy_blocks")
    else:
        offs = offsets.to(torch.int64).cpu()
        o = 0
        for b, n in zip(idx_t.tolist(), lens.tolist()):
            out[o:o + n] = stream[int(offs[b]): int(offs[b]) + n]
            o += n
    return out[:total]


def _all_sizes(vals, dev, group):
    world = dist.get_world_size(group)
    mine = torch.tensor(vals, dtype=torch.int64, device=dev)
    allv = [torch.zeros_like(mine) for _ in range(world)]
    dist.all_gather(allv, mine, group=group)
    return [[int(x) for x in v.cpu()] for v in allv]


def _run_p2p(ops) -> None:
    ops = [op for op in ops if op.tensor.numel() > 0]
    if ops:
        for req in dist.batch_isend_irecv(ops):
            req.wait()


def gather_stream(stream: torch.Tensor, comp_len: torch.Tensor, dst: int = 0, group=None, sidecar=None):
    """Gather every rank's packed compressed stream, block lengths and
    (optionally) sidecar on `dst` -- a gatherv.

    Step 1: all_gather of each rank's (n_blocks, bytes, sidecar entries).
    Step 2: one batch of point-to-point transfers of exactly those sizes:
    every other rank sends, `dst` posts one receive per rank and message.
    Returns (streams, lens[, sidecars]) lists indexed by rank on `dst`
    (its own entries are its inputs, not copies), Nones elsewhere.
    """
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    dev = stream.device
    lens32 = comp_len.to(device=dev, dtype=torch.int32).contiguous()
    side = sidecar.contiguous() if sidecar is not None else None
    sizes = _all_sizes([lens32.numel(), stream.numel(), side.numel() if side is not None else 0], dev, group)
    peer = (lambda r: dist.get_global_rank(group, r)) if group is not None else (lambda r: r)
    ops = []
    if rank == dst:
        streams, lens, sides = [None] * world, [None] * world, [None] * world
        for r in range(world):
            nb, nbytes, nside = sizes[r]
            if r == dst:
                streams[r], lens[r], sides[r] = stream, lens32, side
                continue
            lens[r] = torch.empty(nb, dtype=torch.int32, device=dev)
            streams[r] = torch.empty(nbytes, dtype=torch.uint8, device=dev)
            ops.append(dist.P2POp(dist.irecv, lens[r], peer(r), group, _TAG_LENS))
            ops.append(dist.P2POp(dist.irecv, streams[r], peer(r), group, _TAG_DATA))
            if side is not None:
                sides[r] = torch.empty(nside, dtype=torch.int64, device=dev)
                ops.append(dist.P2POp(dist.irecv, sides[r], peer(r), group, _TAG_SIDE))
    else:
        ops.append(dist.P2POp(dist.isend, lens32, peer(dst), group, _TAG_LENS))
        ops.append(dist.P2POp(dist.isend, stream.contiguous(), peer(dst), group, _TAG_DATA))
        if side is not None:
            ops.append(dist.P2POp(dist.isend, side, peer(dst), group, _TAG_SIDE))
    _run_p2p(ops)
    if rank != dst:
        return (None, None, None) if sidecar is not None else (None, None)
    return (streams, lens, sides) if sidecar is not None else (streams, lens)


def scatter_stream(stream, comp_len, src: int = 0, group=None, sidecar=None, side_per_block: int = 0,
                   scheme: str = "contiguous", device=None):
    """Distributed decode's input exchange: `src` holds one packed stream of
    every block (global block order, as `assemble` indexes a gather) with
    its block lengths and optionally the sidecar ([n_blocks * side_per_block]
    int64); each rank receives its blocks (`rank_blocks(scheme)`).

    Step 1: broadcast of the block count, then of the length array (4 B per
    block), so every rank knows its blocks and sizes.  Step 2: `src` selects
    each rank's blocks (contiguous ranges are slices; round-robin shards go
    through fsehip_copy_blocks on the GPU) and one batch of point-to-point
    transfers delivers them.  Other ranks pass None for stream/comp_len/sidecar
    and give `device` (default: their current GPU under the nccl/RCCL
    backend; required under gloo).
    Returns (stream, comp_len int32, sidecar or None, global block indices).
    """
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    if device is not None:
        dev = torch.device(device)
    elif stream is not None:
        dev = stream.device
    elif dist.get_backend(group) == "nccl":  # RCCL moves device tensors: this rank's current GPU
        dev = torch.device("cuda", torch.cuda.current_device())
    else:
        raise ValueError("scatter_stream: a rank without the stream must pass device= (gloo: 'cpu')")
    peer = (lambda r: dist.get_global_rank(group, r)) if group is not None else (lambda r: r)
    hdr = torch.zeros(3, dtype=torch.int64, device=dev)
    if rank == src:
        hdr[0] = comp_len.numel()
        hdr[1] = side_per_block if sidecar is not None else 0
        hdr[2] = 1 if sidecar is not None else 0
    dist.broadcast(hdr, peer(src), group=group)
    n_blocks, spb, has_side = (int(x) for x in hdr.cpu())
    lens_all = (comp_len.to(device=dev, dtype=torch.int32).contiguous() if rank == src
                else torch.empty(n_blocks, dtype=torch.int32, device=dev))
    if n_blocks:
        dist.broadcast(lens_all, peer(src), group=group)
    lens_cpu = lens_all.cpu().to(torch.int64)
    mine = rank_blocks(n_blocks, rank, world, scheme)
    my_idx = torch.as_tensor(list(mine), dtype=torch.int64)
    my_lens = lens_all[my_idx.to(dev)].contiguous() if len(my_idx) else lens_all[:0]
    ops = []
    if rank == src:
        offsets = exclusive_offsets(lens_cpu)
        side2 = sidecar.view(n_blocks, spb) if has_side else None

        def shard(r):
            idx = rank_blocks(n_blocks, r, world, scheme)
            if scheme == "contiguous":
                a, b = idx.start, idx.stop
                lo = int(offsets[a]) if a < n_blocks else 0
                hi = int(offsets[b - 1] + lens_cpu[b - 1]) if b > a else lo
                s = stream[lo:hi]
                sc = side2[a:b].reshape(-1) if has_side else None
            else:
                ii = torch.as_tensor(list(idx), dtype=torch.int64)
                s = select_blocks(stream, offsets, lens_cpu, ii)
                sc = side2[ii.to(side2.device)].reshape(-1).contiguous() if has_side else None
            return s.contiguous(), sc

        for r in range(world):
            s, sc = shard(r)
            if r == rank:
                out, out_side = s, sc
                continue
            ops.append(dist.P2POp(dist.isend, s, peer(r), group, _TAG_DATA))
            if has_side:
                ops.append(dist.P2POp(dist.isend, sc, peer(r), group, _TAG_SIDE))
    else:
        out = torch.empty(int(lens_cpu[my_idx].sum()) if len(my_idx) else 0, dtype=torch.uint8, device=dev)
        out_side = torch.empty(len(my_idx) * spb, dtype=torch.int64, device=dev) if has_side else None
        ops.append(dist.P2POp(dist.irecv, out, peer(src), group, _TAG_DATA))
        if has_side:
            ops.append(dist.P2POp(dist.irecv, out_side, peer(src), group, _TAG_SIDE))
    _run_p2p(ops)
    return out, my_lens, out_side, mine


def assemble(streams, lens, n_blocks: int, world: int, scheme: str = "contiguous"):
    """On the gathering rank: per-global-block (rank, offset, length) index so
    block b's bytes are streams[rank][offset: offset + length]."""
    index = [None] * n_blocks
    for r in range(world):
        offs = exclusive_offsets(lens[r].cpu())
        for j, b in enumerate(rank_blocks(n_blocks, r, world, scheme)):
            index[b] = (r, int(offs[j]), int(lens[r][j]))
    return index


def concat_global(streams, lens, n_blocks: int, world: int, scheme: str = "contiguous", sides=None):
    """On the gathering rank: one packed stream of every block in global
    order (+ lengths, + sidecar) from the gathered shards -- the input of
    `scatter_stream`.  Contiguous shards concatenate; round-robin shards are
    interleaved block by block (fsehip_copy_blocks on device tensors)."""
    if scheme == "contiguous":
        stream = torch.cat([s for s in streams])
        ln = torch.cat([x.to(torch.int32) for x in lens])
        side = torch.cat(list(sides)) if sides is not None else None
        return stream, ln, side
    if scheme != "round_robin":
        raise ValueError(f"unknown scheme {scheme!r}")
    # rank r's j-th block is global block r + j*world: strided slices
    dev = streams[0].device
    ln = torch.empty(n_blocks, dtype=torch.int32, device=dev)
    src_off = torch.empty(n_blocks, dtype=torch.int64, device=dev)
    base = 0
    for r in range(world):
        ln[r::world] = lens[r].to(device=dev, dtype=torch.int32)
        src_off[r::world] = exclusive_offsets(lens[r]).to(dev) + base
        base += int(streams[r].numel())
    cat = torch.cat([s for s in streams])  # the shards back to back
    stream = select_blocks(cat, src_off, ln, torch.arange(n_blocks))
    side = None
    if sides is not None:
        spb = sides[0].numel() // max(len(lens[0]), 1)
        side = torch.empty(n_blocks, spb, dtype=torch.int64, device=sides[0].device)
        for r in range(world):
            side[r::world] = sides[r].view(-1, spb)
        side = side.reshape(-1)
    return stream, ln, side
