"""Multi-GPU sharding of independent blocks (one process per GPU).

Blocks of the reference format carry no cross-block state, so the data path
needs no collective: each rank compresses / decompresses its own shard of
blocks.  The only exchange is the optional gather of the compressed output
to one rank (RCCL over xGMI with the "nccl" backend, gloo on CPU), which is
timed separately from the throughput metric.

Everything here is backend-agnostic torch.distributed code over tensors, so
the same functions run over RCCL on MI355X and over gloo in the CPU tests.
"""
from __future__ import annotations

import torch
import torch.distributed as dist


def rank_blocks(n_blocks: int, rank: int, world: int, scheme: str = "contiguous") -> range:
    """Global block indices owned by `rank`.

    contiguous: rank r owns [r*q + min(r, m), ...) (q, m = divmod(n, world));
    round_robin: rank r owns r, r + world, r + 2*world, ...
    """
    if scheme == "round_robin":
        return range(rank, n_blocks, world)
    q, m = divmod(n_blocks, world)
    start = rank * q + min(rank, m)
    return range(start, start + q + (1 if rank < m else 0))


def pack_host(slots: torch.Tensor, slot_bytes: int, comp_len: torch.Tensor):
    """Reference (torch) packer: slot layout -> (stream, offsets).  Used on
    CPU tensors in tests; on the GPU use `pack_device` (HIP kernel)."""
    lens = comp_len.to(torch.int64)
    offsets = torch.zeros_like(lens)
    if len(lens) > 1:
        offsets[1:] = torch.cumsum(lens, 0)[:-1]
    total = int(lens.sum())
    stream = torch.empty(total, dtype=torch.uint8, device=slots.device)
    for b in range(len(lens)):
        n = int(lens[b])
        o = int(offsets[b])
        stream[o:o + n] = slots[b * slot_bytes: b * slot_bytes + n]
    return stream, offsets


def pack_device(slots: torch.Tensor, slot_bytes: int, comp_len: torch.Tensor):
    """Slot layout -> contiguous stream on the GPU (fsehip_pack_blocks)."""
    import ctypes as C

    from ._lib import check, load

    lens = comp_len.to(torch.int64)
    offsets = torch.zeros_like(lens)
    if len(lens) > 1:
        offsets[1:] = torch.cumsum(lens, 0)[:-1]
    total = int(lens.sum())
    stream = torch.empty(max(total, 1), dtype=torch.uint8, device=slots.device)
    lib = load()
    hs = C.c_void_p(torch.cuda.current_stream(slots.device).cuda_stream)
    check(lib.fsehip_pack_blocks(C.c_void_p(slots.data_ptr()), slot_bytes,
                                 C.c_void_p(comp_len.data_ptr()), C.c_void_p(offsets.data_ptr()),
                                 len(lens), C.c_void_p(stream.data_ptr()), hs), "fsehip_pack_blocks")
    return stream[:total], offsets


def gather_stream(stream: torch.Tensor, comp_len: torch.Tensor, dst: int = 0, group=None):
    """Gather every rank's packed compressed stream and block lengths on `dst`.

    Step 1: all_gather of the per-rank (n_blocks, bytes) sizes.
    Step 2: gather of the length arrays and of the byte streams, padded to
    the largest rank (torch.distributed.gather needs equal sizes).
    Returns (streams, lens) lists indexed by rank on `dst`, (None, None)
    elsewhere.
    """
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    dev = stream.device
    sizes = torch.tensor([comp_len.numel(), stream.numel()], dtype=torch.int64, device=dev)
    all_sizes = [torch.zeros_like(sizes) for _ in range(world)]
    dist.all_gather(all_sizes, sizes, group=group)
    max_blocks = max(int(s[0]) for s in all_sizes)
    max_bytes = max(int(s[1]) for s in all_sizes)
    lens_pad = torch.zeros(max(max_blocks, 1), dtype=torch.int64, device=dev)
    lens_pad[: comp_len.numel()] = comp_len.to(torch.int64)
    data_pad = torch.zeros(max(max_bytes, 1), dtype=torch.uint8, device=dev)
    data_pad[: stream.numel()] = stream
    if rank == dst:
        lens_list = [torch.empty_like(lens_pad) for _ in range(world)]
        data_list = [torch.empty_like(data_pad) for _ in range(world)]
    else:
        lens_list = data_list = None
    dist.gather(lens_pad, lens_list, dst=dst, group=group)
    dist.gather(data_pad, data_list, dst=dst, group=group)
    if rank != dst:
        return None, None
    streams = [data_list[r][: int(all_sizes[r][1])] for r in range(world)]
    lens = [lens_list[r][: int(all_sizes[r][0])] for r in range(world)]
    return streams, lens


def assemble(streams, lens, n_blocks: int, world: int, scheme: str = "contiguous"):
    """On the gathering rank: per-global-block (rank, offset, length) index so
    block b's bytes are streams[rank][offset: offset + length]."""
    index = [None] * n_blocks
    for r in range(world):
        offs = torch.zeros(len(lens[r]), dtype=torch.int64)
        if len(lens[r]) > 1:
            offs[1:] = torch.cumsum(lens[r].cpu(), 0)[:-1]
        for j, b in enumerate(rank_blocks(n_blocks, r, world, scheme)):
            index[b] = (r, int(offs[j]), int(lens[r][j]))
    return index
