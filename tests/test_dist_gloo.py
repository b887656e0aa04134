"""world_size-2 gloo tests of the multi-GPU path on CPU: block sharding and
the compressed-output gather (the only collective), with blocks produced by
the CPU oracle (test checker) standing in for each rank's GPU output."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from entropy_coders_amd.dist import assemble, gather_stream, pack_host, rank_blocks

N_BLOCKS, BLOCK = 11, 4096


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, scheme, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from oracle import oracle as O

        mine = list(rank_blocks(N_BLOCKS, rank, world, scheme))
        slot = O.compress_bound(BLOCK) + 16
        slot = (slot + 15) // 16 * 16
        slots = torch.zeros(max(len(mine), 1) * slot, dtype=torch.uint8)
        lens = torch.zeros(len(mine), dtype=torch.int32)
        for j, b in enumerate(mine):
            src = O.generate(0, 0.2, 42, b, BLOCK)
            comp, _ = O.compress2(src)
            slots[j * slot: j * slot + len(comp)] = torch.from_numpy(np.frombuffer(comp, np.uint8).copy())
            lens[j] = len(comp)
        stream, _ = pack_host(slots, slot, lens)
        streams, all_lens = gather_stream(stream, lens, dst=0)
        if rank == 0:
            index = assemble(streams, all_lens, N_BLOCKS, world, scheme)
            ok = True
            for b, (r, off, ln) in enumerate(index):
                got = streams[r][off: off + ln].numpy().tobytes()
                want = O.compress2(O.generate(0, 0.2, 42, b, BLOCK))[0]
                ok &= got == want
                ok &= O.decompress2(got, raw_len=BLOCK) == O.generate(0, 0.2, 42, b, BLOCK).tobytes()
            q.put(ok)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("scheme", ["contiguous", "round_robin"])
def test_gather_two_ranks(scheme):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, scheme, q)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
        assert p.exitcode == 0
    assert q.get(timeout=10) is True


@pytest.mark.parametrize("world", [1, 2, 3, 8])
def test_rank_blocks_partition(world):
    for scheme in ("contiguous", "round_robin"):
        seen = []
        for r in range(world):
            seen += list(rank_blocks(N_BLOCKS, r, world, scheme))
        assert sorted(seen) == list(range(N_BLOCKS))
