"""Multi-rank path on the GPU (BASELINE configs[3] in small):
two ranks sharing card 0 with gloo collectives run shard -> HIP encode
(fsehip_compress_blocks) -> pack (fsehip_pack_blocks) -> gatherv to rank 0
-> per-block oracle bytes -> scatter back -> unpack -> HIP decode, for both
block -> rank schemes.  (RCCL needs one GPU per rank, so on a one-GPU box
the collectives run over gloo; the data path is the same HIP code.)"""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

NB, BS, TAIL = 10, 65536, 777  # the last global block is ragged


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
    ok = False
    try:
        from entropy_coders_amd import BlockCodec
        from entropy_coders_amd.dist import (assemble, concat_global, gather_stream, pack_device, rank_blocks,
                                             scatter_stream, unpack_device)
        from oracle import oracle as O

        torch.cuda.set_device(0)
        codec = BlockCodec(device="cuda:0")
        n_glob = NB * BS - TAIL
        raw = codec.generate(0, 0.155, 0x5EED0004, n_glob)
        mine = list(rank_blocks(NB, rank, world, scheme))
        local = torch.cat([raw[b * BS: min((b + 1) * BS, n_glob)] for b in mine])
        cb = codec.compress(local)
        torch.cuda.synchronize()
        ok = int(cb["status"].abs().max()) == 0
        nb = len(mine)
        side = cb["sidecar"][: nb * codec.side_per_block]
        packed, _ = pack_device(cb["out"], codec.slot_bytes, cb["comp_len"])
        streams, lens, sides = gather_stream(packed.cpu(), cb["comp_len"].cpu(), dst=0, sidecar=side.cpu())
        g_stream = g_lens = g_side = None
        if rank == 0:
            host = raw.cpu().numpy()
            for b, (r, off, ln) in enumerate(assemble(streams, lens, NB, world, scheme)):
                want = O.compress2(host[b * BS: min((b + 1) * BS, n_glob)])[0]
                ok &= streams[r][off: off + ln].numpy().tobytes() == want
            g_stream, g_lens, g_side = concat_global(streams, lens, NB, world, scheme, sides)
        my, my_lens, my_side, idx = scatter_stream(g_stream, g_lens, src=0, sidecar=g_side,
                                                   side_per_block=codec.side_per_block, scheme=scheme,
                                                   device="cpu")
        ok &= list(idx) == mine
        slots = unpack_device(my.cuda(), my_lens.cuda(), codec.slot_bytes)
        cb2 = {"n_total": local.numel(), "out": slots, "comp_len": my_lens.cuda(), "sidecar": my_side.cuda()}
        for use_side in (True, False):
            out = torch.full_like(local, 0xA5)
            st = torch.full((nb,), -99, dtype=torch.int32, device="cuda:0")
            codec.decompress_into(cb2, out, st, use_sidecar=use_side)
            torch.cuda.synchronize()
            ok &= int(st.abs().max()) == 0 and bool(torch.equal(out, local))
        # round-robin selection on the device (fsehip_copy_blocks) equals the host slicing
        if rank == 0 and scheme == "round_robin":
            from entropy_coders_amd.dist import exclusive_offsets, select_blocks

            offs = exclusive_offsets(g_lens)
            sel = [9, 0, 4, 7, 1]
            dsel = select_blocks(g_stream.cuda(), offs.cuda(), g_lens.cuda(), sel)
            hsel = select_blocks(g_stream, offs, g_lens, sel)
            ok &= bool(torch.equal(dsel.cpu(), hsel))
    finally:
        flag = torch.tensor([1 if ok else 0])
        dist.all_reduce(flag, op=dist.ReduceOp.MIN)
        if rank == 0:
            q.put(bool(flag.item()))
        dist.destroy_process_group()


@pytest.mark.parametrize("scheme", ["contiguous", "round_robin"])
def test_two_ranks_encode_gather_scatter_decode(scheme):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, scheme, q)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(110)
    codes = [p.exitcode for p in procs]
    for p in procs:
        if p.exitcode is None:
            p.kill()
    assert codes == [0, 0], codes
    assert q.get(timeout=10) is True
