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


def _worker(rank, world, port, scheme, q, backend="gloo", NB=NB, gpu_per_rank=False):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    gpu = rank if gpu_per_rank else 0
    if backend == "nccl":
        torch.cuda.set_device(gpu)
        dist.init_process_group("nccl", rank=rank, world_size=world, device_id=torch.device("cuda", gpu))
    else:
        dist.init_process_group("gloo", rank=rank, world_size=world)
    host_t = (lambda t: t.cpu()) if backend == "gloo" else (lambda t: t)  # RCCL moves device tensors
    ok = False
    try:
        from entropy_coders_amd import BlockCodec
        from entropy_coders_amd.dist import (assemble, concat_global, gather_stream, pack_device, rank_blocks,
                                             scatter_stream, unpack_device)
        from oracle import oracle as O

        torch.cuda.set_device(gpu)
        codec = BlockCodec(device=f"cuda:{gpu}")
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
        streams, lens, sides = gather_stream(host_t(packed), host_t(cb["comp_len"]), dst=0, sidecar=host_t(side))
        g_stream = g_lens = g_side = None
        if rank == 0:
            host = raw.cpu().numpy()
            for b, (r, off, ln) in enumerate(assemble(streams, lens, NB, world, scheme)):
                want = O.compress2(host[b * BS: min((b + 1) * BS, n_glob)])[0]
                ok &= streams[r][off: off + ln].cpu().numpy().tobytes() == want
            g_stream, g_lens, g_side = concat_global(streams, lens, NB, world, scheme, sides)
        my, my_lens, my_side, idx = scatter_stream(g_stream, g_lens, src=0, sidecar=g_side,
                                                   side_per_block=codec.side_per_block, scheme=scheme,
                                                   device="cpu" if backend == "gloo" else None)
        ok &= list(idx) == mine
        slots = unpack_device(my.cuda(), my_lens.cuda(), codec.slot_bytes)
        cb2 = {"n_total": local.numel(), "out": slots, "comp_len": my_lens.cuda(), "sidecar": my_side.cuda()}
        for use_side in (True, False):
            out = torch.full_like(local, 0xA5)
            st = torch.full((nb,), -99, dtype=torch.int32, device=f"cuda:{gpu}")
            codec.decompress_into(cb2, out, st, use_sidecar=use_side)
            torch.cuda.synchronize()
            ok &= int(st.abs().max()) == 0 and bool(torch.equal(out, local))
        # round-robin selection on the device (fsehip_copy_blocks) equals the host slicing
        if rank == 0 and scheme == "round_robin":
            from entropy_coders_amd.dist import exclusive_offsets, select_blocks

            offs = exclusive_offsets(g_lens.cpu())
            sel = [9, 0, 4, 7, 1]
            dsel = select_blocks(g_stream.cuda(), offs.cuda(), g_lens.cuda(), sel)
            hsel = select_blocks(g_stream.cpu(), offs, g_lens.cpu(), sel)
            ok &= bool(torch.equal(dsel.cpu(), hsel))
    finally:
        flag = torch.tensor([1 if ok else 0], device="cpu" if backend == "gloo" else f"cuda:{gpu}")
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


@pytest.mark.parametrize("scheme", ["contiguous", "round_robin"])
def test_rccl_one_rank_encode_gather_scatter_decode(scheme):
    """The RCCL ("nccl") branch of dist.py on hardware: one rank (RCCL
    needs a GPU per rank), device tensors through all_gather, broadcast
    and the scatter's device-side block selection, bytes checked against
    the oracle.  The N-rank p2p transfers run in the driver's multi-GPU
    bench and in the gloo tests above."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_worker, args=(0, 1, _free_port(), scheme, q, "nccl"))
    p.start()
    p.join(110)
    code = p.exitcode
    if code is None:
        p.kill()
    assert code == 0, code
    assert q.get(timeout=10) is True


def test_eight_ranks_round_robin_encode_gather_scatter_decode():
    """C4's shape (BASELINE configs[3]) with 8 ranks on one card: 8 gloo
    ranks sharing card 0, 64 global blocks (8 per rank) sharded round-robin,
    HIP encode -> pack -> gatherv of 8 ranks into rank 0 -> every block's
    bytes against the oracle -> scatter -> HIP decode with and without the
    sidecar on every rank."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 8, port, "round_robin", q, "gloo", 64)) for r in range(8)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(170)
    codes = [p.exitcode for p in procs]
    for p in procs:
        if p.exitcode is None:
            p.kill()
    assert codes == [0] * 8, codes
    assert q.get(timeout=10) is True


def test_bench_c4_rehearsal_eight_ranks():
    """bench.py's own C4 path at 8 ranks (verdict r04 item 5): `--gpus 8
    --strong --scheme round_robin` over 512 MiB of 64 KiB blocks (64 MiB per
    rank), the ranks self-launched, sharing card 0 with gloo collectives:
    HIP encode + decode step on every rank, then pack -> gatherv to rank 0 ->
    scatter -> decode, checked against each rank's source.  One line,
    n_gpus 8, exit 0, c4_exchange.verified."""
    import json
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, FSEHIP_BENCH_BACKEND="gloo", MASTER_ADDR="127.0.0.1")
    cmd = [sys.executable, os.path.join(root, "bench.py"), "--gpus", "8", "--strong", "--scheme", "round_robin",
           "--bytes", str(512 << 20), "--steps", "2", "--warmup", "1", "--no-cpu", "--gather-timeout", "150"]
    r = subprocess.run(cmd, cwd=root, env=env, capture_output=True, text=True, timeout=420)
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-3000:])
    assert len(lines) == 1, r.stdout[-2000:]
    line = json.loads(lines[0])
    print(json.dumps({k: line[k] for k in ("value", "n_gpus", "scaling", "ms_per_step")}))
    print(json.dumps(line["c4_exchange"]))
    assert line["n_gpus"] == 8 and line["scaling"] == "strong" and line["verified_roundtrip"] is True
    c4 = line["c4_exchange"]
    assert c4["verified"] is True and c4["scheme"] == "round_robin" and c4["backend"] == "gloo"
    assert c4["gathered_bytes_into_rank0"] > 0


def _bench_two_ranks(extra_env, tmo="60"):
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, FSEHIP_BENCH_BACKEND="gloo", MASTER_ADDR="127.0.0.1", **extra_env)
    cmd = [sys.executable, os.path.join(root, "bench.py"), "--gpus", "2", "--steps", "2", "--warmup", "1",
           "--bytes", str(8 * 65536 + 4321), "--no-cpu", "--gather-timeout", tmo]
    r = subprocess.run(cmd, cwd=root, env=env, capture_output=True, text=True, timeout=400)
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    return r, lines


@pytest.mark.parametrize("mode", ["raise", "hang"])
def test_bench_two_ranks_exchange_failure_exits_nonzero(mode):
    """bench.py --gpus 2 end to end (two gloo ranks sharing card 0) with the
    C4 exchange forced to fail (every rank raises) or to hang (rank 1 never
    joins, the watchdog ends both ranks): the step's line is still printed
    once, with c4_exchange.verified false, and the run exits with
    EXIT_EXCHANGE_FAILED (4), never 0."""
    import json

    r, lines = _bench_two_ranks({"FSEHIP_BENCH_FAIL_EXCHANGE": mode}, tmo="20")
    assert r.returncode != 0, (r.stdout[-2000:], r.stderr[-3000:])
    assert len(lines) == 1, (r.stdout[-2000:], r.stderr[-3000:])
    line = json.loads(lines[0])
    assert line["n_gpus"] == 2 and line["verified_roundtrip"] is True
    assert line["c4_exchange"]["verified"] is False


def test_bench_two_ranks_exchange_ok():
    """The same run without a forced failure: exit 0, one line, exchange verified."""
    import json

    r, lines = _bench_two_ranks({})
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-3000:])
    assert len(lines) == 1
    line = json.loads(lines[0])
    assert line["c4_exchange"]["verified"] is True and line["verified_roundtrip"] is True


def _two_gpus():
    return torch.cuda.device_count() >= 2


@pytest.mark.skipif(not _two_gpus(), reason="needs two GPUs (one RCCL rank per GPU)")
@pytest.mark.parametrize("scheme", ["contiguous", "round_robin"])
def test_rccl_two_gpus_encode_gather_scatter_decode(scheme):
    """The first real multi-GPU exchange: two ranks on two GPUs over RCCL
    (nccl backend, one rank per device), the same shard -> encode -> gatherv
    -> oracle bytes -> scatter -> decode path as above."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, scheme, q, "nccl", NB, True)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(300)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    assert q.get(timeout=10) is True


@pytest.mark.skipif(not _two_gpus(), reason="needs two GPUs (one RCCL rank per GPU)")
def test_bench_rccl_two_gpus():
    """bench.py --gpus 2 as the driver's SCALE run launches it (self-launched
    ranks, RCCL, one GPU each), on 256 MiB per GPU: one line with n_gpus 2,
    the step verified, the C4 exchange verified over RCCL with its gather
    priced against the xGMI ingress roof (gather_roof_frac present)."""
    import json
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    env.pop("FSEHIP_BENCH_BACKEND", None)
    cmd = [sys.executable, os.path.join(root, "bench.py"), "--gpus", "2", "--steps", "3", "--warmup", "1",
           "--bytes", str(256 << 20), "--no-cpu", "--gather-timeout", "120"]
    r = subprocess.run(cmd, cwd=root, env=env, capture_output=True, text=True, timeout=400)
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-3000:])
    assert len(lines) == 1, r.stdout[-2000:]
    line = json.loads(lines[0])
    print(json.dumps({k: line[k] for k in ("value", "n_gpus", "scaling", "ms_per_step")}))
    print(json.dumps(line["c4_exchange"]))
    assert line["n_gpus"] == 2 and line["verified_roundtrip"] is True
    c4 = line["c4_exchange"]
    assert c4["verified"] is True and c4["backend"] == "nccl" and c4["gather_roof_frac"] is not None
