#!/usr/bin/env python3
"""FSE encode+decode throughput on MI355X (BASELINE.json metric, config C2).

One step = encode 1 GiB of synthetic bytes (16384 x 64 KiB blocks, LUT
generator p=0.155, H ~ 4.02 bits/symbol) into reference-exact fse_compress2
blocks + decode them back, inputs resident in HBM.  N GPUs = N independent
1 GiB shards (weak scaling, no data-path collective).  Rank 0 prints one
JSON line.  Launch N>1 with torch.distributed.run (one rank per GPU).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--no-cpu]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)
METRIC = "FSE encode+decode GiB/s on 1 GiB synthetic bytes; bit-exact round-trip"


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--bytes", type=int, default=1 << 30, help="raw bytes per GPU")
    ap.add_argument("--block", type=int, default=65536)
    ap.add_argument("--prob", type=float, default=0.155)
    ap.add_argument("--kind", type=int, default=0)
    ap.add_argument("--table-log", type=int, default=0)
    ap.add_argument("--ckpt", type=int, default=128)
    ap.add_argument("--nstates", type=int, default=2, choices=(1, 2),
                    help="block format: 2 = fse_compress2 (the headline), 1 = fse_compress")
    ap.add_argument("--no-cpu", action="store_true", help="skip the CPU baseline leg")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--no-c3", action="store_true", help="skip the decode-only (prebuilt tables) line")
    ap.add_argument("--no-sweep", action="store_true", help="skip the C5 distribution / table-log sweep")
    ap.add_argument("--sweep-bytes", type=int, default=256 << 20, help="raw bytes per C5 sweep point")
    ap.add_argument("--host", action="store_true",
                    help="also time the host-streaming pipeline (pinned host buffers, PCIe copies overlapped "
                         "with the kernels); reported separately, never in value")
    ap.add_argument("--gather", action="store_true",
                    help="after the timed steps, pack each rank's blocks on the GPU and gather the "
                         "compressed streams to rank 0 (RCCL); reported separately, never in value")
    return ap.parse_args()


def workload_name(args, n: int) -> str:
    fmt = "fse_compress2" if args.nstates == 2 else "fse_compress"
    gen = {0: "LUT", 1: "geometric", 2: "uniform"}.get(args.kind, f"kind {args.kind}")
    c2 = (args.kind == 0 and args.prob == 0.155 and args.block == 65536 and n == 1 << 30)
    tag = "C2" if c2 else "custom"
    ent = " (H~4.02 bits/sym)" if c2 else ""
    return (f"{tag}: {n / 2**30:g} GiB per GPU as {-(-n // args.block)} x {args.block // 1024} KiB independent "
            f"blocks, {gen} generator p={args.prob}{ent}, encode ({fmt}-exact) + decode")


def cpu_baseline(src_host: np.ndarray, block: int, budget_s: float) -> dict:
    """The parity oracle (C restatement of the reference, -O3) on host cores.

    Sample: whole 64 KiB blocks of the same C2 data, compressed+decompressed by
    `threads` pthreads; repeated over the first blocks until ~budget_s of wall
    time has been spent (bounded), throughput = raw bytes / wall time.
    """
    from oracle import oracle as O

    threads = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or min(os.cpu_count() or 1, 16)
    n_blocks = len(src_host) // block
    # calibrate on a small slice
    sample = src_host[: block * min(n_blocks, max(threads * 4, 64))]
    t0 = time.perf_counter()
    comp, lens, slot = O.compress2_blocks(sample, block, threads)
    out = O.decompress2_blocks(comp, slot, lens, block, len(sample), threads)
    t1 = time.perf_counter()
    assert np.array_equal(out, sample)
    per_byte = (t1 - t0) / len(sample)
    n_take = int(min(len(src_host), max(len(sample), budget_s / max(per_byte, 1e-12))))
    n_take -= n_take % block
    reps, total, wall = 0, 0, 0.0
    sample = src_host[:n_take]
    while wall < budget_s * 0.5 and reps < 8:
        t0 = time.perf_counter()
        comp, lens, slot = O.compress2_blocks(sample, block, threads)
        tc = time.perf_counter()
        out = O.decompress2_blocks(comp, slot, lens, block, len(sample), threads)
        t1 = time.perf_counter()
        wall += t1 - t0
        total += len(sample)
        reps += 1
    assert np.array_equal(out, sample)
    # single-core, bench-exact block (benches/fse_benchmark.rs:30-52)
    b32 = O.generate(0, 0.2, 0x5EED0001, 0, 1 << 15)
    c32, _ = O.compress2(b32)
    t0 = time.perf_counter()
    it = 0
    while time.perf_counter() - t0 < 1.0:
        O.compress2(b32)
        it += 1
    enc1 = it * len(b32) / (time.perf_counter() - t0)
    t0 = time.perf_counter()
    it = 0
    while time.perf_counter() - t0 < 1.0:
        O.decompress2(c32, cap=1 << 16)
        it += 1
    dec1 = it * len(b32) / (time.perf_counter() - t0)
    return {
        "value": round(total / wall / 2**30, 4),
        "unit": "GiB/s",
        "cores": threads,
        "kind": "port",
        "sample": f"{reps} x {n_take >> 20} MiB of the same C2 data ({n_take // block} x 64 KiB blocks), "
                  f"compress2+decompress2 round trip, {threads} pthreads, oracle/fse_oracle.c -O3",
        "single_core_32KiB_lut0.2": {"encode_MiB_s": round(enc1 / 2**20, 1),
                                     "decode_MiB_s": round(dec1 / 2**20, 1)},
    }


C5_SWEEP = [  # BASELINE.json configs[4]: (name, generator kind, LUT p, table log)
    *[("near-uniform (0..239, H~7.9 bits)", 2, 0.0, L) for L in (9, 10, 11, 12)],
    *[("skewed (LUT p=0.77, H~1.0 bit)", 0, 0.77, L) for L in (9, 10, 11, 12)],
    ("LUT p=0.05 (normalize_slow path)", 0, 0.05, 9),
]


def c5_sweep(dev, nbytes: int, block: int, ckpt: int, reps: int = 3) -> list:
    """C5 distribution sweep on one GPU, after the timed step: encode and
    decode of `nbytes` per distribution and explicit table log (histogram.rs:95
    normalize(L)), HIP-event timed, round trip verified.  Reported beside the
    bench line, never in `value`."""
    import torch

    from entropy_coders_amd import BlockCodec

    stream = torch.cuda.current_stream(dev)
    rows = []
    for name, kind, prob, L in C5_SWEEP:
        codec = BlockCodec(block_size=block, table_log=L, ckpt_interval=ckpt, device=dev)
        src = codec.generate(kind, prob, 0x5EED0005, nbytes)
        cb = codec.alloc(nbytes)
        out = torch.empty(nbytes, dtype=torch.uint8, device=dev)
        st = torch.zeros(codec.n_blocks(nbytes), dtype=torch.int32, device=dev)
        codec.compress_into(src, cb)
        codec.decompress_into(cb, out, st)
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
        ev[0].record(stream)
        for _ in range(reps):
            codec.compress_into(src, cb)
        ev[1].record(stream)
        for _ in range(reps):
            codec.decompress_into(cb, out, st)
        ev[2].record(stream)
        torch.cuda.synchronize(dev)
        enc_ms = ev[0].elapsed_time(ev[1]) / reps
        dec_ms = ev[1].elapsed_time(ev[2]) / reps
        ok = (int(cb["status"].abs().max()) == 0 and int(st.abs().max()) == 0 and bool(torch.equal(out, src)))
        comp = int(cb["comp_len"].to(torch.int64).sum())
        rows.append({"dist": name, "table_log": L, "compressed_ratio": round(comp / nbytes, 4),
                     "encode_GiB_s": round(nbytes / (enc_ms * 1e-3) / 2**30, 1),
                     "decode_GiB_s": round(nbytes / (dec_ms * 1e-3) / 2**30, 1),
                     "roundtrip_GiB_s": round(nbytes / ((enc_ms + dec_ms) * 1e-3) / 2**30, 1), "verified": ok})
        del codec, src, cb, out, st
    return rows


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # one rank per GPU over RCCL ("nccl"); FSEHIP_BENCH_BACKEND=gloo rehearses the
    # multi-rank logic on a one-GPU box (ranks share the card, CPU collectives)
    backend = os.environ.get("FSEHIP_BENCH_BACKEND", "nccl")
    gpu = local % max(torch.cuda.device_count(), 1)
    torch.cuda.set_device(gpu)
    dev = torch.device("cuda", gpu)
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)
    cdev = dev if backend == "nccl" else torch.device("cpu")  # where collective tensors live

    from entropy_coders_amd import BlockCodec

    codec = BlockCodec(block_size=args.block, table_log=args.table_log, ckpt_interval=args.ckpt,
                       device=dev, nstates=args.nstates)
    n = args.bytes
    seed = 0x5EED0002 ^ (rank * 0x1000193)
    src = codec.generate(args.kind, args.prob, seed, n)
    cb = codec.alloc(n)
    out = torch.empty(n, dtype=torch.uint8, device=dev)
    dstat = torch.zeros(codec.n_blocks(n), dtype=torch.int32, device=dev)
    stream = torch.cuda.current_stream(dev)

    def barrier():
        if world > 1:
            if backend == "nccl":
                dist.barrier(device_ids=[gpu])
            else:
                dist.barrier()

    for _ in range(args.warmup):
        codec.compress_into(src, cb)
        codec.decompress_into(cb, out, dstat)
    torch.cuda.synchronize(dev)

    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True),
           torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for k in range(args.steps):
        ev[k][0].record(stream)
        codec.compress_into(src, cb)
        ev[k][1].record(stream)
        codec.decompress_into(cb, out, dstat)
        ev[k][2].record(stream)
    torch.cuda.synchronize(dev)
    barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=cdev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    enc_ms = float(np.mean([e[0].elapsed_time(e[1]) for e in ev]))
    dec_ms = float(np.mean([e[1].elapsed_time(e[2]) for e in ev]))

    # verification (outside the timed region): statuses and exact round trip
    ok = (int(cb["status"].abs().max()) == 0 and int(dstat.abs().max()) == 0
          and bool(torch.equal(out, src)))
    comp_bytes = int(cb["comp_len"].to(torch.int64).sum())
    nb = codec.n_blocks(n)
    def n_ckpt(ln):  # sidecar entries of a block of ln bytes (pairs for 2-state, symbols for 1-state)
        return (ln // 2) // args.ckpt + 1 if args.nstates == 2 else (ln - 1) // args.ckpt + 1

    side_bytes = 8 * sum(n_ckpt(min(args.block, n - b * args.block)) for b in range(nb)) if args.ckpt else 0
    if world > 1:
        flag = torch.tensor([1 if ok else 0], device=cdev)
        dist.all_reduce(flag, op=dist.ReduceOp.MIN)
        ok = bool(flag.item())

    # C3 (BASELINE configs[2]): decode only, decode tables prebuilt and untimed
    c3 = None
    comp_bytes_pre = int(cb["comp_len"].to(torch.int64).sum())
    if not args.no_c3:
        tabs = codec.build_dtables(cb)
        torch.cuda.synchronize(dev)
        e3 = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        codec.decompress_dt_into(cb, tabs, out, dstat)
        e3[0].record(stream)
        for _ in range(args.steps):
            codec.decompress_dt_into(cb, tabs, out, dstat)
        e3[1].record(stream)
        torch.cuda.synchronize(dev)
        c3_ms = e3[0].elapsed_time(e3[1]) / args.steps
        c3_ok = int(dstat.abs().max()) == 0 and bool(torch.equal(out, src))
        c3 = {"workload": "C3-style decode only on the blocks above (prebuilt decode tables, untimed): "
                          f"{comp_bytes_pre / 2**30:.3f} GiB compressed -> {n / 2**30:.3f} GiB",
              "decode_ms": round(c3_ms, 4), "decode_GiB_s": round(n / (c3_ms * 1e-3) / 2**30, 2),
              "roofline_frac": None, "verified": c3_ok}
        ok = ok and c3_ok

    host_info = None
    if args.host:
        from entropy_coders_amd.stream import HostPipeline

        pipe = HostPipeline(codec, chunk_blocks=1024)
        host_src = src.cpu().pin_memory()
        c_out = pipe.alloc_compress_out(n)  # pinned outputs, allocated once
        d_out = pipe.alloc_decompress_out(n)
        w_stream, w_lens, w_side, _ = pipe.compress(host_src[: 4 * 1024 * args.block], c_out)  # warm-up
        pipe.decompress(w_stream, w_lens, w_side, 4 * 1024 * args.block, d_out)
        torch.cuda.synchronize(dev)
        h0 = time.perf_counter()
        hs_stream, hs_lens, hs_side, hs_status = pipe.compress(host_src, c_out)
        h1 = time.perf_counter()
        h_out, h_stat = pipe.decompress(hs_stream, hs_lens, hs_side, n, d_out)
        h2 = time.perf_counter()
        h_ok = (int(hs_status.abs().max()) == 0 and int(h_stat.abs().max()) == 0
                and bool(torch.equal(h_out, host_src)))
        host_info = {"workload": "the same 1 GiB from pinned host memory, 64 MiB chunks, H2D/D2H on their "
                                 "own streams overlapped with the kernels (PCIe-inclusive)",
                     "compress_GiB_s": round(n / (h1 - h0) / 2**30, 2),
                     "decompress_GiB_s": round(n / (h2 - h1) / 2**30, 2),
                     "compressed_bytes": int(hs_stream.numel()), "verified": h_ok}
        ok = ok and h_ok
        del host_src, hs_stream, h_out, c_out, d_out

    gather_info = None
    if args.gather:
        from entropy_coders_amd.dist import gather_stream, pack_device

        packed, _ = pack_device(cb["out"], codec.slot_bytes, cb["comp_len"])  # warm-up (allocation)
        del packed
        torch.cuda.synchronize(dev)
        barrier()
        g0 = time.perf_counter()
        packed, _ = pack_device(cb["out"], codec.slot_bytes, cb["comp_len"])
        torch.cuda.synchronize(dev)
        tp = time.perf_counter()
        if world > 1:
            streams, _ = gather_stream(packed, cb["comp_len"], dst=0)
        torch.cuda.synchronize(dev)
        g1 = time.perf_counter()
        gather_info = {"packed_bytes_per_rank": int(packed.numel()),
                       "pack_ms": round((tp - g0) * 1e3, 3),
                       "pack_plus_gather_ms": round((g1 - g0) * 1e3, 3),
                       "gather_GB_s": round(world * packed.numel() / max(g1 - tp, 1e-9) / 1e9, 2)
                       if world > 1 else None}

    if rank == 0:
        enc_bytes = n + comp_bytes + side_bytes  # raw read + compressed (+ sidecar) written
        dec_bytes = comp_bytes + side_bytes + n  # compressed (+ sidecar) read + raw written
        dom = ("fse_encode_blocks", enc_ms, enc_bytes) if enc_ms >= dec_ms else \
              ("fse_decode_blocks", dec_ms, dec_bytes)
        achieved = dom[2] / (dom[1] * 1e-3) / 1e9
        traffic = None
        tpath = os.path.join(ROOT, "profiles", "traffic.json")
        if os.path.exists(tpath):
            try:
                with open(tpath) as f:
                    t = json.load(f).get(dom[0])
                traffic = int(t["bytes_per_launch"]) if t else None
            except Exception:
                traffic = None
        line = {
            "metric": METRIC,
            "value": round(world * n * args.steps / elapsed / 2**30, 3),
            "unit": "GiB/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic",
            "config": {
                "workload": workload_name(args, n),
                "format": "2-state (fse_compress2)" if args.nstates == 2 else "1-state (fse_compress)",
                "block_size": args.block,
                "table_log": args.table_log or "optimal (11)",
                "ckpt_interval": f"{args.ckpt} {'pairs' if args.nstates == 2 else 'symbols'}",
                "parallelism": f"dp{world} (blocks sharded per GPU, no collective in the step)",
            },
            "roofline": {
                "bound": "hbm",
                "kernel": dom[0],
                "achieved": round(achieved, 1),
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4),
                "traffic": traffic,
                "traffic_source": "profiles/traffic.json: rocprofv3 FETCH_SIZE x2 (gfx950 correction) + WRITE_SIZE, per launch",
                "algorithmic_bytes_per_launch": dom[2],
            },
            "encode_ms": round(enc_ms, 4),
            "decode_ms": round(dec_ms, 4),
            "encode_GiB_s": round(n / (enc_ms * 1e-3) / 2**30, 2),
            "decode_GiB_s": round(n / (dec_ms * 1e-3) / 2**30, 2),
            "compressed_ratio": round(comp_bytes / n, 5),
            "verified_roundtrip": ok,
        }
        if c3 is not None:
            c3["roofline_frac"] = round(dec_bytes / (c3["decode_ms"] * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)
            line["c3_decode_only"] = c3
        if gather_info is not None:
            line["gather"] = gather_info
        if host_info is not None:
            line["host_pipeline"] = host_info
        if not args.no_sweep and args.nstates == 2:
            sw = c5_sweep(dev, args.sweep_bytes, args.block, args.ckpt)
            line["c5_sweep"] = {"workload": f"C5: {args.sweep_bytes >> 20} MiB per distribution and table log, "
                                            "encode + decode (2-state), 1 GPU", "rows": sw}
            ok = ok and all(r["verified"] for r in sw)
            line["verified_roundtrip"] = ok
        if world == 1 and not args.no_cpu:
            line["cpu_baseline"] = cpu_baseline(src.cpu().numpy(), args.block, args.cpu_seconds)
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()
    if not ok:
        sys.exit(3)


if __name__ == "__main__":
    main()
