#!/usr/bin/env python3
"""FSE encode+decode throughput on MI355X (BASELINE.json metric, config C2).

One step = encode 1 GiB of synthetic bytes (16384 x 64 KiB blocks, LUT
generator p=0.155, H ~ 4.02 bits/symbol) into reference-exact fse_compress2
blocks + decode them back, inputs resident in HBM.  N GPUs = N independent
1 GiB shards (weak scaling, no data-path collective; --strong: 1 GiB in total
split over the N GPUs).  Rank 0 prints one JSON line.

`--gpus N` (N > 1) without a torch.distributed.run environment starts the N
ranks itself: a child `python -m torch.distributed.run --nproc-per-node N`
launched before this process touches the GPU, one rank per GPU over RCCL.
With N > 1 the compressed shards are then gathered to rank 0 (gatherv) and
scattered back for decode, timed separately from `value` (C4).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--strong] [--no-cpu]
"""
from __future__ import annotations

import argparse
import json
import math
import os
import socket
import subprocess
import sys
import threading
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
    ap.add_argument("--bytes", type=int, default=1 << 30,
                    help="raw bytes per GPU (weak scaling) or in total (--strong)")
    ap.add_argument("--strong", action="store_true",
                    help="strong scaling: --bytes in total, split by blocks over the ranks")
    ap.add_argument("--block", type=int, default=65536)
    ap.add_argument("--prob", type=float, default=0.155)
    ap.add_argument("--kind", type=int, default=0)
    ap.add_argument("--table-log", type=int, default=0)
    ap.add_argument("--ckpt", type=int, default=64,
                    help="sidecar checkpoint interval (pairs for 2-state blocks): 64 gives 512 segments per "
                         "64 KiB block, decoded by 512-thread workgroups (sidecar 8 B per 64 pairs, ~12%% of "
                         "the compressed bytes at C2); 128 halves the sidecar at ~7%% more decode time")
    ap.add_argument("--nstates", type=int, default=2, choices=(1, 2),
                    help="block format: 2 = fse_compress2 (the headline), 1 = fse_compress")
    ap.add_argument("--no-cpu", action="store_true", help="skip the CPU baseline leg")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--no-c3", action="store_true", help="skip the decode-only (prebuilt tables) line")
    ap.add_argument("--c3-blocks", type=int, default=32768,
                    help="C3 size: blocks of C2 data (32768 x 64 KiB ~ 1 GiB compressed, SURVEY 8(d))")
    ap.add_argument("--no-serial", action="store_true", help="skip the sidecar-less decode line")
    ap.add_argument("--no-onestate", action="store_true", help="skip the 1-state format line")
    ap.add_argument("--no-sweep", action="store_true", help="skip the C5 distribution / table-log sweep")
    ap.add_argument("--no-host-calls", action="store_true",
                    help="skip the per-call latency of the host fse_compress2 / fse_decompress2 drop-ins")
    ap.add_argument("--sweep-bytes", type=int, default=1 << 30,
                    help="raw bytes per C5 sweep point (the step's 1 GiB: at 256 MiB = 4096 blocks over ~2300 "
                         "resident encode slots the last partial round of slow skewed blocks dominated)")
    ap.add_argument("--host", action="store_true",
                    help="also time the host-streaming pipeline (pinned host buffers, PCIe copies overlapped "
                         "with the kernels); reported separately, never in value")
    ap.add_argument("--no-gather", action="store_true",
                    help="N > 1: skip the gather of the compressed shards to rank 0 and the scatter back "
                         "(reported separately, never in value)")
    ap.add_argument("--gather-timeout", type=float, default=180.0,
                    help="N > 1: seconds the exchange may take; past that every rank ends (rank 0 first "
                         "prints the line, the exchange marked as timed out) instead of hanging in a collective")
    ap.add_argument("--scheme", default="round_robin", choices=("round_robin", "contiguous"),
                    help="block -> rank mapping of the gather/scatter (C4: block b on GPU b mod N)")
    return ap.parse_args()


def self_launch(args) -> None:
    """`--gpus N` outside torch.distributed.run: run the N ranks as a child
    torch.distributed.run (this process has not touched the GPU: only argparse
    ran) and exit with its status."""
    if args.gpus <= 1 or "WORLD_SIZE" in os.environ:
        return
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__), *sys.argv[1:]]
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    sys.exit(subprocess.call(cmd, env=env))


def host_cpu() -> dict:
    """Host cores for the CPU baseline: this process's CPU affinity (`nproc`),
    the cgroup CPU quota if one is set, and the CPU model."""
    try:
        n_aff = len(os.sched_getaffinity(0))
    except AttributeError:
        n_aff = os.cpu_count() or 1
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
        if q != "max":
            quota = int(q) / int(per)
    except (OSError, ValueError):
        pass
    model = None
    try:
        with open("/proc/cpuinfo") as f:
            for ln in f:
                if ln.startswith("model name"):
                    model = ln.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    usable = n_aff if quota is None else max(1, min(n_aff, int(quota)))
    return {"nproc": n_aff, "cgroup_cpu_quota": quota, "usable_cores": usable, "model": model}


EXIT_STEP_UNVERIFIED = 3  # the timed step (or a verified side line) failed its check
EXIT_EXCHANGE_FAILED = 4  # the step verified, the C4 exchange failed or timed out


class ExchangeGuard:
    """Watchdog around the C4 exchange (collectives that may never complete).

    `on_timeout()` runs on the timer thread if `timeout` seconds pass before
    `finish()`: it prints what the rank has to say and returns the exit code,
    and the process ends with it (os._exit: a rank blocked in a collective
    cannot be unwound).  One lock and a done flag make the two outcomes
    exclusive: once `finish()` has run, a late timer does nothing; once the
    timer has begun, `finish()` blocks until the process is gone, so no
    second line is printed."""

    def __init__(self, timeout: float, on_timeout):
        self._lock = threading.Lock()
        self._done = False
        self._on_timeout = on_timeout
        self._timer = threading.Timer(timeout, self._fire)
        self._timer.daemon = True

    def _fire(self) -> None:
        with self._lock:
            if self._done:
                return
            self._done = True
            code = EXIT_EXCHANGE_FAILED
            try:
                code = self._on_timeout()
            finally:
                sys.stdout.flush()
                sys.stderr.flush()
                os._exit(code)

    def start(self) -> "ExchangeGuard":
        self._timer.start()
        return self

    def finish(self) -> None:
        with self._lock:
            self._done = True
        self._timer.cancel()


def forced_exchange_failure() -> str | None:
    """Test hook (tests/test_gpu_dist.py, tests/test_dist_gloo.py): FSEHIP_BENCH_FAIL_EXCHANGE
    = "raise" makes every rank's exchange raise, "hang" makes rank 1 never
    reach it (rank 0 then waits in a collective until the watchdog fires)."""
    v = os.environ.get("FSEHIP_BENCH_FAIL_EXCHANGE", "")
    return v if v in ("raise", "hang") else None


def workload_name(args, n: int) -> str:
    fmt = "fse_compress2" if args.nstates == 2 else "fse_compress"
    gen = {0: "LUT", 1: "geometric", 2: "uniform"}.get(args.kind, f"kind {args.kind}")
    lut = args.kind == 0 and args.prob == 0.155 and args.block == 65536
    c2 = lut and n == 1 << 30
    # C4 (BASELINE configs[3]): 8 GiB in total, round-robin over the ranks
    c4 = (lut and n == 8 << 30 and getattr(args, "strong", False) and args.scheme == "round_robin"
          and args.gpus > 1)
    tag = "C2" if c2 else "C4" if c4 else "custom"
    ent = " (H~4.02 bits/sym)" if lut else ""
    where = "in total (strong scaling)" if getattr(args, "strong", False) else "per GPU"
    return (f"{tag}: {n / 2**30:g} GiB {where} as {-(-n // args.block)} x {args.block // 1024} KiB independent "
            f"blocks, {gen} generator p={args.prob}{ent}, encode ({fmt}-exact) + decode")


def _median_rate(fn, nbytes: int, budget_s: float) -> float:
    """Criterion-like: repeat fn in batches for ~budget_s, median bytes/s."""
    rates = []
    t_end = time.perf_counter() + budget_s
    batch = 1
    while time.perf_counter() < t_end or len(rates) < 5:
        t0 = time.perf_counter()
        for _ in range(batch):
            fn()
        dt = time.perf_counter() - t0
        rates.append(batch * nbytes / dt)
        if dt < 0.02:
            batch *= 2
    return float(np.median(rates))


def cpu_baseline(src_host: np.ndarray, block: int, budget_s: float) -> dict:
    """The parity oracle (C restatement of the reference, -O3) on host cores.

    (ii) All usable host cores: whole 64 KiB blocks of the same C2 data,
    compressed+decompressed by one pthread per usable core -- min(CPU
    affinity, cgroup CPU quota), so threads never time-share a quota -- and
    repeated over the first blocks until ~budget_s/2 of wall time has been
    spent, throughput = raw bytes / wall time.  The same round trip on ONE
    thread is timed beside it (`single_core_c2_GiB_s`) so the multi-core
    figure can be checked against cores x single-core.
    (i) Single core, single block (benches/fse_benchmark.rs semantics): C1
    (64 KiB geometric p=0.5) and the bench-exact 32 KiB LUT p=0.2 block,
    median of repeated batches.
    """
    from oracle import oracle as O

    host = host_cpu()
    threads = host["usable_cores"]
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
    # output buffers allocated and faulted in once (an untimed first round
    # trip), then reused: the timed reps measure the coder, not first-touch
    # page faults on ~2.4 GB of fresh buffers per rep
    comp, lens, slot = O.compress2_blocks(sample, block, threads)
    out = O.decompress2_blocks(comp, slot, lens, block, len(sample), threads)
    while wall < budget_s * 0.5 and reps < 8:
        t0 = time.perf_counter()
        O.compress2_blocks(sample, block, threads, dst=comp, lens=lens)
        O.decompress2_blocks(comp, slot, lens, block, len(sample), threads, out=out)
        t1 = time.perf_counter()
        wall += t1 - t0
        total += len(sample)
        reps += 1
    assert np.array_equal(out, sample)
    # the same C2 round trip on one thread (bounded: ~budget_s/8)
    one = src_host[: block * min(n_blocks, 64)]
    t_one, n_one = 0.0, 0
    c1, l1, s1 = O.compress2_blocks(one, block, 1)
    o1 = O.decompress2_blocks(c1, s1, l1, block, len(one), 1)
    while t_one < budget_s / 8 or n_one == 0:
        t0 = time.perf_counter()
        O.compress2_blocks(one, block, 1, dst=c1, lens=l1)
        O.decompress2_blocks(c1, s1, l1, block, len(one), 1, out=o1)
        t_one += time.perf_counter() - t0
        n_one += len(one)
    assert np.array_equal(o1, one)
    single_c2 = n_one / t_one / 2**30
    single = {}
    for name, kind, prob, nb in (("C1_64KiB_geometric_p0.5", 1, 0.5, 1 << 16),
                                 ("bench_exact_32KiB_lut_p0.2", 0, 0.2, 1 << 15)):
        blk = O.generate(kind, prob, 0x5EED0001, 0, nb)
        cblk, _ = O.compress2(blk)
        assert O.decompress2(cblk, cap=1 << 17) == blk.tobytes()
        single[name] = {
            "compressed_ratio": round(len(cblk) / nb, 4),
            "encode_MiB_s": round(_median_rate(lambda: O.compress2(blk), nb, 1.0) / 2**20, 1),
            "decode_MiB_s": round(_median_rate(lambda: O.decompress2(cblk, cap=1 << 17), nb, 1.0) / 2**20, 1)}
    return {
        "value": round(total / wall / 2**30, 4),
        "unit": "GiB/s",
        "cores": threads,
        "kind": "port",
        "sample": f"{reps} x {n_take >> 20} MiB of the same C2 data ({n_take // block} x 64 KiB blocks), "
                  f"compress2+decompress2 round trip, {threads} pthreads (one per usable core: "
                  f"min(affinity {host['nproc']}, cgroup quota {host['cgroup_cpu_quota']})), "
                  f"oracle/fse_oracle.c -O3",
        "single_core_c2_GiB_s": round(single_c2, 4),
        "vs_cores_x_single": round(total / wall / 2**30 / (threads * single_c2), 3),
        "host": host,
        "single_core": single,
    }


def host_call_latency(reps: int = 20) -> dict:
    """Per-call latency of the reference-shaped host entry points (lib.rs:112-248
    drop-ins: one 64 KiB C2 block per call, host buffers, PCIe copies and the
    kernels inside the call), median of `reps`, beside the oracle (the C
    restatement of the crate, -O3) on one host core doing the same call."""
    from entropy_coders_amd import compress, compress2, decompress, decompress2, decompress2_many
    from oracle import oracle as O

    src = O.generate(0, 0.155, 0x5EED0002, 0, 65536)
    comp2, _ = compress2(src)
    comp1, _ = compress(src)
    if decompress2(comp2) != src.tobytes() or decompress(comp1) != src.tobytes():
        raise RuntimeError("host-call round trip differs from the source")

    def med_us(fn):
        fn()
        ts = []
        for _ in range(reps):
            t0 = time.perf_counter()
            fn()
            ts.append(time.perf_counter() - t0)
        return round(float(np.median(ts)) * 1e6, 1)

    cap = 1 << 17
    # the batching drop-in: 1,000 crate streams (the oracle's bytes) in one call
    many = [O.compress2(O.generate(0, 0.155, 0x5EED0002, i, 65536))[0] for i in range(1000)]
    if decompress2_many(many[:8], 65536) != [O.generate(0, 0.155, 0x5EED0002, i, 65536).tobytes()
                                             for i in range(8)]:
        raise RuntimeError("fse_decompress2_many differs from the source")
    many_np = [np.frombuffer(c, dtype=np.uint8) for c in many]
    many_dst = np.empty(len(many) * 65536, dtype=np.uint8)
    t_many = med_us(lambda: decompress2_many(many_np, 65536, raw=True, dst=many_dst))
    t_one = med_us(lambda: [O.decompress2(c, cap) for c in many[:32]]) / 32
    return {"workload": "one 64 KiB C2 block per call (host buffers in and out), median of "
                        f"{reps} calls; oracle = the C restatement on one host core",
            "fse_decompress2_many_1000": {"workload": "1,000 crate-format 64 KiB C2 streams in one "
                                                      "fse_decompress2_many call (host buffers, PCIe included)",
                                          "ms": round(t_many / 1e3, 3), "us_per_stream": round(t_many / 1000, 1),
                                          "oracle_one_core_ms": round(t_one * 1000 / 1e3, 3),
                                          "vs_one_core": round(t_one * 1000 / t_many, 2)},
            "fse_compress2_us": med_us(lambda: compress2(src)),
            "fse_decompress2_us": med_us(lambda: decompress2(comp2, cap)),
            "fse_compress_us": med_us(lambda: compress(src)),
            "fse_decompress_us": med_us(lambda: decompress(comp1, cap)),
            "oracle_compress2_us": med_us(lambda: O.compress2(src)),
            "oracle_decompress2_us": med_us(lambda: O.decompress2(comp2, cap)),
            "verified": True}


FSE_ERR_ENCODER_INIT = -17  # include/fse_status.h

C5_SWEEP = [  # BASELINE.json configs[4]: (name, generator kind, LUT p, table log)
    *[("near-uniform (0..239, H~7.9 bits)", 2, 0.0, L) for L in (9, 10, 11, 12, 13, 14, 15)],
    *[("skewed (LUT p=0.77, H~1.0 bit)", 0, 0.77, L) for L in (9, 10, 11, 12, 13, 14, 15)],
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
        if L == 15:
            # the crate's new_first_symbol panics at L = 15 unless both seed
            # symbols (the block's last two bytes) have a power-of-two count
            # (fse.rs:210-218): seed every block with two symbols outside
            # the alphabet (count 1 -> norm -1), so the row times real blocks
            full_b = nbytes // block
            seeds = src[: full_b * block].view(full_b, block)
            seeds[:, -2] = 250
            seeds[:, -1] = 251
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
        # At L = 15 the crate's Encoder::new_first_symbol (fse.rs:210-218)
        # panics whenever a seed symbol's count is not a power of two (its
        # wrapped u32 index leaves the table): those blocks report
        # ENCODER_INIT, as the reference would panic on them.  Every other
        # block must encode and round-trip exactly.
        est = cb["status"]
        good = est == 0
        n_init = int((est == FSE_ERR_ENCODER_INIT).sum())
        nb = codec.n_blocks(nbytes)
        full = nbytes // block
        ok = int(((est != 0) & (est != FSE_ERR_ENCODER_INIT)).sum()) == 0
        if ok and bool(good.any()):
            ok = int(st[good].abs().max()) == 0
        if ok and bool(good.any()):
            g = good[:full]
            ok = bool(torch.equal(out[: full * block].view(full, block)[g], src[: full * block].view(full, block)[g]))
            if nb > full and bool(good[full]):
                ok = ok and bool(torch.equal(out[full * block:], src[full * block:]))
        comp = int(cb["comp_len"].to(torch.int64).sum())
        row = {"dist": name, "table_log": L, "compressed_ratio": round(comp / nbytes, 4),
               "encode_GiB_s": round(nbytes / (enc_ms * 1e-3) / 2**30, 1),
               "decode_GiB_s": round(nbytes / (dec_ms * 1e-3) / 2**30, 1),
               "roundtrip_GiB_s": round(nbytes / ((enc_ms + dec_ms) * 1e-3) / 2**30, 1), "verified": ok}
        if L == 15:
            row["note"] = "last two bytes of every block set to symbols 250, 251 (new_first_symbol panics at L=15 otherwise)"
        if n_init:
            row["encoder_init_blocks"] = f"{n_init}/{nb} (reference panics in new_first_symbol; rates not meaningful)"
        rows.append(row)
        del codec, src, cb, out, st
    return rows


def load_traffic(name: str):
    """HBM bytes per launch of kernel `name` from profiles/traffic.json
    (tools/pmc_summary.py over the FETCH_SIZE / WRITE_SIZE passes), or None."""
    tpath = os.path.join(ROOT, "profiles", "traffic.json")
    try:
        with open(tpath) as f:
            t = json.load(f).get(name)
        return int(t["bytes_per_launch"]) if t else None
    except (OSError, ValueError, KeyError, TypeError):
        return None


def roofline_lds(kernel: str, ms: float, profiled: bool = True, alg_bytes: int = 0):
    """LDS-side roofline of a kernel whose launch took `ms` (HIP events, this
    run): its LDS-array cycles per launch summed over the CUs (rocprofv3
    SQ_LDS_IDX_ACTIVE, profiles/lds.json from the tools/gpu_run.sh pmc: pass +
    tools/lds_summary.py, same workload) per CU-cycle of this launch, at the
    clock measured in the profiled launch, against the LDS's peak of one
    array cycle per clock (MI355X_MICROARCH.md §LDS).  Conflict cycles are
    counted in (they occupy the array); `useful_frac` leaves them out."""
    if not profiled:
        return None
    try:
        with open(os.path.join(ROOT, "profiles", "lds.json")) as f:
            doc = json.load(f)
        k = doc["kernels"][kernel]
    except (OSError, ValueError, KeyError, TypeError):
        return None
    clk = k.get("clock_ghz")
    if not clk:
        return None
    cycles = ms * 1e-3 * clk * 1e9 * doc.get("cus", 256)
    busy = k["lds_array_cycles_per_launch"] / cycles
    useful = (k["lds_array_cycles_per_launch"] - k["bank_conflict_cycles_per_launch"]) / cycles
    out = {"bound": "lds", "kernel": kernel, "unit": "LDS-array cycles per CU-cycle", "achieved": round(busy, 4),
           "peak": 1.0, "frac": round(busy, 4), "useful_frac": round(useful, 4),
           "conflict_share": round(k["bank_conflict_cycles_per_launch"] / max(k["lds_array_cycles_per_launch"], 1), 4),
           "lds_array_cycles_per_launch": k["lds_array_cycles_per_launch"], "clock_ghz": clk,
           "source": "profiles/lds.json: rocprofv3 SQ_LDS_IDX_ACTIVE / SQ_LDS_BANK_CONFLICT / GRBM_GUI_ACTIVE per "
                     "launch (tools/gpu_run.sh pmc:, tools/lds_summary.py); time = this run's HIP events"}
    # the launch can take no less than its LDS-array cycles at one per CU-cycle:
    # the HBM-roofline fraction this design could reach with the LDS 100 % busy
    min_ms = k["lds_array_cycles_per_launch"] / (doc.get("cus", 256) * clk * 1e9) * 1e3
    out["min_ms_at_full_lds"] = round(min_ms, 4)
    if alg_bytes:
        out["ceiling_hbm_frac"] = round(alg_bytes / (min_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)
    if k.get("split"):
        out["split"] = k["split"]
    return out


def roofline(kernel: str, ms: float, alg_bytes: int, what: str, profiled: bool = True) -> dict:
    """`profiled`: the workload is the one tools/prof_bench.py measures (C2 / C3
    data, 64 KiB blocks, 64-pair checkpoints, optimal table log); otherwise its
    per-launch traffic does not apply and `traffic` is null."""
    achieved = alg_bytes / (ms * 1e-3) / 1e9
    return {"bound": "hbm", "kernel": kernel, "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": load_traffic(kernel) if profiled else None,
            "traffic_source": "profiles/traffic.json: rocprofv3 FETCH_SIZE x2 (gfx950 correction) + WRITE_SIZE, "
                              "per launch (tools/gpu_run.sh traffic, tools/pmc_summary.py)",
            "algorithmic_bytes_per_launch": alg_bytes, "timed": what}


def main():
    args = parse()
    self_launch(args)
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
        import datetime

        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        tmo = datetime.timedelta(seconds=300)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev, timeout=tmo)
        else:
            dist.init_process_group(backend, timeout=tmo)
    cdev = dev if backend == "nccl" else torch.device("cpu")  # where collective tensors live

    from entropy_coders_amd import BlockCodec

    codec = BlockCodec(block_size=args.block, table_log=args.table_log, ckpt_interval=args.ckpt,
                       device=dev, nstates=args.nstates)
    if args.strong:  # --bytes in total: the rank's blocks of the global order (--scheme)
        from entropy_coders_amd.dist import rank_blocks

        total_blocks = -(-args.bytes // args.block)
        mine = rank_blocks(total_blocks, rank, world, args.scheme)
        tail = args.block * total_blocks - args.bytes  # the last global block may be short
        n = len(mine) * args.block - (tail if total_blocks - 1 in mine else 0)
        job_bytes = args.bytes
    else:
        n = args.bytes
        job_bytes = world * n
    # the configuration profiles/traffic.json was measured on (tools/prof_bench.py)
    prof_base = (args.kind == 0 and args.prob == 0.155 and args.block == 65536 and args.nstates == 2
                 and args.ckpt == 64 and args.table_log == 0)
    prof_cfg = prof_base and n == 1 << 30
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
    # sentinels: a timed step that wrote nothing cannot pass the checks below
    out.fill_(0xA5)
    dstat.fill_(-99)
    cb["status"].fill_(-99)
    torch.cuda.synchronize(dev)

    # two events per step: before the encode and between encode and decode;
    # a step's decode ends where the next step's encode event is recorded
    # (each event costs ~5 us of GPU time between the kernels, profiles/r06/e/prof)
    ev_enc = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps + 1)]
    ev_mid = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps)]
    barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for k in range(args.steps):
        ev_enc[k].record(stream)
        codec.compress_into(src, cb)
        ev_mid[k].record(stream)
        codec.decompress_into(cb, out, dstat)
    ev_enc[args.steps].record(stream)
    torch.cuda.synchronize(dev)
    barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=cdev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    enc_ms = float(np.mean([ev_enc[k].elapsed_time(ev_mid[k]) for k in range(args.steps)]))
    dec_ms = float(np.mean([ev_mid[k].elapsed_time(ev_enc[k + 1]) for k in range(args.steps)]))

    # verification (outside the timed region): statuses and exact round trip
    ok = (int(cb["status"].abs().max()) == 0 and int(dstat.abs().max()) == 0
          and bool(torch.equal(out, src)))
    comp_bytes = int(cb["comp_len"].to(torch.int64).sum())
    nb = codec.n_blocks(n)

    def side_bytes_of(n_raw):  # sidecar bytes actually written/read for n_raw bytes of blocks
        if not args.ckpt:
            return 0
        per = (lambda ln: (ln // 2) // args.ckpt + 1) if args.nstates == 2 else (lambda ln: (ln - 1) // args.ckpt + 1)
        nbk = -(-n_raw // args.block)
        return 8 * sum(per(min(args.block, n_raw - b * args.block)) for b in range(nbk))

    side_bytes = side_bytes_of(n)
    if world > 1:
        flag = torch.tensor([1 if ok else 0], device=cdev)
        dist.all_reduce(flag, op=dist.ReduceOp.MIN)
        ok = bool(flag.item())

    # C4 exchange (N > 1): gatherv of the compressed shards to rank 0, then the
    # scatter back for distributed decode; verified by decoding what came back
    enc_bytes = n + comp_bytes + side_bytes  # raw read + compressed (+ sidecar) written
    dec_bytes = comp_bytes + side_bytes + n  # compressed (+ sidecar) read + raw written

    def step_line() -> dict:  # the timed step's part of the line
        line = {
            "metric": METRIC,
            "value": round(job_bytes * args.steps / elapsed / 2**30, 3),
            "unit": "GiB/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "strong" if args.strong else "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic",
            "config": {
                "workload": workload_name(args, args.bytes if args.strong else n),
                "format": "2-state (fse_compress2)" if args.nstates == 2 else "1-state (fse_compress)",
                "block_size": args.block,
                "bytes_per_gpu": n,
                "table_log": args.table_log or "optimal (11)",
                "ckpt_interval": f"{args.ckpt} {'pairs' if args.nstates == 2 else 'symbols'}",
                "parallelism": f"dp{world} (blocks sharded per GPU, no collective in the step)",
            },
            "timed_region": ("K encode + decode steps per rank on HBM-resident blocks, barrier + synchronize on "
                             "both sides, max over ranks; no collective inside (the N > 1 gather / scatter is "
                             "timed on its own in c4_exchange)"),
            # dominant kernel of the step: encode (one launch per step)
            "roofline": roofline("fse_encode_blocks", enc_ms, enc_bytes, "encode launch, HIP events", prof_cfg),
            "roofline_decode": roofline("fse_decode_blocks", dec_ms, dec_bytes,
                                        "decode-table + decode launches, HIP events", prof_cfg),
            # the encoder is bound by its LDS (random table gathers, histogram
            # atomics), not by HBM: its LDS-array occupancy beside the HBM line
            "roofline_lds": roofline_lds("fse_encode_blocks", enc_ms, prof_cfg, enc_bytes),
            "encode_ms": round(enc_ms, 4),
            "decode_ms": round(dec_ms, 4),
            "encode_GiB_s": round(n / (enc_ms * 1e-3) / 2**30, 2),
            "decode_GiB_s": round(n / (dec_ms * 1e-3) / 2**30, 2),
            "compressed_ratio": round(comp_bytes / n, 5),
            "verified_roundtrip": ok,
        }
        if enc_ms < dec_ms:
            line["roofline"], line["roofline_decode"] = line["roofline_decode"], line["roofline"]
        return line

    gather_info = None
    exchange_failed = False
    if world > 1 and not args.no_gather:
        # A collective that never completes would hold every rank, and the step's
        # line with them: past --gather-timeout each rank ends itself (os._exit
        # from a timer thread; the collectives release the GIL while they wait),
        # rank 0 after printing the line with the exchange marked timed out.
        # Either way a failed exchange ends the run with EXIT_EXCHANGE_FAILED
        # (the step's own line still printed), so it is never read as clean.
        def give_up() -> int:
            if rank == 0:
                line = step_line()
                line["c4_exchange"] = {"error": f"no result within {args.gather_timeout:g} s", "verified": False}
                print(json.dumps(line), flush=True)
            print(f"rank {rank}: C4 exchange timed out", file=sys.stderr, flush=True)
            return EXIT_EXCHANGE_FAILED if ok else EXIT_STEP_UNVERIFIED

        # ranks other than 0 wait 15 s longer: torch.distributed.run stops the
        # whole group once any rank exits, so rank 0 goes first with the line
        guard = ExchangeGuard(args.gather_timeout + (15.0 if rank else 0.0), give_up).start()
        try:
            forced = forced_exchange_failure()
            if forced == "raise":
                raise RuntimeError("forced exchange failure (FSEHIP_BENCH_FAIL_EXCHANGE=raise)")
            if forced == "hang" and rank == 1:
                time.sleep(10 * args.gather_timeout + 60)  # never joins: rank 0 waits in its collective
            gather_info = c4_exchange(args, codec, cb, src, world, rank, dev, cdev, backend, barrier)
        except Exception as e:  # reported in the line; the timed step above stands on its own checks
            gather_info = {"error": f"{type(e).__name__}: {e}"[:400], "verified": False}
            print(f"rank {rank}: C4 exchange failed: {gather_info['error']}", file=sys.stderr, flush=True)
        # the exchange is outside the timed step: its check (all ranks) is
        # c4_exchange.verified; verified_roundtrip stays the step's own
        try:
            flag = torch.tensor([1 if gather_info["verified"] else 0], device=cdev)
            dist.all_reduce(flag, op=dist.ReduceOp.MIN)
            gather_info["verified"] = bool(flag.item())
        except Exception as e:
            gather_info["verified"] = False
            gather_info.setdefault("error", f"{type(e).__name__}: {e}"[:400])
        guard.finish()
        if not gather_info["verified"]:
            exchange_failed = True
            print(f"rank {rank}: C4 exchange not verified", file=sys.stderr, flush=True)

    # the same blocks decoded without their sidecar (the format the
    # CPU crate writes): serial per block, several blocks per workgroup
    serial = None
    if not args.no_serial and world == 1 and args.nstates == 2:
        codec.decompress_into(cb, out, dstat, use_sidecar=False)  # warm-up
        out.fill_(0xA5)
        dstat.fill_(-99)
        torch.cuda.synchronize(dev)
        es = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        reps = 2
        es[0].record(stream)
        for _ in range(reps):
            codec.decompress_into(cb, out, dstat, use_sidecar=False)
        es[1].record(stream)
        torch.cuda.synchronize(dev)
        s_ms = es[0].elapsed_time(es[1]) / reps
        s_ok = int(dstat.abs().max()) == 0 and bool(torch.equal(out, src))
        serial = {"workload": "the step's compressed blocks decoded without the sidecar (decode tables + "
                              "serial_ring_kernel, symbols deferred to sym_map_kernel), HIP events",
                  "decode_ms": round(s_ms, 4), "decode_GiB_s": round(n / (s_ms * 1e-3) / 2**30, 2),
                  "verified": s_ok}
        ok = ok and s_ok

    # C3 (BASELINE configs[2]): decode only, decode tables prebuilt and untimed,
    # on its own 32768 blocks of C2 data (~1 GiB compressed)
    c3 = None
    if not args.no_c3 and world == 1:
        n3 = args.c3_blocks * args.block
        del out
        src3 = codec.generate(args.kind, args.prob, 0x5EED0003, n3)
        cb3 = codec.alloc(n3)
        codec.compress_into(src3, cb3)
        tabs = codec.build_dtables(cb3)
        out3 = torch.empty(n3, dtype=torch.uint8, device=dev)
        st3 = torch.zeros(codec.n_blocks(n3), dtype=torch.int32, device=dev)
        codec.decompress_dt_into(cb3, tabs, out3, st3)  # warm-up
        out3.fill_(0xA5)
        st3.fill_(-99)
        torch.cuda.synchronize(dev)
        e3 = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        e3[0].record(stream)
        for _ in range(args.steps):
            codec.decompress_dt_into(cb3, tabs, out3, st3)
        e3[1].record(stream)
        torch.cuda.synchronize(dev)
        c3_ms = e3[0].elapsed_time(e3[1]) / args.steps
        c3_ok = int(cb3["status"].abs().max()) == 0 and int(st3.abs().max()) == 0 and bool(torch.equal(out3, src3))
        comp3 = int(cb3["comp_len"].to(torch.int64).sum())
        c3_bytes = comp3 + side_bytes_of(n3) + n3  # compressed + sidecar read, raw written
        c3 = {"workload": f"C3: decode only, {args.c3_blocks} x {args.block // 1024} KiB blocks of C2 data "
                          f"({comp3 / 2**30:.3f} GiB compressed -> {n3 / 2**30:.3f} GiB), decode tables and "
                          "sidecar prebuilt and untimed",
              "decode_ms": round(c3_ms, 4), "decode_GiB_s": round(n3 / (c3_ms * 1e-3) / 2**30, 2),
              "roofline": roofline("fse_decode_blocks_c3", c3_ms, c3_bytes,
                                   "decode launches (prebuilt tables), HIP events",
                                   prof_base and args.c3_blocks == 32768),
              # the same launch priced on the reference format's bytes only
              # (compressed read + raw written; the sidecar is this port's own)
              "frac_reference_format_bytes": round((comp3 + n3) / (c3_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
              "roofline_lds": roofline_lds("fse_decode_blocks_c3", c3_ms, prof_base and args.c3_blocks == 32768,
                                           c3_bytes),
              "verified": c3_ok}
        ok = ok and c3_ok
        del src3, cb3, tabs, out3, st3

    # the same 1 GiB in the 1-state format (fse_compress blocks,
    # lib.rs:112-141 / 187-211), encode + decode with its sidecar, verified
    one_state = None
    if not args.no_onestate and world == 1 and args.nstates == 2:
        # checkpoints every 2 x ckpt symbols (the 2-state step's segment length in symbols: one
        # segment per thread of the 512-thread workgroups; 1,057-1,061 vs 1,013-1,020 GiB/s
        # decode at 4 x ckpt, same box)
        c1 = BlockCodec(block_size=args.block, ckpt_interval=int(os.environ.get("FSEHIP_CKPT1", 2 * args.ckpt)),
                        device=dev, nstates=1)
        cb1 = c1.alloc(n)
        out1 = torch.empty(n, dtype=torch.uint8, device=dev)
        st1 = torch.zeros(c1.n_blocks(n), dtype=torch.int32, device=dev)
        c1.compress_into(src, cb1)  # warm-up
        c1.decompress_into(cb1, out1, st1)
        out1.fill_(0xA5)
        st1.fill_(-99)
        torch.cuda.synchronize(dev)
        e1 = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
        reps = 3
        e1[0].record(stream)
        for _ in range(reps):
            c1.compress_into(src, cb1)
        e1[1].record(stream)
        for _ in range(reps):
            c1.decompress_into(cb1, out1, st1)
        e1[2].record(stream)
        torch.cuda.synchronize(dev)
        enc1, dec1 = e1[0].elapsed_time(e1[1]) / reps, e1[1].elapsed_time(e1[2]) / reps
        ok1 = int(cb1["status"].abs().max()) == 0 and int(st1.abs().max()) == 0 and bool(torch.equal(out1, src))
        one_state = {"workload": "the step's 1 GiB as 1-state blocks (fse_compress), encode + decode with the "
                                 f"sidecar ({c1.ckpt_interval}-symbol checkpoints), HIP events",
                     "compressed_ratio": round(int(cb1["comp_len"].to(torch.int64).sum()) / n, 5),
                     "encode_GiB_s": round(n / (enc1 * 1e-3) / 2**30, 2),
                     "decode_GiB_s": round(n / (dec1 * 1e-3) / 2**30, 2),
                     "roundtrip_GiB_s": round(n / ((enc1 + dec1) * 1e-3) / 2**30, 2), "verified": ok1}
        ok = ok and ok1
        del c1, cb1, out1, st1

    host_info = None
    if args.host and world == 1:
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

    # every table of the run checked its atomic ranks (fse_device.hpp
    # wave_build_spread); a fallback is a table rebuilt with peer-mask ranks
    rank_check = codec.rank_fallbacks()
    if rank == 0:
        line = step_line()
        line["rank_check"] = {"fallback_tables": rank_check,
                              "what": "tables of this run (all of them check their LDS-atomic ranks) rebuilt with "
                                      "peer-mask ranks because the check failed; 0 on a correct GPU"}
        if c3 is not None:
            line["c3_decode_only"] = c3
        if serial is not None:
            line["sidecar_less_decode"] = serial
        if one_state is not None:
            line["one_state"] = one_state
        if gather_info is not None:
            line["c4_exchange"] = gather_info
        if host_info is not None:
            line["host_pipeline"] = host_info
        if not args.no_sweep and args.nstates == 2 and world == 1:
            sw = c5_sweep(dev, args.sweep_bytes, args.block, args.ckpt)
            line["c5_sweep"] = {"workload": f"C5: {args.sweep_bytes >> 20} MiB per distribution and table log, "
                                            "encode + decode (2-state), 1 GPU", "rows": sw}
            ok = ok and all(r["verified"] for r in sw)
            line["verified_roundtrip"] = ok
        if world == 1 and not args.no_cpu:
            line["cpu_baseline"] = cpu_baseline(src.cpu().numpy(), args.block, args.cpu_seconds)
        if world == 1 and not args.no_host_calls:
            # after the verified step: a failure here is recorded in the line
            # (and fails the run's verification) but never loses the line
            try:
                line["host_call_latency"] = host_call_latency()
            except Exception as e:
                line["host_call_latency"] = {"error": f"{type(e).__name__}: {e}"[:300], "verified": False}
                ok = False
                line["verified_roundtrip"] = False
        print(json.dumps(line), flush=True)
    if world > 1:
        # every rank stays until rank 0 has printed the line (a rank exiting
        # non-zero first would make torch.distributed.run stop rank 0)
        try:
            barrier()
        except Exception as e:
            print(f"rank {rank}: final barrier failed: {type(e).__name__}: {e}"[:300], file=sys.stderr, flush=True)
        dist.destroy_process_group()
    if not ok:
        sys.exit(EXIT_STEP_UNVERIFIED)
    if exchange_failed:
        sys.exit(EXIT_EXCHANGE_FAILED)


def c4_exchange(args, codec, cb, src, world, rank, dev, cdev, backend, barrier) -> dict:
    """BASELINE configs[3] / SURVEY 8(e): pack each rank's blocks on the GPU,
    gatherv them (lengths, bytes, sidecar) to rank 0 over RCCL, then scatter
    the global stream back and decode each rank's received shard.  Timed
    separately from `value`; the gather is reported as achieved GB/s into
    rank 0 against the 7-link xGMI ingress roof."""
    import torch

    from entropy_coders_amd.dist import (concat_global, gather_stream, pack_device, scatter_stream,
                                         unpack_device)

    nb = codec.n_blocks(cb["n_total"])
    side = cb["sidecar"][: nb * codec.side_per_block] if args.ckpt else None
    to_c = (lambda t: t) if backend == "nccl" else (lambda t: t.cpu() if t is not None else None)

    packed, _ = pack_device(cb["out"], codec.slot_bytes, cb["comp_len"])
    torch.cuda.synchronize(dev)
    barrier()
    g0 = time.perf_counter()
    packed, _ = pack_device(cb["out"], codec.slot_bytes, cb["comp_len"])
    torch.cuda.synchronize(dev)
    tp = time.perf_counter()
    res = gather_stream(to_c(packed), to_c(cb["comp_len"]), dst=0, sidecar=to_c(side))
    torch.cuda.synchronize(dev)
    barrier()
    g1 = time.perf_counter()
    streams, lens, sides = res
    recv_bytes = 0
    g_stream = g_lens = g_side = None
    n_global = 0
    sizes = torch.tensor([nb], dtype=torch.int64, device=cdev)
    allnb = [torch.zeros_like(sizes) for _ in range(world)]
    import torch.distributed as dist

    dist.all_gather(allnb, sizes)
    n_global = int(sum(int(x) for x in allnb))
    if rank == 0:
        recv_bytes = sum(int(s.numel()) for r, s in enumerate(streams) if r != 0)
        recv_bytes += sum(int(s.numel()) * 8 for r, s in enumerate(sides) if r != 0 and s is not None)
        g_stream, g_lens, g_side = concat_global(streams, lens, n_global, world, args.scheme,
                                                 sides if side is not None else None)
    torch.cuda.synchronize(dev)
    barrier()
    s0 = time.perf_counter()
    my, my_lens, my_side, idx = scatter_stream(g_stream, g_lens, src=0, sidecar=g_side,
                                               side_per_block=codec.side_per_block, scheme=args.scheme,
                                               device=cdev)
    torch.cuda.synchronize(dev)
    barrier()
    s1 = time.perf_counter()
    # decode what came back: rank r's j-th block of the global order is its local block j
    my, my_lens = my.to(dev), my_lens.to(dev)
    slots = unpack_device(my, my_lens, codec.slot_bytes)
    cb2 = {"n_total": cb["n_total"], "out": slots, "comp_len": my_lens,
           "sidecar": my_side.to(dev) if my_side is not None else cb["sidecar"]}
    out2 = torch.full((cb["n_total"],), 0xA5, dtype=torch.uint8, device=dev)
    st2 = torch.full((nb,), -99, dtype=torch.int32, device=dev)
    codec.decompress_into(cb2, out2, st2, use_sidecar=my_side is not None)
    torch.cuda.synchronize(dev)
    ok = (len(idx) == nb and int(st2.abs().max()) == 0 and bool(torch.equal(out2, src))
          and bool(torch.equal(my_lens.cpu(), cb["comp_len"].cpu())))
    xgmi_roof = 153.0 * min(world - 1, 7)
    gather_gbs = recv_bytes / max(g1 - tp, 1e-9) / 1e9
    return {"scheme": args.scheme, "backend": backend,
            "packed_bytes_rank0": int(packed.numel()),
            "gathered_bytes_into_rank0": recv_bytes,
            "pack_ms": round((tp - g0) * 1e3, 3),
            "gather_ms": round((g1 - tp) * 1e3, 3),
            "gather_GB_s_into_rank0": round(gather_gbs, 2),
            "xgmi_ingress_roof_GB_s": xgmi_roof,
            "gather_roof_frac": round(gather_gbs / xgmi_roof, 4) if backend == "nccl" else None,
            "scatter_ms": round((s1 - s0) * 1e3, 3),
            "verified": ok}


if __name__ == "__main__":
    main()
