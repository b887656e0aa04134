"""Recompute the bench line's HBM-roofline fractions from a rocprofv3 kernel
trace of the same command (tools/kernel_by_grid.py rows), so profiles/
reproduce the line: encode, C2 decode (header parse + tables + decode) and
C3 decode-only, from the per-(kernel, grid) average durations.

    python tools/frac_check.py profiles/r05/nosweep/bench_prof.json \
        profiles/r05/nosweep/bench_kernel_trace.csv
"""
import csv
import json
import sys
from collections import defaultdict

PEAK = 8000.0  # GB/s


def rows(trace):
    r = defaultdict(list)
    for x in csv.DictReader(open(trace)):
        if "fsehip" not in x["Kernel_Name"]:
            continue
        g = int(x["Grid_Size_X"]) // max(int(x["Workgroup_Size_X"]), 1)
        r[(x["Kernel_Name"], g)].append((int(x["End_Timestamp"]) - int(x["Start_Timestamp"])) / 1e6)
    return r


def avg(r, name, grid):
    v = [t for (k, g), ts in r.items() if name in k and g == grid for t in ts]
    return (sum(v) / len(v), len(v)) if v else (0.0, 0)


def main():
    line = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
    r = rows(sys.argv[2])
    nb = line["config"].get("n_blocks", 16384) if isinstance(line.get("config"), dict) else 16384
    c3b = 32768
    out = []
    enc, n = avg(r, "encode_blocks_kernel<11, 64, 2>", nb)
    alg = line["roofline"]["algorithmic_bytes_per_launch"]
    out.append(("encode", n, enc, alg / enc / 1e6 / PEAK, line["roofline"]["frac"]))
    hp, _ = avg(r, "hdr_parse_kernel<11>", nb // 16)
    dt, _ = avg(r, "dtable_blocks_kernel<11>", nb)
    dt = dt or avg(r, "dtable_par_kernel<11>", nb)[0]
    dp, n = avg(r, "decode_pre_kernel<11, 45056u, 2, 1, 512u>", nb)
    rd = line["roofline_decode"]
    dec = hp + dt + dp
    out.append(("C2 decode (parse+tables+decode)", n, dec, rd["algorithmic_bytes_per_launch"] / dec / 1e6 / PEAK,
                rd["frac"]))
    c3, n = avg(r, "decode_pre_kernel<11, 45056u, 2, 1, 512u>", c3b)
    rc = line["c3_decode_only"]["roofline"]
    out.append(("C3 decode-only", n, c3, rc["algorithmic_bytes_per_launch"] / c3 / 1e6 / PEAK, rc["frac"]))
    print(f"{'launch':34s} {'calls':>5s} {'rocprof avg ms':>14s} {'frac (rocprof)':>14s} {'frac (bench)':>12s} {'diff':>7s}")
    for name, n, ms, f, fb in out:
        print(f"{name:34s} {n:5d} {ms:14.4f} {f:14.4f} {fb:12.4f} {100 * (f / fb - 1):+6.1f}%")


if __name__ == "__main__":
    main()
