"""Summarise rocprofv3 FETCH_SIZE / WRITE_SIZE passes (tools/gpu_run.sh traffic over
tools/prof_bench.py) into per-launch HBM bytes for the fse kernels, with the
gfx950 corrections of MI355X_MICROARCH.md (HBM section): counters are in
KiB; FETCH_SIZE reports half the bytes of wide coalesced reads, so it is
doubled (upper bound for narrower access); WRITE_SIZE is taken as reported.

Launches are told apart by kernel name and grid (workgroups): C2 runs 16384
blocks, C3 32768; the decode's second launch (66 KiB stage, 67584u) only
decodes blocks deferred by the first, none on C2 data.

    python tools/pmc_summary.py gpurun_out/traffic [--json profiles/traffic.json]
"""
import csv
import glob
import json
import sys
from collections import defaultdict


def classify(kernel: str, groups: int, nth: int = 0):
    """Launch kind; `nth` = 0-based occurrence of this kernel name in the run
    (the pipelined decode runs a fixed grid: tools/prof_bench.py launches it
    twice on C2, then twice on C3)."""
    c3 = groups == 32768
    if "decode_pipe_kernel" in kernel:
        return "fse_decode_blocks" + ("_c3" if nth >= 2 else "")
    if "encode_blocks_kernel" in kernel:
        return "fse_encode_blocks" + ("_c3_input" if c3 else "")
    if "dtable_blocks_kernel" in kernel or "dtable_par_kernel" in kernel:
        return "fse_build_dtables" + ("_c3" if c3 else "")
    if "hdr_parse_kernel" in kernel:  # 16 headers per workgroup: 1,024 at C2, 2,048 at C3
        return "fse_hdr_parse" + ("_c3" if groups == 2048 else "")
    if "decode_pre_kernel" in kernel:
        if "67584u" in kernel:  # the list pass: a fixed grid, C2 launches first (twice), then C3
            return "fse_decode_deferred" + ("_c3" if nth >= 2 else "")
        return "fse_decode_blocks" + ("_c3" if c3 else "")
    for k, name in (("serial_ring_kernel", "fse_decode_serial"), ("serial2_decode_kernel", "fse_decode_serial2"), ("decode_blocks_kernel", "fse_decode_fused"),
                    ("decode1_serial_kernel", "fse_decode1_serial"), ("pack_blocks_kernel", "fse_pack_blocks"),
                    ("copy_blocks_kernel", "fse_copy_blocks"), ("generate_kernel", "fse_generate")):
        if k in kernel:
            return name
    return None


def load(d, counter):
    vals = defaultdict(list)
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        seen = defaultdict(set)
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] != counter:
                continue
            groups = int(r["Grid_Size"]) // max(int(r["Workgroup_Size"]), 1)
            seen[r["Kernel_Name"]].add(int(r["Dispatch_Id"]))
            name = classify(r["Kernel_Name"], groups, len(seen[r["Kernel_Name"]]) - 1)
            if name:
                vals[name].append(float(r["Counter_Value"]) * 1024.0)
    return vals


def main():
    d = sys.argv[1]
    fetch = load(f"{d}/fetch", "FETCH_SIZE")
    write = load(f"{d}/write", "WRITE_SIZE")
    out = {}
    for name in sorted(set(fetch) | set(write)):
        f = fetch.get(name, [])
        w = write.get(name, [])
        # last launch of each kind (the first may see a cold Infinity Cache)
        fb = 2.0 * f[-1] if f else None
        wb = w[-1] if w else None
        out[name] = {"bytes_per_launch": (fb or 0) + (wb or 0), "fetch_bytes_corrected": fb,
                     "fetch_bytes_raw": f[-1] if f else None, "write_bytes": wb, "launches": max(len(f), len(w))}
        print(name, json.dumps(out[name]))
    if "--json" in sys.argv:
        path = sys.argv[sys.argv.index("--json") + 1]
        with open(path, "w") as fh:
            json.dump(out, fh, indent=1)


if __name__ == "__main__":
    main()
