"""Summarise rocprofv3 FETCH_SIZE / WRITE_SIZE passes (tools/traffic.sh) into
per-launch HBM bytes for the fse kernels, with the gfx950 corrections of
MI355X_MICROARCH.md (HBM section): counters are in KiB; FETCH_SIZE reports
half the bytes of wide coalesced reads, so it is doubled (upper bound for
narrower access); WRITE_SIZE is taken as reported.

    python tools/pmc_summary.py gpurun_out/traffic [--json profiles/traffic.json]
"""
import csv
import glob
import json
import sys
from collections import defaultdict

KERNELS = {"encode_blocks_kernel": "fse_encode_blocks", "decode_blocks_kernel": "fse_decode_blocks_fused",
           "decode_pre_kernel": "fse_decode_blocks", "dtable_blocks_kernel": "fse_build_dtables",
           "decode1_serial_kernel": "fse_decode1_serial",
           "pack_blocks_kernel": "fse_pack_blocks", "generate_kernel": "fse_generate"}


def load(d, counter):
    vals = defaultdict(list)
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] != counter:
                continue
            for k, name in KERNELS.items():
                if k in r["Kernel_Name"]:
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
        out[name] = {"fetch_bytes_corrected": fb, "fetch_bytes_raw": f[-1] if f else None,
                     "write_bytes": wb, "hbm_bytes": (fb or 0) + (wb or 0), "launches": max(len(f), len(w))}
        print(name, json.dumps(out[name]))
    if "--json" in sys.argv:
        path = sys.argv[sys.argv.index("--json") + 1]
        with open(path, "w") as fh:
            json.dump({k: {"bytes_per_launch": v["hbm_bytes"], **v} for k, v in out.items()}, fh, indent=1)


if __name__ == "__main__":
    main()
