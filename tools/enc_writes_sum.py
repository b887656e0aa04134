"""Summarise tools/enc_writes.sh: bytes per encode launch (second launch of
each configuration A-D, see tools/enc_writes.py) for WRITE_SIZE and
FETCH_SIZE x 2 (the gfx950 correction), and the attribution
payload = A - C, sidecar = A - B, header + merge = D.

    python tools/enc_writes_sum.py gpurun_out/encw [--json out.json]"""
import csv
import glob
import json
import sys
from collections import defaultdict


def per_dispatch(d, counter):
    vals = defaultdict(float)
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if "encode_blocks_kernel" in r["Kernel_Name"] and r["Counter_Name"] == counter:
                vals[int(r["Dispatch_Id"])] += float(r["Counter_Value"])
    return [vals[k] for k in sorted(vals)]


def main():
    d = sys.argv[1]
    w = per_dispatch(f"{d}/write", "WRITE_SIZE")
    f = per_dispatch(f"{d}/fetch", "FETCH_SIZE")
    names = "ABCD"
    # counters are in KiB; launches 2i (first) and 2i + 1 (second) belong to config i
    W = {names[i]: w[2 * i + 1] * 1024 for i in range(4)} if len(w) >= 8 else {}
    F = {names[i]: 2 * f[2 * i + 1] * 1024 for i in range(4)} if len(f) >= 8 else {}
    logs = {}
    for line in open(f"{d}/write.log"):
        p = line.split()
        if len(p) == 5 and p[0] in names:
            logs[p[0]] = {"compressed": float(p[2]), "sidecar_written": float(p[4])}
    out = {"write_bytes": W, "fetch_bytes_x2": F, "algorithmic": logs}
    if W:
        out["attribution"] = {"payload_stores": W["A"] - W["C"], "sidecar": W["A"] - W["B"],
                              "header_and_merge": W["D"], "write_over_compressed_plus_sidecar":
                              W["A"] / (logs["A"]["compressed"] + logs["A"]["sidecar_written"])}
    print(json.dumps(out, indent=1))
    if "--json" in sys.argv:
        json.dump(out, open(sys.argv[sys.argv.index("--json") + 1], "w"), indent=1)


if __name__ == "__main__":
    main()
