"""Summarise tools/pmc_phases.sh: encode-kernel counters per ablation level."""
import csv
import glob
import sys

d = sys.argv[1]
for D in ("8", "1", "2", "4", "0"):
    vals = {}
    for f in glob.glob(f"{d}/{D}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if "encode_blocks" in r["Kernel_Name"]:
                vals[r["Counter_Name"]] = float(r["Counter_Value"])
    print(f"debug={D}: " + "  ".join(f"{k}={v:.3g}" for k, v in sorted(vals.items())))
