"""Summarise rocprofv3 counter passes of the encode kernel: one line per run
directory (tools/pmc_phases.sh, tools/pmc_phases_lds.sh: d<FSEHIP_DEBUG>;
tools/pmc_enc_var.sh: d<lanes>/e<lanes>).  Usage: pmc_phases_table.py DIR [run,run,...]"""
import csv
import glob
import os
import sys

d = sys.argv[1]
runs = sys.argv[2].split(",") if len(sys.argv) > 2 else sorted(
    os.path.basename(p) for p in glob.glob(f"{d}/*") if os.path.isdir(p))
for D in runs:
    vals = {}
    for f in glob.glob(f"{d}/{D}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if "encode_blocks" in r["Kernel_Name"]:
                vals[r["Counter_Name"]] = float(r["Counter_Value"])
    print(f"{D}: " + "  ".join(f"{k}={v:.3g}" for k, v in sorted(vals.items())))
