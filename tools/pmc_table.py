"""Print SQ counters per fse kernel from a tools/pmc_*.sh output dir (last dispatch of each kernel)."""
import csv
import glob
import sys
from collections import defaultdict

d = sys.argv[1]
vals = defaultdict(dict)
for f in sorted(glob.glob(f"{d}/p*/**/*counter_collection.csv", recursive=True)):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"]
        if "fsehip" not in k:
            continue
        k = k.split("(")[0].replace("void ", "").replace("fsehip::", "")
        vals[k][r["Counter_Name"]] = float(r["Counter_Value"])
for k, v in vals.items():
    print(k)
    for c, x in sorted(v.items()):
        print(f"   {c:24s} {x:.4g}")
for f in glob.glob(f"{d}/kt/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        print(f"{r['Name'][:70]:70s} calls={r['Calls']} avg_us={float(r['AverageNs'])/1e3:.1f}")
