"""Per (kernel, grid) launch statistics from a rocprofv3 kernel trace, so
launches of different sizes (C2 1 GiB vs C3 2 GiB) are not averaged
together as in the --stats summary.

    python tools/kernel_by_grid.py gpurun_out/prof/run_kernel_trace.csv
"""
import csv
import sys
from collections import defaultdict

rows = defaultdict(list)
for r in csv.DictReader(open(sys.argv[1])):
    if "fsehip" not in r["Kernel_Name"]:
        continue
    groups = int(r["Grid_Size_X"]) // max(int(r["Workgroup_Size_X"]), 1)
    rows[(r["Kernel_Name"], groups)].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
print(f"{'kernel':72s} {'workgroups':>10s} {'calls':>5s} {'avg ms':>9s} {'min ms':>9s}")
for (k, g), v in sorted(rows.items(), key=lambda kv: -sum(kv[1])):
    print(f"{k[:72]:72s} {g:10d} {len(v):5d} {sum(v) / len(v):9.4f} {min(v):9.4f}")
