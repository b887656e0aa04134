"""LDS-side roofline inputs from the SQ counter passes of tools/gpu_run.sh pmc:
(over tools/prof_bench.py): per fse kernel launch kind (last launch of each
kind), the LDS-array cycles of one launch summed over the CUs
(SQ_LDS_IDX_ACTIVE), the bank-conflict cycles among them
(SQ_LDS_BANK_CONFLICT), the LDS instructions, and the GPU clock of the
profiled launch (GRBM_GUI_ACTIVE over 8 XCDs / the launch's duration in the
same pass).  bench.py turns these into `roofline_lds`: LDS-array cycles per
CU-cycle of the live launch against the peak of one per cycle
(MI355X_MICROARCH.md §LDS: 64 banks, one LDS cycle per lane group when
conflict-free).

    python tools/lds_summary.py gpurun_out/pmc [--json profiles/lds.json]
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_summary import classify  # noqa: E402

CUS = 256
KEYS = ("SQ_LDS_IDX_ACTIVE", "SQ_LDS_BANK_CONFLICT", "SQ_INSTS_LDS", "GRBM_GUI_ACTIVE")


def main():
    d = sys.argv[1]
    vals = defaultdict(dict)
    dur = defaultdict(dict)  # kind -> counter -> duration (ns) of the launch it came from
    for f in sorted(glob.glob(f"{d}/p*/**/*counter_collection.csv", recursive=True)):
        seen = defaultdict(set)
        for r in csv.DictReader(open(f)):
            groups = int(r["Grid_Size"]) // max(int(r["Workgroup_Size"]), 1)
            seen[r["Kernel_Name"]].add(int(r["Dispatch_Id"]))
            name = classify(r["Kernel_Name"], groups, len(seen[r["Kernel_Name"]]) - 1)
            if not name or r["Counter_Name"] not in KEYS:
                continue
            vals[name][r["Counter_Name"]] = float(r["Counter_Value"])  # last launch wins
            dur[name][r["Counter_Name"]] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    out = {}
    for name, v in sorted(vals.items()):
        if "SQ_LDS_IDX_ACTIVE" not in v or "GRBM_GUI_ACTIVE" not in v:
            continue
        gpu_cycles = v["GRBM_GUI_ACTIVE"] / 8.0  # summed over the 8 XCDs
        ns = dur[name]["GRBM_GUI_ACTIVE"]
        clk = gpu_cycles / ns if ns > 0 else None  # GHz
        row = {
            "lds_array_cycles_per_launch": int(v["SQ_LDS_IDX_ACTIVE"]),
            "bank_conflict_cycles_per_launch": int(v.get("SQ_LDS_BANK_CONFLICT", 0)),
            "lds_instructions_per_launch": int(v.get("SQ_INSTS_LDS", 0)),
            "gpu_cycles_per_launch": int(gpu_cycles),
            "clock_ghz": round(clk, 4) if clk else None,
            "lds_busy_per_cu_cycle_profiled": round(v["SQ_LDS_IDX_ACTIVE"] / (CUS * gpu_cycles), 4),
        }
        out[name] = row
        print(name, json.dumps(row))
    if "--json" in sys.argv:
        path = sys.argv[sys.argv.index("--json") + 1]
        if os.path.exists(path):  # keep the probe-derived splits (tools/lds_split*.py) of the kernels
            old = json.load(open(path)).get("kernels", {})
            for name, row in out.items():
                if "split" in old.get(name, {}):
                    row["split"] = old[name]["split"]
        with open(path, "w") as fh:
            json.dump({"source": "rocprofv3 --pmc SQ pass (tools/gpu_run.sh pmc:SQ_LDS_IDX_ACTIVE,...) over "
                                 "tools/prof_bench.py, last launch of each kind; tools/lds_summary.py",
                       "cus": CUS, "kernels": out}, fh, indent=1)


if __name__ == "__main__":
    main()
