"""Summarise the SQ counter passes of tools/gpu_run.sh pmc: (over
tools/prof_bench.py) per fse kernel launch kind (last launch of each kind),
with per-symbol ratios: VALU and LDS instructions per symbol (wave
instructions x 64 lanes / raw bytes), LDS bank-conflict cycles as a fraction
of LDS-array cycles, and the wave-cycle split (issuing / waiting / stalled).

    python tools/pmc_sq.py gpurun_out/pmc [--json profiles/r02_pmc.json]
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_summary import classify  # noqa: E402

RAW = {"": 1 << 30, "_c3": 32768 * 65536, "_c3_input": 32768 * 65536}


def main():
    d = sys.argv[1]
    vals = defaultdict(dict)
    for f in sorted(glob.glob(f"{d}/p*/**/*counter_collection.csv", recursive=True)):
        seen = defaultdict(set)
        for r in csv.DictReader(open(f)):
            groups = int(r["Grid_Size"]) // max(int(r["Workgroup_Size"]), 1)
            seen[r["Kernel_Name"]].add(int(r["Dispatch_Id"]))
            name = classify(r["Kernel_Name"], groups, len(seen[r["Kernel_Name"]]) - 1)
            if not name:
                continue
            vals[name][r["Counter_Name"]] = float(r["Counter_Value"])  # last launch wins
    out = {}
    for name, v in sorted(vals.items()):
        raw = RAW["_c3" if name.endswith("_c3") else "_c3_input" if name.endswith("_c3_input") else ""]
        row = dict(v)
        if "SQ_INSTS_VALU" in v:
            row["valu_lane_ops_per_symbol"] = round(v["SQ_INSTS_VALU"] * 64 / raw, 3)
        if "SQ_INSTS_LDS" in v:
            row["lds_lane_ops_per_symbol"] = round(v["SQ_INSTS_LDS"] * 64 / raw, 3)
        if v.get("SQ_LDS_IDX_ACTIVE"):
            row["lds_bank_conflict_frac"] = round(v.get("SQ_LDS_BANK_CONFLICT", 0) / v["SQ_LDS_IDX_ACTIVE"], 4)
        wc = v.get("SQ_WAVE_CYCLES")
        if wc:
            for k in ("SQ_ACTIVE_INST_ANY", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_WAIT_INST_LDS"):
                if k in v:
                    row[k.lower() + "_frac_of_wave_cycles"] = round(v[k] / wc, 4)
        if v.get("GRBM_GUI_ACTIVE") and "SQ_LDS_IDX_ACTIVE" in v:
            # LDS-array busy cycles per CU per GPU cycle (256 CUs)
            # GRBM_GUI_ACTIVE sums the 8 XCDs: per-XCD cycles = / 8
            row["lds_busy_per_cu_cycle"] = round(v["SQ_LDS_IDX_ACTIVE"] / (v["GRBM_GUI_ACTIVE"] / 8 * 256), 4)
        out[name] = row
        print(name, json.dumps({k: x for k, x in row.items() if not k.startswith("SQ_") and not k.startswith("GRBM")}))
    if "--json" in sys.argv:
        with open(sys.argv[sys.argv.index("--json") + 1], "w") as fh:
            json.dump({"source": "rocprofv3 --pmc SQ passes (tools/gpu_run.sh pmc:) over tools/prof_bench.py, "
                                 "last launch of each kind", "raw_bytes_per_launch": RAW, "kernels": out}, fh, indent=1)


if __name__ == "__main__":
    main()
