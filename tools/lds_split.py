"""Split the segment decoder's LDS-array cycles per 64-lane pair step into
its table gathers and its payload read (verdict r04 item 3), from three
counter passes (tools/gpu_run.sh pmc: + tools/lds_summary.py) over the same
workload: the product and two one-read probes built with
tools/variant_build.sh --
  FSEHIP_ABL=256: one more random table-like gather per pair (an extra
                  ds_read_b32: LDS instructions +1 per pair step);
  FSEHIP_ABL=512: the payload read widened to the word below as well (the
                  compiler merges it into the existing read: same instruction
                  count, the extra cycles are those of a second payload word).
Writes the split into profiles/lds.json (kernels[...]["split"]), where
bench.py's roofline_lds picks it up.

    python tools/lds_split.py gpurun_out/r05_e profiles/lds.json
"""
import json
import sys

PAIRS = {"fse_decode_blocks": 16384 * 32767, "fse_decode_blocks_c3": 32768 * 32767}  # C2 / C3 pair steps


def load(path):
    out = {}
    for line in open(path):
        name, _, js = line.partition(" ")
        if js.startswith("{"):
            out[name] = json.loads(js)
    return out


def main():
    d, lds_json = sys.argv[1], sys.argv[2]
    base = load(f"{d}/lds_libfsehip.so.txt")
    t = load(f"{d}/lds_libfsehip_abl256.so.txt")
    p = load(f"{d}/lds_libfsehip_abl512.so.txt")
    doc = json.load(open(lds_json))
    for k, pairs in PAIRS.items():
        steps = pairs / 64.0  # wave-wide pair steps
        b = base[k]["lds_array_cycles_per_launch"] / steps
        bi = base[k]["lds_instructions_per_launch"] / steps
        dt = (t[k]["lds_array_cycles_per_launch"] - base[k]["lds_array_cycles_per_launch"]) / steps
        dti = (t[k]["lds_instructions_per_launch"] - base[k]["lds_instructions_per_launch"]) / steps
        dp = (p[k]["lds_array_cycles_per_launch"] - base[k]["lds_array_cycles_per_launch"]) / steps
        gather = dt / max(dti, 1e-9)  # cycles per extra table-like gather instruction
        tables = 2.0 * gather
        rest = b - tables
        split = {"unit": "LDS-array cycles per 64-lane pair step", "total": round(b, 2),
                 "lds_instructions_per_step": round(bi, 3),
                 "table_gathers": round(tables, 2), "per_table_gather": round(gather, 2),
                 "payload_read_and_other": round(rest, 2), "second_payload_word": round(dp, 2),
                 "conflict_free_gather_floor": 2.0,
                 "source": "product vs FSEHIP_ABL=256 / 512 builds, one rocprofv3 SQ pass each "
                           "(tools/gpu_r05_e.sh, tools/lds_split.py)"}
        doc["kernels"].setdefault(k, dict(base[k]))["split"] = split
        print(k, json.dumps(split))
    json.dump(doc, open(lds_json, "w"), indent=1)


if __name__ == "__main__":
    main()
