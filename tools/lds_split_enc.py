"""Split the encoder's LDS-array cycles into its two gathers per state step
(encoder "Round 5" item 9), from one counter pass over
the product and over two one-gather probes built with tools/variant_build.sh
(tools/gpu_r05_v.sh / gpu_r05_w.sh):
  FSEHIP_ENC_ABL=64:  one more stateTable gather per pair (chain 0's
                      address one bank over);
  FSEHIP_ENC_ABL=128: one more transform gather per pair (the neighbour
                      symbol's);
their reads folded into a register tested once, so nothing waits on them.
The probes' extra LDS instructions count the wave pair-steps of a launch.
Also reads the C2 encode times of the three builds (enc_split_time.txt) for
what one more gather per pair costs in time.  Writes the split into
profiles/lds.json (kernels["fse_encode_blocks"]["split"]), where bench.py's
roofline_lds picks it up; rerun after refreshing profiles/lds.json.

    python tools/lds_split_enc.py profiles/r05/enc_lds_split profiles/lds.json
"""
import json
import statistics
import sys

K = "fse_encode_blocks"
BLOCKS = 16384  # C2: 1 GiB of 64 KiB blocks


def load(path):
    for line in open(path):
        name, _, js = line.partition(" ")
        if name == K and js.startswith("{"):
            return json.loads(js)
    raise SystemExit(f"{path}: no {K} line")


def times(path):
    out = {}
    for line in open(path):
        lib, _, rest = line.partition(": ")
        if rest.startswith("C2 "):
            out.setdefault(lib.strip(), []).append(float(rest.split()[1]))
    return {k: statistics.median(v) for k, v in out.items()}


def main():
    d, lds_json = sys.argv[1], sys.argv[2]
    base = load(f"{d}/lds_libfsehip.so.txt")
    st = load(f"{d}/lds_libfsehip_est.so.txt")
    tt = load(f"{d}/lds_libfsehip_ett.so.txt")
    steps = st["lds_instructions_per_launch"] - base["lds_instructions_per_launch"]
    c_st = (st["lds_array_cycles_per_launch"] - base["lds_array_cycles_per_launch"]) / steps
    c_tt = (tt["lds_array_cycles_per_launch"] - base["lds_array_cycles_per_launch"]) / steps
    k_st = (st["bank_conflict_cycles_per_launch"] - base["bank_conflict_cycles_per_launch"]) / steps
    k_tt = (tt["bank_conflict_cycles_per_launch"] - base["bank_conflict_cycles_per_launch"]) / steps
    gathers = 2.0 * steps * (c_st + c_tt)
    t = times(f"{d}/enc_split_time.txt")
    split = {"unit": "LDS-array cycles per wave gather instruction",
             "stateTable_gather": round(c_st, 2), "stateTable_gather_conflicts": round(k_st, 2),
             "transform_gather": round(c_tt, 2), "transform_gather_conflicts": round(k_tt, 2),
             "wave_pair_steps_per_block": round(steps / BLOCKS, 1),
             "gather_share_of_lds_cycles": round(gathers / base["lds_array_cycles_per_launch"], 3),
             "ms_per_extra_gather_per_pair": {"stateTable": round(t["libfsehip_est.so"] - t["libfsehip.so"], 3),
                                              "transform": round(t["libfsehip_ett.so"] - t["libfsehip.so"], 3)},
             "source": "product vs FSEHIP_ENC_ABL=64 / 128 builds, one rocprofv3 SQ pass each, C2 encode medians "
                       "(tools/gpu_r05_v.sh, tools/gpu_r05_w.sh, tools/lds_split_enc.py)"}
    doc = json.load(open(lds_json))
    doc["kernels"][K]["split"] = split
    json.dump(doc, open(lds_json, "w"), indent=1)
    print(K, json.dumps(split))


if __name__ == "__main__":
    main()
