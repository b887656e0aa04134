"""One line of the numbers that matter from a bench.py JSON line (stdin)."""
import json
import sys


def get(d, *path):
    for p in path:
        if not isinstance(d, dict) or p not in d:
            return None
        d = d[p]
    return d


line = sys.stdin.read().strip().splitlines()[-1]
d = json.loads(line)
fields = [("value", ("value",)), ("ms/step", ("ms_per_step",)), ("enc_ms", ("encode_ms",)), ("dec_ms", ("decode_ms",)),
          ("enc_frac", ("roofline", "frac")), ("c3_ms", ("c3_decode_only", "decode_ms")),
          ("c3_frac", ("c3_decode_only", "roofline", "frac")), ("nosc_GiB_s", ("sidecar_less_decode", "decode_GiB_s")),
          ("rank_fb", ("rank_check", "fallback_tables")), ("n_gpus", ("n_gpus",))]
print("  ".join(f"{k}={get(d, *p)}" for k, p in fields if get(d, *p) is not None))
