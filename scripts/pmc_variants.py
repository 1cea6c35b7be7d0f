"""Per-variant PMC summary of scripts/ab_variants.sh output: median per-dispatch counters of the marching kernel.
Usage: python3 scripts/pmc_variants.py <out_dir> <variant names...>"""
import collections
import csv
import os
import statistics
import sys


def summary(path, key="alex_march"):
    rows = [r for r in csv.DictReader(open(path)) if key in r["Kernel_Name"]]
    by = collections.defaultdict(dict)
    for r in rows:
        by[int(r["Dispatch_Id"])][r["Counter_Name"]] = float(r["Counter_Value"])
    sel = list(by.values())
    return {k: statistics.median(s[k] for s in sel) for k in sel[0]}, len(sel)


if __name__ == "__main__":
    out = sys.argv[1]
    for v in sys.argv[2:]:
        p = os.path.join(out, f"pmc_{v}")
        f = [os.path.join(dp, n) for dp, _, ns in os.walk(p) for n in ns if n.endswith("counter_collection.csv")][0]
        s, n = summary(f)
        busy = s.get("SQ_ACTIVE_INST_VALU", 0) * 4 / (1024 * s["GRBM_GUI_ACTIVE"] / 8) if "GRBM_GUI_ACTIVE" in s else None
        print(v, n, {k: round(x / 1e6, 2) for k, x in s.items()}, "valu_busy", round(busy, 3) if busy else None)
