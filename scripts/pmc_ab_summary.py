"""Per-build PMC summary of scripts/gpu_march_ab.sh output (median per dispatch of the marching kernel): HBM bytes per
cell (2 x FETCH_SIZE + WRITE_SIZE, KB units, the gfx950 correction of scripts/pmc_summary.py), VALU instructions,
VALU busy, wave cycles. Usage: python3 scripts/pmc_ab_summary.py gpurun_out/<tag> main <variants...> [--cells N]"""
import collections
import csv
import glob
import statistics
import sys


def summary(out, v, key="alex_march"):
    res = {}
    for f in glob.glob(f"{out}/pmc_{v}/*/run_counter_collection.csv"):
        by = collections.defaultdict(lambda: collections.defaultdict(float))
        for r in csv.DictReader(open(f)):
            if key in r["Kernel_Name"]:
                by[int(r["Dispatch_Id"])][r["Counter_Name"]] += float(r["Counter_Value"])
        for k in next(iter(by.values())):
            res[k] = statistics.median(d[k] for d in by.values())
    return res


if __name__ == "__main__":
    args = sys.argv[1:]
    cells = 268435456
    if "--cells" in args:
        i = args.index("--cells")
        cells = int(args[i + 1])
        del args[i:i + 2]
    out, names = args[0], args[1:]
    for v in names:
        s = summary(out, v)
        fe, wr = s.get("FETCH_SIZE", 0) * 2048, s.get("WRITE_SIZE", 0) * 1024
        busy = s["SQ_ACTIVE_INST_VALU"] * 4 / (1024 * s["GRBM_GUI_ACTIVE"] / 8)
        print(f"{v}: {(fe + wr) / cells:.2f} B/cell (read {fe / cells:.2f}, write {wr / cells:.2f}), "
              f"VALU {s['SQ_INSTS_VALU'] / 1e6:.1f}M, busy {busy:.3f}, wave cycles {s['SQ_WAVE_CYCLES'] / 1e6:.1f}M, "
              f"GRBM_GUI_ACTIVE {s['GRBM_GUI_ACTIVE'] / 1e6:.2f}M")
