#!/usr/bin/env python3
"""Summarise a scripts/profile.sh run into committed artefacts under profiles/.

    python scripts/pmc_summary.py gpurun_out/prof_<tag> <tag>

Writes profiles/<tag>_kernel_stats.csv (the rocprofv3 --stats summary, verbatim),
profiles/<tag>_summary.md (per-kernel averages of every collected counter) and updates
profiles/pmc_traffic.json, which bench.py reads for roofline.traffic / valu_busy — keyed by the kernel's template
instance and stamped with the sha of its sources (bench.py kernel_src_sha), so a later source change voids it.

HBM bytes follow MI355X_MICROARCH.md's gfx950 correction: FETCH_SIZE (KB) counts 16-B
coalesced reads at half their size (calibrated here on count_kernel: a 268 MB stream reads
as 134 MB), so bytes = 2 * FETCH_SIZE * 1024 + WRITE_SIZE * 1024.
"""
import csv
import glob
import json
import os
import re
import shutil
import sys
from collections import defaultdict

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench import kernel_src_sha  # noqa: E402  (the repo root's bench.py: the same hash it checks)

KERNELS = {"alex_step_kernel": "alex_step", "alex_march_kernel": "alex_march", "windy_fast_kernel": "windy_fast", "windy_exact_kernel": "windy_exact",
           "windy_rows_kernel": "windy_rows", "adv_obs_plain_kernel": "adv_obs_plain",
           "count_kernel": "count", "advenv_post_kernel": "advenv_post",
           "adv_observation_kernel": "adv_observation", "random_actions_kernel": "random_actions"}


def short(name):
    for k, v in KERNELS.items():
        if k in name:
            m = re.search(k + r"<([^>]*)>", name)
            return v + (f"<{m.group(1)}>" if m else "")
    return None


def timed_means(prof_dir, skip=20):
    """Per-kernel mean duration (us) over the launches after the first `skip` of each kernel (the bench's
    untimed warm-up steps), from the kernel trace of the same run."""
    path = os.path.join(prof_dir, "trace", "run_kernel_trace.csv")
    if not os.path.exists(path):
        return {}
    per = defaultdict(list)
    with open(path) as f:
        for row in csv.DictReader(f):
            s = short(row["Kernel_Name"])
            if s:
                per[s].append((int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) / 1e3)
    return {s: sum(v[skip:]) / len(v[skip:]) for s, v in per.items() if len(v) > skip}


def main(prof_dir, tag, out_dir="profiles"):
    os.makedirs(out_dir, exist_ok=True)
    stats = os.path.join(prof_dir, "trace", "run_kernel_stats.csv")
    dur = {}
    if os.path.exists(stats):
        shutil.copy(stats, os.path.join(out_dir, f"{tag}_kernel_stats.csv"))
        with open(stats) as f:
            for row in csv.DictReader(f):
                s = short(row["Name"])
                if s:
                    dur[s] = (int(row["Calls"]), float(row["AverageNs"]) / 1e3)
    vals = defaultdict(lambda: defaultdict(list))
    meta = {}
    for path in glob.glob(os.path.join(prof_dir, "pmc_*", "run_counter_collection.csv")):
        with open(path) as f:
            for row in csv.DictReader(f):
                s = short(row["Kernel_Name"])
                if not s:
                    continue
                vals[s][row["Counter_Name"]].append(float(row["Counter_Value"]))
                meta[s] = (int(row["Grid_Size"]), int(row["LDS_Block_Size"]), int(row["Scratch_Size"]),
                           int(row["VGPR_Count"]), int(row["SGPR_Count"]))
    lines = [f"# rocprofv3 summary — {tag}", "",
             "Source: `bash scripts/profile.sh " + tag + "` on one MI355X (bench.py workload; kernel trace + stats in one "
             "run, each PMC group in its own run). Durations from the --stats pass; counters are per-launch means.",
             "HBM bytes = 2*FETCH_SIZE + WRITE_SIZE (KB units, gfx950 half-counting of 16-B reads).", "",
             "`avg us (timed)` = mean over the launches after the 20 warm-up steps (kernel trace), the figure to compare",
             "with bench.py's kernel_ms; `avg us` = the --stats mean over all launches.", "",
             "| kernel | calls | avg us | avg us (timed) | grid | LDS | scratch | VGPR | SGPR |",
             "|---|---|---|---|---|---|---|---|---|"]
    tm = timed_means(prof_dir)
    for s in sorted(set(dur) | set(meta)):
        c, us = dur.get(s, (0, float("nan")))
        g, lds, scr, v, sg = meta.get(s, (0, 0, 0, 0, 0))
        lines.append(f"| {s} | {c} | {us:.1f} | {tm.get(s, float('nan')):.1f} | {g} | {lds} | {scr} | {v} | {sg} |")
    lines += ["", "| kernel | counter | mean per launch |", "|---|---|---|"]
    traffic = {}
    for s in sorted(vals):
        for cn in sorted(vals[s]):
            v = vals[s][cn]
            lines.append(f"| {s} | {cn} | {sum(v) / len(v):.6g} |")
        if "FETCH_SIZE" in vals[s] and "WRITE_SIZE" in vals[s]:
            fe = sum(vals[s]["FETCH_SIZE"]) / len(vals[s]["FETCH_SIZE"]) * 1024 * 2
            wr = sum(vals[s]["WRITE_SIZE"]) / len(vals[s]["WRITE_SIZE"]) * 1024
            traffic[s] = {"read_bytes": fe, "write_bytes": wr, "bytes_per_launch": fe + wr}
            lines.append(f"| {s} | HBM bytes (corrected) | {fe + wr:.6g} (read {fe:.4g}, write {wr:.4g}) |")
        if "SQ_ACTIVE_INST_VALU" in vals[s] and "GRBM_GUI_ACTIVE" in vals[s]:
            # SQ_ACTIVE_INST_VALU counts quad-cycles (a wave64 VALU op holds a 16-lane SIMD for 4 cycles);
            # GRBM_GUI_ACTIVE is summed over the 8 XCDs: VALU-busy share of the 1024 SIMDs over the launch
            va = sum(vals[s]["SQ_ACTIVE_INST_VALU"]) / len(vals[s]["SQ_ACTIVE_INST_VALU"])
            gr = sum(vals[s]["GRBM_GUI_ACTIVE"]) / len(vals[s]["GRBM_GUI_ACTIVE"])
            busy = va * 4 / (1024 * gr / 8)
            traffic.setdefault(s, {})["valu_busy"] = busy
        if "SQ_INSTS_VALU" in vals[s]:  # VALU instructions issued per launch (all waves)
            traffic.setdefault(s, {})["valu_insts"] = sum(vals[s]["SQ_INSTS_VALU"]) / len(vals[s]["SQ_INSTS_VALU"])
            lines.append(f"| {s} | VALU busy (SQ_ACTIVE_INST_VALU x 4 / (1024 SIMDs x GRBM_GUI_ACTIVE / 8)) | {busy:.3f} |")
    with open(os.path.join(out_dir, f"{tag}_summary.md"), "w") as f:
        f.write("\n".join(lines) + "\n")
    tj = os.path.join(out_dir, "pmc_traffic.json")
    cur = json.load(open(tj)) if os.path.exists(tj) else {}
    for s, t in traffic.items():
        # src_sha: the kernel's sources as profiled; bench.py reports these figures only for the same sources
        cur[s] = dict(t, tag=tag, avg_us=dur.get(s, (0, None))[1], timed_avg_us=tm.get(s), src_sha=kernel_src_sha(s))
    with open(tj, "w") as f:
        json.dump(cur, f, indent=1, sort_keys=True)
    print("\n".join(lines))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], *(sys.argv[3:4]))
