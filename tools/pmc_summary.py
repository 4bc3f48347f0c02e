"""Summarise rocprofv3 --pmc / --kernel-trace CSVs per kernel (average per dispatch).

Usage: python tools/pmc_summary.py gpurun_out/prof_TAG [--json out.json] [--panels S]

Reads every */run_counter_collection.csv under the directory (one pass per
counter group, tools/gpu_prof.sh) and trace/run_kernel_stats.csv.  Units:
SQ_* cycle counters are as reported (quad-cycles for SQ_WAVE_CYCLES /
SQ_BUSY_CYCLES / SQ_WAIT_* / SQ_ACTIVE_INST_*, per MI355X_MICROARCH.md);
FETCH_SIZE / WRITE_SIZE are KiB.  HBM bytes per launch follow the guide's
gfx950 correction: FETCH_SIZE reports half the bytes of wide streaming reads,
so fetch bytes are reported both raw and x2; WRITE_SIZE is taken as exact.
"""
import argparse
import csv
import glob
import json
import os
import re
from collections import defaultdict


def short(name):
    m = re.search(r"(draw_kernel<[^>]*>|pair_mfma_kernel|xt_count_kernel|unique_kernel|[A-Za-z0-9_]+kernel[^(]*)", name)
    return m.group(1) if m else name[:60]


def load(d):
    per = defaultdict(lambda: defaultdict(list))   # kernel -> counter -> [values per dispatch]
    for path in glob.glob(os.path.join(d, "*", "run_counter_collection.csv")):
        with open(path) as fh:
            for row in csv.DictReader(fh):
                per[short(row["Kernel_Name"])][row["Counter_Name"]].append(float(row["Counter_Value"]))
    stats = {}
    sp = os.path.join(d, "trace", "run_kernel_stats.csv")
    if os.path.exists(sp):
        with open(sp) as fh:
            for row in csv.DictReader(fh):
                stats[short(row["Name"])] = {"calls": int(row["Calls"]), "avg_ns": float(row["AverageNs"]),
                                             "pct": float(row["Percentage"])}
    return per, stats


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--json")
    ap.add_argument("--panels", type=int, default=10 ** 6)
    ap.add_argument("--config", default="sf_e_110")
    args = ap.parse_args()
    per, stats = load(args.dir)
    out = {"dir": args.dir, "panels_per_launch": args.panels, "kernels": {}}
    for k in sorted(set(per) | set(stats)):
        if k not in stats and not k.startswith(("draw", "pair", "xt", "unique")):
            continue
        c = {name: sum(v) / len(v) for name, v in per[k].items()}
        e = {"trace": stats.get(k), "counters": c}
        if "FETCH_SIZE" in c:
            e["fetch_bytes_raw"] = c["FETCH_SIZE"] * 1024
            e["fetch_bytes_x2"] = c["FETCH_SIZE"] * 2048
        if "WRITE_SIZE" in c:
            e["write_bytes"] = c["WRITE_SIZE"] * 1024
        if "SQ_INSTS_VALU" in c and k.startswith("draw"):
            e["valu_insts_per_panel"] = c["SQ_INSTS_VALU"] / args.panels
            e["lds_insts_per_panel"] = c.get("SQ_INSTS_LDS", 0) / args.panels
            e["salu_insts_per_panel"] = c.get("SQ_INSTS_SALU", 0) / args.panels
        if "SQ_BUSY_CYCLES" in c and "SQ_ACTIVE_INST_VALU" in c and "SQ_WAVE_CYCLES" in c:
            e["valu_active_per_wave_cycle"] = c["SQ_ACTIVE_INST_VALU"] / max(c["SQ_WAVE_CYCLES"], 1)
        out["kernels"][k] = e
    s = json.dumps(out, indent=1)
    print(s)
    if args.json:
        with open(args.json, "w") as fh:
            fh.write(s + "\n")


if __name__ == "__main__":
    main()
