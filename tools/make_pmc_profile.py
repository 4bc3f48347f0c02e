"""Build profiles/pmc_<config>.json (read by bench.py) from a tools/gpu_prof.sh output directory.

    python tools/make_pmc_profile.py gpurun_out/prof_TAG --config sf_e_110 --panels 1000000 \
        --source "profiles/r01_..." [--out profiles/pmc_sf_e_110.json]

HBM bytes per launch follow MI355X_MICROARCH.md's HBM section: FETCH_SIZE is doubled (gfx950 tallies
wide streaming reads at half their bytes), WRITE_SIZE is taken as exact.  The VALU issue fraction of
the draw kernel = SQ_INSTS_VALU x 2 cycles (wave64 on a SIMD-32) / (1024 SIMDs x GRBM_GUI_ACTIVE / 8
XCDs), the fraction of the chip's VALU issue slots the kernel used.
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import pmc_summary  # noqa: E402

SIMDS = 1024


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--config", default="sf_e_110")
    ap.add_argument("--panels", type=int, default=10 ** 6)
    ap.add_argument("--source", default="")
    ap.add_argument("--out")
    args = ap.parse_args()
    per, stats = pmc_summary.load(args.dir)
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench  # noqa: E402  (source_sha: the kernel sources these counters belong to)
    out = {"config": args.config, "panels": args.panels, "source_sha": bench.source_sha(),
           "source": args.source or args.dir,
           "method": "rocprofv3 --pmc passes, one counter group per run (tools/gpu_prof.sh); FETCH_SIZE x2 "
                     "per MI355X_MICROARCH.md HBM section; WRITE_SIZE exact",
           "per_kernel": {}}
    draw_name = None
    for k in sorted(set(per) | set(stats)):
        c = {name: sum(v) / len(v) for name, v in per[k].items()}
        if not c and k not in stats:
            continue
        e = {"avg_ns": (stats.get(k) or {}).get("avg_ns")}
        if "FETCH_SIZE" in c:
            e["fetch_bytes_x2"] = c["FETCH_SIZE"] * 2048
        if "WRITE_SIZE" in c:
            e["write_bytes"] = c["WRITE_SIZE"] * 1024
        if "fetch_bytes_x2" in e and "write_bytes" in e:
            e["hbm_bytes_per_launch"] = e["fetch_bytes_x2"] + e["write_bytes"]
            if e.get("avg_ns"):
                e["hbm_GBps"] = e["hbm_bytes_per_launch"] / e["avg_ns"]
        if c.get("SQ_VALU_MFMA_BUSY_CYCLES") and c.get("GRBM_GUI_ACTIVE"):
            # MFMA pipe busy cycles summed over the SIMDs / (1024 SIMDs x the kernel's cycles)
            e["mfma_busy_frac"] = c["SQ_VALU_MFMA_BUSY_CYCLES"] / (SIMDS * c["GRBM_GUI_ACTIVE"] / 8)
        if k.startswith("draw") and "SQ_INSTS_VALU" in c:
            draw_name = k
            gui = c.get("GRBM_GUI_ACTIVE")
            ns = e["avg_ns"]
            issue = {"valu_insts_per_launch": c["SQ_INSTS_VALU"],
                     "valu_insts_per_panel": c["SQ_INSTS_VALU"] / args.panels,
                     "salu_insts_per_panel": c.get("SQ_INSTS_SALU", 0) / args.panels,
                     "lds_insts_per_panel": c.get("SQ_INSTS_LDS", 0) / args.panels}
            if gui:
                issue["valu_issue_frac"] = c["SQ_INSTS_VALU"] * 2 / (SIMDS * gui / 8)
                if ns:
                    issue["clock_GHz"] = gui / 8 / (ns * 1e-9) / 1e9
            if gui and c.get("SQ_ACTIVE_INST_VALU"):
                # SQ_ACTIVE_INST_VALU counts quad-cycles: the fraction of SIMD cycles with a VALU
                # instruction of this kernel in flight (~1 = the VALU pipe never idles)
                issue["valu_active_frac"] = c["SQ_ACTIVE_INST_VALU"] * 4 / (SIMDS * gui / 8)
            if c.get("SQ_ACTIVE_INST_LDS"):
                issue["lds_bank_conflict_per_active_lds"] = c.get("SQ_LDS_BANK_CONFLICT", 0) / c["SQ_ACTIVE_INST_LDS"]
            if c.get("SQ_WAVE_CYCLES"):
                issue["wait_inst_any_frac"] = c.get("SQ_WAIT_INST_ANY", 0) / c["SQ_WAVE_CYCLES"]
                issue["wait_any_frac"] = c.get("SQ_WAIT_ANY", 0) / c["SQ_WAVE_CYCLES"]
                issue["active_inst_any_frac"] = c.get("SQ_ACTIVE_INST_ANY", 0) / c["SQ_WAVE_CYCLES"]
                if gui:
                    # occupancy: resident wave-cycles (SQ_WAVE_CYCLES counts quad-cycles) per SIMD-cycle
                    issue["mean_waves_per_simd"] = 4 * c["SQ_WAVE_CYCLES"] / (SIMDS * gui / 8)
            issue["note"] = ("VALU issue fraction = SQ_INSTS_VALU x 2 cycles (wave64 on SIMD-32) / "
                             "(1024 SIMDs x GRBM_GUI_ACTIVE/8)")
            out["draw_issue"] = issue
        out["per_kernel"][k] = e
    if draw_name:
        out["kernel"] = draw_name
        out["draw_kernel"] = draw_name
        out["hbm_bytes_per_launch"] = out["per_kernel"][draw_name].get("hbm_bytes_per_launch")
    s = json.dumps(out, indent=1)
    print(s)
    if args.out:
        with open(args.out, "w") as fh:
            fh.write(s + "\n")


if __name__ == "__main__":
    main()
