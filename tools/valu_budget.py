"""Class-weighted VALU budget of draw_lane_kernel: the dynamic VALU mix per class
and what it should cost, against the measured kernel time.

    hipcc --offload-arch=gfx950 -O3 -std=c++17 -S --cuda-device-only -DCSA_LANE_STAMPS \\
        -o /tmp/csa_stamps.s citizensassemblies-replication_amd/csrc/csa_legacy.hip
    python tools/valu_budget.py /tmp/csa_stamps.s profiles/r04_valu_budget/lane_stamps_sf_e_110.json \\
        [--pmc profiles/pmc_sf_e_110.json] [--kernel draw_lane_kernelILi32ELi28ELi14E]

The CSA_LANE_STAMPS build marks the regions of the step loop with asm comments (";@region NAME") and
counts, per wave, how often each region runs (tools/lane_stamps.py on the GPU box: a region counts
when any lane of the wave enters it, which is when its VALU issue).  This script walks the kernel's
ISA in layout order, attributes every VALU instruction to the region whose marker precedes it, splits
it into the two issue classes measured by tools/coissue.hip / tools/valu_rate.hip (valu_mix.classify:
"full" = two-operand add/and/or/xor/mov/lshr with VGPR or constant operands -- two waves' such
instructions run at once on a SIMD; "half" = everything else, one per ~4.2 cycles per SIMD) and
multiplies by the region's runs per wave.  Rare paths laid out inside a region are counted as if they
ran with it (an overestimate of a few instructions per step).  Diagnostic only.
"""
import argparse
import collections
import json
import re
import sys
import os

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from valu_mix import classify, kernel_body  # noqa: E402

# region -> execution counter of tools/lane_stamps.py ("once" = once per wave)
RUNS = {"prologue": "once", "loop": "loop", "philox": "philox", "step": "step", "pick": "pick", "update": "pick",
        "store": "store", "cascade": "loop", "round": "round", "pass2": "pass2", "pass1": "pass1", "book": "loop",
        "nocand": "nocand", "kcheck": "kcheck", "ending": "ending", "tail": "once"}
# SIMD cycles per wave64 instruction (tools/coissue.hip, profiles/r04_valu_budget/coissue.jsonl: four waves
# per SIMD of one op: v_xor 2.47, v_bfi / v_bcnt 4.35, v_mul_i32_i24 / v_lshlrev / v_add with an SGPR
# operand 4.2; one wave alone issues at most one VALU per ~5 cycles)
COST = {"full": 2.47, "half": 4.3}
QUAD = 4.0   # SQ_ACTIVE_INST_VALU counts one quad-cycle per VALU instruction of a wave (coissue calibration)


def regions(text, needle):
    """Static VALU per region in layout order.  The compiler sinks the pick's every-step work (pick-list
    accumulation, key / slack decrements, pool drop) below the conditional pick-list store, so inside the
    "store" region only the instructions under the store's exec mask (s_and_saveexec ... s_or_b64 exec)
    count as "store"; the rest of that region runs with every pick ("update")."""
    body = kernel_body(text, needle)
    cur = "prologue"
    per = collections.defaultdict(collections.Counter)
    ops = collections.defaultdict(collections.Counter)
    seen_loop = False
    in_store = None          # the saved-exec SGPRs of the store branch while inside it
    for raw in body.splitlines():
        m = re.search(r";@region (\w+)", raw)
        if m:
            cur = m.group(1)
            seen_loop = True
            in_store = None
            continue
        line = raw.split(";")[0].strip()
        if not line or line.startswith((".", "_")) or line.endswith(":"):
            continue
        reg = cur if seen_loop else "prologue"
        if cur == "store":
            ms = re.match(r"s_and_saveexec_b64 (s\[\d+:\d+\]), vcc", line)
            if ms and in_store is None:
                in_store = ms.group(1)
            elif in_store and line.startswith("s_or_b64 exec, exec, " + in_store):
                in_store = ""            # past the store's join: the rest runs with every pick
            reg = "store" if in_store else "update"
        name, cls = classify(line)
        if name is None:
            continue
        # code laid out after the last marker that closes the loop (the fused pack / exit) is the tail
        per[reg][cls] += 1
        ops[reg][name] += 1
    return per, ops


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("asm")
    ap.add_argument("stamps", help="tools/lane_stamps.py JSON (region_runs_per_wave, ms, panels, waves)")
    ap.add_argument("--pmc", help="profiles/pmc_<config>.json (draw_issue: VALU per panel, clock)")
    ap.add_argument("--kernel", default="draw_lane_kernelILi32ELi28ELi14ELb1E")
    ap.add_argument("--panels-per-wave", type=int, default=32)
    ap.add_argument("--out")
    args = ap.parse_args()
    per, ops = regions(open(args.asm).read(), args.kernel)
    st = json.load(open(args.stamps))
    runs = dict(st["region_runs_per_wave"], once=1.0)
    ppw = args.panels_per_wave
    rows, dyn = [], collections.Counter()
    for reg in sorted(per, key=lambda r: list(RUNS).index(r) if r in RUNS else 99):
        r = runs.get(RUNS.get(reg, "once"), 1.0)
        d = {c: per[reg][c] * r / ppw for c in ("full", "half")}
        dyn.update(d)
        rows.append({"region": reg, "static_full": per[reg]["full"], "static_half": per[reg]["half"],
                     "runs_per_wave": r, "valu_per_panel_full": d["full"], "valu_per_panel_half": d["half"],
                     "top_ops": ops[reg].most_common(6)})
    tot = dyn["full"] + dyn["half"]
    out = {"kernel": args.kernel, "regions": rows, "valu_per_panel": {"full": dyn["full"], "half": dyn["half"],
                                                                      "total": tot, "half_frac": dyn["half"] / tot},
           "cost_cycles": COST}
    prof = json.load(open(args.pmc)) if args.pmc else None
    pmc = prof["draw_issue"] if prof else None
    if pmc:
        meas_valu = pmc["valu_insts_per_panel"]
        clk = pmc["clock_GHz"] * 1e9
        ns = prof["per_kernel"][prof["draw_kernel"]]["avg_ns"]
        out["pmc_valu_per_panel"] = meas_valu
        out["model_vs_pmc"] = tot / meas_valu
        # per-panel SIMD cycles: the kernel's time x clock x 1024 SIMDs / panels
        panels = st["panels"]
        ms = (ns or 0) * 1e-6 or st["ms"]
        simd_cyc = ms * 1e-3 * clk * 1024 / panels
        scale = meas_valu / tot        # the measured count, split in the model's proportions
        budget_class = (dyn["full"] * COST["full"] + dyn["half"] * COST["half"]) * scale
        out.update({"measured_ms": ms, "clock_GHz": clk / 1e9, "simd_cycles_per_panel": simd_cyc,
                    "budget_single_issue_cycles_per_panel": meas_valu * QUAD,
                    "budget_class_weighted_cycles_per_panel": budget_class,
                    "frac_of_single_issue_budget": meas_valu * QUAD / simd_cyc,
                    "frac_of_class_weighted_budget": budget_class / simd_cyc})
    s = json.dumps(out, indent=1)
    print(s)
    if args.out:
        with open(args.out, "w") as fh:
            fh.write(s + "\n")


if __name__ == "__main__":
    main()
