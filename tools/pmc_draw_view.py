"""Print the draw kernel's SQ counters per panel from tools/gpu_pmc_draw.sh output dirs."""
import json
import subprocess
import sys

for d in sys.argv[1:]:
    out = subprocess.run([sys.executable, "tools/pmc_summary.py", d], capture_output=True, text=True).stdout
    data = json.loads(out)
    for k, v in data["kernels"].items():
        if "draw" not in k:
            continue
        c = v["counters"]
        ns = v["trace"]["avg_ns"] if v.get("trace") else 0
        clk = c.get("GRBM_GUI_ACTIVE", 0) / 8 / (ns * 1e-9) / 1e9 if ns else 0
        valu = c.get("SQ_INSTS_VALU", 0)
        util = valu * 2 / (1024 * c.get("GRBM_GUI_ACTIVE", 1) / 8)
        wc = max(c.get("SQ_WAVE_CYCLES", 1), 1)
        print("%s  %s  %.3f ms  clk %.2f GHz  VALU/panel %.0f  SALU/panel %.0f  LDS/panel %.0f  VALU util %.2f  "
              "waves %d  active %.2f  wait_inst %.2f  wait_any %.2f  lds_conf/active %.2f" % (
                  d, k, ns / 1e6, clk, valu / 1e6, c.get("SQ_INSTS_SALU", 0) / 1e6, c.get("SQ_INSTS_LDS", 0) / 1e6,
                  util, c.get("SQ_WAVES", 0), c.get("SQ_ACTIVE_INST_ANY", 0) / wc,
                  c.get("SQ_WAIT_INST_ANY", 0) / wc, c.get("SQ_WAIT_ANY", 0) / wc,
                  c.get("SQ_LDS_BANK_CONFLICT", 0) / max(c.get("SQ_ACTIVE_INST_LDS", 1), 1)))
