"""Static VALU mix of one kernel in a device .s file, priced with the measured issue table.

    hipcc --offload-arch=gfx950 -O3 -std=c++17 -S --cuda-device-only -o /tmp/csa.s csrc/csa_legacy.hip
    python tools/valu_mix.py /tmp/csa.s draw_lane_kernelILi32ELi28ELi14E [profiles/valu_enc_mi355x.jsonl]

Diagnostic only.  The issue table (profiles/valu_enc_mi355x.jsonl, 8 waves/SIMD) puts gfx950 VALU ops in two
classes: ~2.3 cycles per wave64 instruction (add/sub/and/or/xor/not/mov, lshrrev, mul_f32, with VGPR,
inline-constant or literal operands) and ~4.2 (an SGPR operand, lshlrev, bcnt, bfe, min/max, 3-source ops,
DPP, mul/mad, cndmask, cmp).  The static count weights every instruction once (no trip counts), so it says
which ops a kernel's code is made of, not how often each runs.
"""
import re
import sys
import collections

FULL = {"v_add_u32", "v_sub_u32", "v_subrev_u32", "v_and_b32", "v_or_b32", "v_xor_b32", "v_not_b32",
        "v_mov_b32", "v_lshrrev_b32", "v_mul_f32", "v_add_f32"}


def kernel_body(text, needle):
    m = re.search(r"^(_Z\w*%s\w*):" % re.escape(needle), text, re.M)
    if not m:
        raise SystemExit("kernel %s not found" % needle)
    end = text.find(".Lfunc_end", m.end())
    return text[m.end():end]


def classify(line):
    parts = line.split(None, 1)
    op = parts[0]
    if not op.startswith("v_") or op.startswith(("v_readlane", "v_readfirstlane", "v_writelane")):
        return None, None
    base = re.sub(r"_(e32|e64|dpp|sdwa)$", "", op)
    args = parts[1] if len(parts) > 1 else ""
    srcs = [a.strip() for a in args.split(",")[1:]]
    sgpr = any(re.match(r"^-?(s\[|s\d|vcc|exec|m0|ttmp)", a) for a in srcs)
    if "_dpp" in op or "row_" in args or "quad_perm" in args:
        cls = "half"
    elif base in FULL and not sgpr:
        cls = "full"
    else:
        cls = "half"
    return base + ("(sgpr)" if sgpr else "") + ("(dpp)" if "_dpp" in op or "row_" in args else ""), cls


def main():
    text = open(sys.argv[1]).read()
    body = kernel_body(text, sys.argv[2])
    hist = collections.Counter()
    cls_n = collections.Counter()
    for raw in body.splitlines():
        line = raw.split(";")[0].strip()
        if not line or line.startswith((".", "_")) or line.endswith(":"):
            continue
        name, cls = classify(line)
        if name is None:
            continue
        hist[name] += 1
        cls_n[cls] += 1
    tot = sum(cls_n.values())
    cyc = 2.35 * cls_n["full"] + 4.2 * cls_n["half"]
    print("static VALU %d: full-rate %d, half-rate %d, priced %.0f cycles (%.2f per instruction)"
          % (tot, cls_n["full"], cls_n["half"], cyc, cyc / max(tot, 1)))
    for k, v in hist.most_common(40):
        print("%6d  %s" % (v, k))


if __name__ == "__main__":
    main()
