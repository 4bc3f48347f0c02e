"""Generate golden vectors by driving the UNMODIFIED reference in Philox mode.

Runs only where /root/reference exists (this dev container).  Nothing from the
reference is copied: it is imported from /root/reference at run time, its RNG
is monkeypatched (no source edits), and only its OUTPUTS are written, as small
JSON fixtures under tests/golden/.  The GPU box never runs this script.

Philox verification mode (stream defined in
oracle/philox.py):
  * wrap analysis.legacy_find               -> panel += 1, attempt = -1
                                               (also records pick order)
  * wrap analysis.find_random_sample_legacy -> attempt += 1, step = 0
  * wrap legacy.find_max_ratio_cat          -> word = philox(seed, panel,
                                               attempt, step); step += 1
  * random.randint (as seen by legacy.py)   -> 1 + ((word * b) >> 32)
Because ``randint(1, b)`` becomes a pure function of ``b`` within one step,
repeated calls at every argmax improvement (legacy.py:149) are harmless: the
last one, made with the argmax's ``remaining``, is the one the reference uses.

Also writes MT-mode goldens: the reference's PUBLISHED seed-0 LEGACY selection
probabilities (reference_output/ and analysis/ *_ratio_product_data.csv) and
the seed-1 statistics pins from analysis/*_statistics.txt.

Usage:  python tools/make_goldens.py [case ...]
"""
import csv
import hashlib
import json
import os
import sys
import time
import types

import numpy as np

REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.normpath(os.path.join(HERE, ".."))
GOLD = os.path.join(REPO, "tests", "golden")
INST = os.path.join(GOLD, "instances")
sys.path.insert(0, REPO)

from oracle.philox import legacy_word, legacy_randint  # noqa: E402

# (case name, instance dir, k, S, seed)
CASES = [
    ("couples_s0", "couples_panel_from_twenty_people_no_constraints_2", 2, 10000, 0),
    ("couples_s1", "couples_panel_from_twenty_people_no_constraints_2", 2, 10000, 1),
    ("example_small_20_s0", "example_small_20", 20, 10000, 0),
    ("example_large_200_s0", "example_large_200", 200, 1000, 0),
    ("sf_e_110_s0", "sf_e_110", 110, 200, 0),
    ("sf_e_tight_110_s1", "sf_e_tight_110", 110, 200, 1),
    ("pathological_5_s0", "pathological_5", 5, 2000, 0),
    ("rejecty_6_s3", "rejecty_6", 6, 2000, 3),
    ("synthetic8192_200_s0", "synthetic8192_200", 200, 200, 0),
]


def import_reference():
    """Import legacy.py / analysis.py unmodified; stub modules the LEGACY path never uses."""
    if REF not in sys.path:
        sys.path.insert(0, REF)
    for name, attrs in (("seaborn", {}), ("leximin", {"find_distribution_leximin": None}),
                        ("xmin", {"find_distribution_xmin": None})):
        if name not in sys.modules:
            mod = types.ModuleType(name)
            for a, v in attrs.items():
                setattr(mod, a, v)
            sys.modules[name] = mod
    import matplotlib
    matplotlib.use("Agg")
    import legacy  # noqa: F401
    import analysis
    return sys.modules["legacy"], analysis


class PhiloxHarness:
    def __init__(self, legacy, analysis, seed):
        self.legacy, self.analysis, self.seed = legacy, analysis, seed
        self.panel, self.attempt, self.step, self.word = -1, -1, 0, None
        self.attempts, self.picks = [], []
        self.selection_errors = []     # per panel: attempts that raised SelectionError (legacy.py:34-36)

    def __enter__(self):
        lg, an = self.legacy, self.analysis
        self.saved = (an.legacy_find, an.find_random_sample_legacy, lg.find_max_ratio_cat,
                      lg.random.randint)
        orig_find, orig_draw, orig_ratio, _ = self.saved
        h = self

        def legacy_find(*a, **kw):
            h.panel += 1
            h.attempt = -1
            h.selection_errors.append(0)
            out = orig_find(*a, **kw)
            h.attempts.append(h.attempt + 1)
            h.picks.append(list(out))
            return out

        def find_random_sample_legacy(*a, **kw):
            h.attempt += 1
            h.step = 0
            try:
                return orig_draw(*a, **kw)
            except lg.SelectionError:
                h.selection_errors[-1] += 1   # analysis.py:152-153 restarts; the rest are rejections
                raise

        def find_max_ratio_cat(*a, **kw):
            h.word = legacy_word(h.seed, h.panel, h.attempt, h.step)
            h.step += 1
            return orig_ratio(*a, **kw)

        an.legacy_find = legacy_find
        an.find_random_sample_legacy = find_random_sample_legacy
        lg.find_max_ratio_cat = find_max_ratio_cat
        lg.random.randint = lambda a, b: legacy_randint(h.word, b)
        return self

    def __exit__(self, *exc):
        lg, an = self.legacy, self.analysis
        (an.legacy_find, an.find_random_sample_legacy, lg.find_max_ratio_cat,
         lg.random.randint) = self.saved
        return False


def pack(panels, n):
    W = (n + 63) // 64
    out = np.zeros((len(panels), W), np.uint64)
    for i, panel in enumerate(panels):
        for p in panel:
            out[i, p >> 6] |= np.uint64(1) << np.uint64(p & 63)
    return out


def sha(arr):
    return hashlib.sha256(np.ascontiguousarray(arr).tobytes()).hexdigest()


def run_case(legacy, analysis, case, inst_dir, k, S, seed):
    d = os.path.join(INST, inst_dir)
    inst = analysis.read_instance(os.path.join(d, "categories.csv"), os.path.join(d, "respondents.csv"), k)
    n = len(inst.agents)
    t0 = time.time()
    with PhiloxHarness(legacy, analysis, seed) as h:
        alloc, found, hist = analysis.legacy_probabilities(inst, S, seed)
    dt = time.time() - t0
    panels = [tuple(sorted(p)) for p in h.picks]
    counts = np.zeros(n, np.int64)
    for p in panels:
        counts[list(p)] += 1
    X = np.zeros((S, n), np.float64)
    for i, p in enumerate(panels):
        X[i, list(p)] = 1.0
    pairs = np.rint(X.T @ X).astype(np.int64)
    iu = np.triu_indices(n, 1)
    upper = pairs[iu]
    ref_pair_probs = np.fromiter(hist.get_dict().values(), np.float64, count=n * (n - 1) // 2)
    # cross-checks of the captured panels against the reference's own outputs
    assert all(alloc[i] == counts[i] / S for i in range(n)), "alloc mismatch"
    assert len(found) == len(set(panels)), "unique mismatch"
    assert np.array_equal(ref_pair_probs, upper / S), "pair histogram mismatch"
    g = {
        "case": case, "instance": inst_dir, "k": k, "S": S, "seed": seed, "n": n,
        "rng": "philox4x32-10 verification mode (oracle/philox.py)",
        "generator": "tools/make_goldens.py driving the unmodified reference",
        "reference_seconds": round(dt, 3),
        "counts": counts.tolist(),
        "unique": len(found),
        "attempts": h.attempts,
        # attempts - 1 = SelectionError restarts (analysis.py:152-153) + min-quota rejections
        # (the "Rejected" prints, analysis.py:155-159), split per panel
        "selection_errors": h.selection_errors,
        "rejections": [a - 1 - e for a, e in zip(h.attempts, h.selection_errors)],
        "panels_sha256": sha(pack(panels, n)),
        "pair_upper_sha256": sha(upper.astype(np.int64)),
        "pair_upper_sum": int(upper.sum()),
        "pair_prob_sha256": sha(ref_pair_probs),
        "first_panels": [list(p) for p in panels[:256]],
        "first_picks": h.picks[:64],
    }
    if n <= 200:
        g["pair_upper"] = upper.tolist()
        g["alloc"] = [alloc[i] for i in range(n)]
    return g


# check_same_address cases (legacy.py:78-99, 103-113): the reference harness never sets the flag
# (analysis.py:150-151), so these drive find_random_sample_legacy directly in a legacy_find-shaped
# restart loop (deepcopy, SelectionError -> next attempt, check_min_cats -> next attempt), with an
# address column committed next to the instance.  (case, instance dir, k, S, seed)
ADDRESS_CASES = [
    ("address_example_small_20_s2", "example_small_20", 20, 2000, 2),
    ("address_sf_e_tight_110_s1", "sf_e_tight_110", 110, 150, 1),
]
ADDR_COLS = ["primary_address1", "primary_zip"]


def write_addresses(inst_dir, n, seed=0):
    """Synthetic households: sizes 1-4 (40/30/20/10 %), members in shuffled agent order; the street
    part repeats across zip codes, so equal address1 alone is not the same address."""
    path = os.path.join(INST, inst_dir, "addresses.csv")
    if os.path.exists(path):
        return path
    rng = np.random.default_rng(seed)
    order = rng.permutation(n)
    rows = [None] * n
    h = i = 0
    while i < n:
        size = int(rng.choice([1, 2, 3, 4], p=[0.4, 0.3, 0.2, 0.1]))
        street = "%d Main St" % (h % max(4, n // 16))
        zipc = "Z%03d" % (h % 37)
        for p in order[i:i + size]:
            rows[p] = (street, zipc)
        i += size
        h += 1
    with open(path, "w", newline="", encoding="utf-8") as fh:
        w = csv.writer(fh)
        w.writerow(ADDR_COLS)
        w.writerows(rows)
    return path


def read_addresses(path):
    with open(path, encoding="utf-8") as fh:
        return {i: dict(r) for i, r in enumerate(csv.DictReader(fh))}


def address_case(legacy, analysis, case, inst_dir, k, S, seed, mode):
    import copy
    import random
    d = os.path.join(INST, inst_dir)
    inst = analysis.read_instance(os.path.join(d, "categories.csv"), os.path.join(d, "respondents.csv"), k)
    n = len(inst.agents)
    columns_data = read_addresses(write_addresses(inst_dir, n))
    picks, attempts, single = [], [], []
    harness = PhiloxHarness(legacy, analysis, seed) if mode == "philox" else None
    if harness:
        harness.__enter__()
    else:
        random.seed(seed)
    t0 = time.time()
    try:
        for i in range(S):
            a = -1
            while True:
                a += 1
                cats, people = copy.deepcopy(inst.categories), copy.deepcopy(inst.agents)
                if harness:
                    harness.panel, harness.attempt, harness.step = i, a, 0
                rec = {"panel": i, "attempt": a}
                try:
                    sel, lines = legacy.find_random_sample_legacy(cats, people, columns_data, k, True, ADDR_COLS)
                except legacy.SelectionError:
                    if len(single) < 40:
                        single.append(dict(rec, status="SelectionError"))
                    continue
                ok, _ = legacy.check_min_cats(cats)
                if len(single) < 40:
                    single.append(dict(rec, status="ok", picks=list(sel), lines=lines,
                                       selected=[[c, f, v["selected"], v["remaining"]] for c in cats
                                                 for f, v in cats[c].items()],
                                       people_left=sorted(people)))
                if not ok:
                    continue
                picks.append(list(sel))
                attempts.append(a + 1)
                break
    finally:
        if harness:
            harness.__exit__(None, None, None)
    panels = [tuple(sorted(p)) for p in picks]
    counts = np.zeros(n, np.int64)
    for p in panels:
        counts[list(p)] += 1
    return {"case": case, "instance": inst_dir, "k": k, "S": S, "seed": seed, "n": n, "rng": mode,
            "columns": ADDR_COLS, "addresses": "tests/golden/instances/%s/addresses.csv" % inst_dir,
            "generator": "tools/make_goldens.py driving the unmodified reference's find_random_sample_legacy "
                         "with check_same_address=True in a legacy_find-shaped restart loop",
            "reference_seconds": round(time.time() - t0, 3), "counts": counts.tolist(),
            "unique": len(set(panels)), "attempts": attempts, "panels_sha256": sha(pack(panels, n)),
            "picks": picks if S * k <= 50000 else picks[:200], "single_attempts": single}


def mt_goldens():
    out = {}
    for name, k, rel in (
        ("couples_panel_from_twenty_people_no_constraints", 2,
         "analysis/couples_panel_from_twenty_people_no_constraints_2_ratio_product_data.csv"),
        ("example_small", 20, "reference_output/example_small_20_ratio_product_data.csv"),
        ("example_small", 20, "analysis/example_small_20_ratio_product_data.csv"),
        ("example_large", 200, "reference_output/example_large_200_ratio_product_data.csv"),
    ):
        with open(os.path.join(REF, rel), encoding="utf-8") as fh:
            probs = [float(r["selection probability"]) for r in csv.DictReader(fh)]
        out[rel] = {"instance": "%s_%d" % (name, k), "k": k, "S": 10000, "seed": 0,
                    "selection_probability": probs}
    # seed-1 statistics pins (analysis/*_statistics.txt)
    out["statistics_seed1"] = {
        "couples_panel_from_twenty_people_no_constraints_2": {"unique": 100, "minimizer_prop": "0.1020"},
        "example_small_20": {"unique": 10000, "minimizer_prop": "0.0096"},
    }
    return out


def main(argv):
    if not os.path.isdir(REF):
        sys.exit("reference not present; goldens are committed under tests/golden/")
    legacy, analysis = import_reference()
    want = set(argv)
    for case, inst_dir, k, S, seed in CASES:
        if want and case not in want:
            continue
        g = run_case(legacy, analysis, case, inst_dir, k, S, seed)
        path = os.path.join(GOLD, "philox_%s.json" % case)
        with open(path, "w") as fh:
            json.dump(g, fh, separators=(",", ":"))
        print("%-24s n=%-5d S=%-6d unique=%-6d attempts=%d  %.1fs" % (
            case, g["n"], S, g["unique"], sum(g["attempts"]), g["reference_seconds"]), file=sys.stderr)
    if not want or "mt" in want:
        with open(os.path.join(GOLD, "mt_published.json"), "w") as fh:
            json.dump(mt_goldens(), fh, separators=(",", ":"))
    for case, inst_dir, k, S, seed in ADDRESS_CASES:
        if want and case not in want and "address" not in want:
            continue
        g = {mode: address_case(legacy, analysis, case, inst_dir, k, S, seed, mode) for mode in ("philox", "mt")}
        with open(os.path.join(GOLD, "%s.json" % case), "w") as fh:
            json.dump(g, fh, separators=(",", ":"))
        print("%-28s philox unique=%d attempts=%d  mt unique=%d attempts=%d" % (
            case, g["philox"]["unique"], sum(g["philox"]["attempts"]), g["mt"]["unique"],
            sum(g["mt"]["attempts"])), file=sys.stderr)


if __name__ == "__main__":
    main(sys.argv[1:])
