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
    ("synthetic8192_200_s0", "synthetic8192_200", 200, 6, 0),
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

    def __enter__(self):
        lg, an = self.legacy, self.analysis
        self.saved = (an.legacy_find, an.find_random_sample_legacy, lg.find_max_ratio_cat,
                      lg.random.randint)
        orig_find, orig_draw, orig_ratio, _ = self.saved
        h = self

        def legacy_find(*a, **kw):
            h.panel += 1
            h.attempt = -1
            out = orig_find(*a, **kw)
            h.attempts.append(h.attempt + 1)
            h.picks.append(list(out))
            return out

        def find_random_sample_legacy(*a, **kw):
            h.attempt += 1
            h.step = 0
            return orig_draw(*a, **kw)

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


if __name__ == "__main__":
    main(sys.argv[1:])
