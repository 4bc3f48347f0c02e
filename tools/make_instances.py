"""Generate the synthetic benchmark / parity instances.

Writes ``tests/golden/instances/<name>_<k>/{categories,respondents}.csv``.
The public reference instances (couples, example_small_20, example_large_200)
are copied verbatim as input fixtures when /root/reference is present.

Instances generated here (numpy ``default_rng(0)``):

* ``sf_e_110``  -- shape of the withheld sf_e_110 pool (n=1727, k=110, C=7,
  F=31).  Feature layout a:3 b:4 c:12 d:3 e:5 f:2 g:2 and population marginals
  from the reference's data/sf_e_110/intersections.csv (category pairs (a,b),
  (c,a), (a,d), (a,e), (a,f), (g,a)); each share floored at 0.002 and
  renormalised.  Pool: per category a..g, tilt p*exp(N(0,0.3)), renormalise,
  draw n features i.i.d.  Quotas min=floor(0.9 k p), max=ceil(1.1 k p).
* ``sf_e_tight_110`` -- the same pool with min=floor(k p), max=ceil(k p)
  (restart-heavy: exercises SelectionError / rejection paths).
* ``synthetic8192_200`` -- n=8192, C=10, category j has 2+(j mod 5) features
  (F=40), shares ~ Dirichlet(2), features i.i.d., quotas floor(0.9kp)/ceil(1.1kp).
* ``pathological_5`` / ``rejecty_6`` -- tiny restart- / rejection-heavy instances.

The sf_e marginals are cached in ``tests/golden/instances/sf_e_marginals.json``
so the generator also runs where /root/reference is absent.
"""
import csv
import json
import math
import os
import shutil
import sys
from collections import defaultdict

import numpy as np

REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))
OUT = os.path.join(HERE, "..", "tests", "golden", "instances")

SFE_LAYOUT = [("a", 3), ("b", 4), ("c", 12), ("d", 3), ("e", 5), ("f", 2), ("g", 2)]
SFE_PAIRS = {"a": ("a", "b"), "b": ("a", "b"), "c": ("c", "a"), "d": ("a", "d"),
             "e": ("a", "e"), "f": ("a", "f"), "g": ("g", "a")}


def sfe_marginals():
    cache = os.path.join(OUT, "sf_e_marginals.json")
    path = os.path.join(REF, "data", "sf_e_110", "intersections.csv")
    if not os.path.exists(path):
        with open(cache) as fh:
            return json.load(fh)
    marg = defaultdict(float)
    with open(path, encoding="utf-8") as fh:
        for row in csv.DictReader(fh):
            c1, f1, c2, f2 = row["category 1"], row["feature 1"], row["category 2"], row["feature 2"]
            share = float(row["population share"])
            for cat, feat in ((c1, f1), (c2, f2)):
                if SFE_PAIRS[cat] == (c1, c2):
                    marg[(cat, feat)] += share
    out = {}
    for cat, nf in SFE_LAYOUT:
        feats = ["%s%d" % (cat, i + 1) for i in range(nf)]
        p = np.array([max(marg[(cat, f)], 0.002) for f in feats])
        p = p / p.sum()
        out[cat] = {f: float(x) for f, x in zip(feats, p)}
    with open(cache, "w") as fh:
        json.dump(out, fh, indent=1)
    return out


def write_instance(name, k, cats, people, cat_order):
    d = os.path.join(OUT, "%s_%d" % (name, k))
    os.makedirs(d, exist_ok=True)
    with open(os.path.join(d, "categories.csv"), "w", newline="", encoding="utf-8") as fh:
        w = csv.writer(fh)
        w.writerow(["category", "feature", "min", "max"])
        for cat in cat_order:
            for feat, (mi, ma) in cats[cat].items():
                w.writerow([cat, feat, mi, ma])
    with open(os.path.join(d, "respondents.csv"), "w", newline="", encoding="utf-8") as fh:
        w = csv.writer(fh)
        w.writerow(cat_order)
        for person in people:
            w.writerow(person)
    return d


def quotas(p, k, tight):
    if tight:
        return math.floor(k * p), math.ceil(k * p)
    return math.floor(0.9 * k * p), math.ceil(1.1 * k * p)


def fix_quotas(cat_quota, k):
    """Keep sum(min) <= k <= sum(max) per category (analysis.py:174-176)."""
    mins = sum(v[0] for v in cat_quota.values())
    maxs = sum(v[1] for v in cat_quota.values())
    assert mins <= k <= maxs, (mins, k, maxs)
    return cat_quota


def make_sfe(n=1727, k=110):
    marg = sfe_marginals()
    rng = np.random.default_rng(0)
    cat_order = [c for c, _ in SFE_LAYOUT]
    cols = []
    for cat in cat_order:
        feats = list(marg[cat])
        p = np.array([marg[cat][f] for f in feats])
        q = p * np.exp(rng.normal(0.0, 0.3, size=len(p)))
        q = q / q.sum()
        idx = rng.choice(len(feats), size=n, p=q)
        cols.append([feats[i] for i in idx])
    people = list(zip(*cols))
    for tight, name in ((False, "sf_e"), (True, "sf_e_tight")):
        cats = {}
        for cat in cat_order:
            cats[cat] = fix_quotas({f: quotas(marg[cat][f], k, tight) for f in marg[cat]}, k)
        write_instance(name, k, cats, people, cat_order)


def make_synthetic(n=8192, k=200, C=10):
    rng = np.random.default_rng(0)
    cat_order = ["cat%d" % j for j in range(C)]
    cols, cats = [], {}
    for j, cat in enumerate(cat_order):
        nf = 2 + (j % 5)
        p = rng.dirichlet([2.0] * nf)
        feats = ["%s_f%d" % (cat, i) for i in range(nf)]
        idx = rng.choice(nf, size=n, p=p)
        cols.append([feats[i] for i in idx])
        cats[cat] = fix_quotas({f: quotas(float(x), k, False) for f, x in zip(feats, p)}, k)
    write_instance("synthetic8192", k, cats, list(zip(*cols)), cat_order)


def make_pathological(seed=210, name="pathological"):
    """Small restart-heavy instance (stdlib random.Random(seed) recipe).

    Seed 210 gives n=30, k=5, 3 categories; about 16 attempts per accepted
    panel, with both SelectionError restarts (legacy.py:34) and min-quota
    rejections (analysis.py:155-159).  Seed 50 (n=30, k=6) is rejection-heavy.
    """
    import random
    R = random.Random(seed)
    n = R.choice([20, 30, 40])
    k = R.choice([5, 6, 8])
    nfs = [2, 3, R.choice([2, 4])]
    cat_order = ["x", "y", "z"]
    cats = {}
    for c, nf in enumerate(nfs):
        parts = [0] * nf
        for _ in range(k):
            parts[R.randrange(nf)] += 1
        q = {}
        for i in range(nf):
            lo = max(0, parts[i] - R.choice([0, 0, 1]))
            hi = parts[i] + R.choice([0, 0, 1])
            q["%s%d" % (cat_order[c], i)] = (lo, max(hi, lo))
        cats[cat_order[c]] = fix_quotas(q, k)
    people = []
    for _ in range(n):
        b = R.randrange(6)
        row = []
        for c in range(3):
            i = (b + R.randrange(2)) % nfs[c] if R.random() < 0.6 else R.randrange(nfs[c])
            row.append("%s%d" % (cat_order[c], i))
        people.append(row)
    write_instance(name, k, cats, people, cat_order)


def copy_public():
    for name in ("couples_panel_from_twenty_people_no_constraints_2", "example_small_20",
                 "example_large_200"):
        src = os.path.join(REF, "data", name)
        if not os.path.isdir(src):
            continue
        dst = os.path.join(OUT, name)
        os.makedirs(dst, exist_ok=True)
        for fn in ("categories.csv", "respondents.csv"):
            shutil.copyfile(os.path.join(src, fn), os.path.join(dst, fn))


if __name__ == "__main__":
    os.makedirs(OUT, exist_ok=True)
    copy_public()
    make_sfe()
    make_synthetic()
    make_pathological(210, "pathological")
    make_pathological(50, "rejecty")
    print("instances written to", os.path.normpath(OUT), file=sys.stderr)
