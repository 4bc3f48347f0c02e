"""Extract the reference's published LEGACY statistics lines into tests/golden/published_stats.json.

Reads reference_output/*_statistics.txt and analysis/*_statistics.txt under the reference
checkout (read-only, this container only) and keeps, per instance, the formatted strings the
reference printed (analysis.py:568-597): the 99% upper confidence bound and the sample
proportion it came from, the gini coefficient and the geometric mean of the seed-0 LEGACY
allocation.  The allocations themselves are in tests/golden/mt_published.json.

    python tools/extract_published_stats.py [/root/reference]
"""
import json
import os
import re
import sys

REF = sys.argv[1] if len(sys.argv) > 1 else "/root/reference"
FILES = {
    "example_small_20": ("reference_output/example_small_20_statistics.txt",
                         "reference_output/example_small_20_ratio_product_data.csv"),
    "example_large_200": ("reference_output/example_large_200_statistics.txt",
                          "reference_output/example_large_200_ratio_product_data.csv"),
    "couples_panel_from_twenty_people_no_constraints_2": (
        "analysis/couples_panel_from_twenty_people_no_constraints_2_statistics.txt",
        "analysis/couples_panel_from_twenty_people_no_constraints_2_ratio_product_data.csv"),
}
out = {}
for inst, (stats, alloc_key) in FILES.items():
    with open(os.path.join(REF, stats), encoding="utf-8") as fh:
        text = fh.read()
    m = re.search(r"LEGACY minimum probability:\t≤ ([0-9.]+%) .*sample proportion ([0-9.]+) and sample size", text)
    out[inst] = {
        "source": stats,
        "alloc_key": alloc_key,
        "ucb": m.group(1),
        "minimizer_prop": m.group(2),
        "gini": re.search(r"gini coefficient of LEGACY:\t([0-9.]+%)", text).group(1),
        "geometric_mean": re.search(r"geometric mean of LEGACY:\t([0-9.]+%)", text).group(1),
    }
dst = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "golden",
                   "published_stats.json")
with open(dst, "w") as fh:
    json.dump(out, fh, indent=1, ensure_ascii=False)
print(json.dumps(out, indent=1, ensure_ascii=False))
