"""Summarise rocprofv3 --pmc CSVs per kernel (sum over dispatches of each kernel instance)."""
import collections
import csv
import re
import sys

for f in sys.argv[1:]:
    rows = list(csv.DictReader(open(f)))
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    for r in rows:
        k = r["Kernel_Name"]
        m = re.search(r"(k_score\w*<[^>]*>|k_\w+)", k)
        if not m or not any(t in k for t in ("k_score", "k_prune")):
            continue
        name = m.group(0)
        disp[name].add(r["Dispatch_Id"])
        agg[name][r["Counter_Name"]] += float(r["Counter_Value"])
    for name, d in agg.items():
        nd = len(disp[name])
        print(f, name, {a: f"{b / nd:.4g}" for a, b in sorted(d.items())})
