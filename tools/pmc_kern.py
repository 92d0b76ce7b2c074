"""Mean per-dispatch PMC counters of the kernels whose name contains a pattern, from one or more
rocprofv3 --pmc counter_collection.csv files (one per pass).
Usage: python tools/pmc_kern.py <pattern>[,<pattern>...] <csv> [<csv> ...]"""
import collections
import csv
import json
import re
import sys


def main():
    pats = sys.argv[1].split(",")
    out = {}
    for path in sys.argv[2:]:
        per = collections.defaultdict(lambda: collections.defaultdict(float))
        names = {}
        for r in csv.DictReader(open(path)):
            m = re.search(r"(k_\w+)", r["Kernel_Name"])
            name = m.group(1) if m else r["Kernel_Name"][:40]
            if not any(p in r["Kernel_Name"] for p in pats):
                continue
            key = (name, r["Dispatch_Id"])
            names[key] = name
            per[key][r["Counter_Name"]] += float(r["Counter_Value"])
        by = collections.defaultdict(list)
        for key, d in per.items():
            by[key[0]].append(d)
        for name, ds in by.items():
            o = out.setdefault(name, {"dispatches": len(ds)})
            for c in sorted({c for d in ds for c in d}):
                o[c] = round(sum(d.get(c, 0.0) for d in ds) / len(ds))
    for name, o in out.items():
        wc = o.get("SQ_WAVE_CYCLES")
        if wc:
            for c in ("SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY",
                      "SQ_WAIT_INST_LDS", "SQ_ACTIVE_INST_LDS", "SQ_ACTIVE_INST_SCA"):
                if c in o:
                    o[c + "_frac"] = round(o[c] / wc, 4)
        if o.get("SQ_LDS_IDX_ACTIVE"):
            o["lds_conflict_frac"] = round(o.get("SQ_LDS_BANK_CONFLICT", 0) / o["SQ_LDS_IDX_ACTIVE"], 4)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
