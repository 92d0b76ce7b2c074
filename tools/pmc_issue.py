"""Issue-side view of the dominant scoring kernel from a rocprofv3 --pmc pass over
`bench.py --steps 1 --warmup 0 ...` (counters: SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY SQ_WAIT_ANY
SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES
GRBM_GUI_ACTIVE).  Per MI355X_MICROARCH.md: WAVE_CYCLES = ACTIVE_INST_ANY + WAIT_ANY +
WAIT_INST_ANY (disjoint, quad-cycles); SQ_VALU_MFMA_BUSY_CYCLES counts cycles (32 per 32x32x16 bf16
MFMA).  Writes profiles/score_issue.json (read by bench.py into roofline.issue_view).
Usage: python tools/pmc_issue.py <counter_collection.csv> [kernel=k_score_tiles_ex] [num_cus=256]"""
import collections
import csv
import json
import os
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    path = sys.argv[1]
    kern = sys.argv[2] if len(sys.argv) > 2 else "k_score_tiles_ex"
    cus = int(sys.argv[3]) if len(sys.argv) > 3 else 256
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    for r in csv.DictReader(open(path)):
        m = re.search(r"(k_\w+)", r["Kernel_Name"])
        if not m or m.group(1) != kern:
            continue
        per[r["Dispatch_Id"]][r["Counter_Name"]] += float(r["Counter_Value"])
    if not per:
        raise SystemExit(f"no dispatch of {kern} in {path}")
    n = len(per)
    mean = {c: sum(d.get(c, 0.0) for d in per.values()) / n
            for c in sorted({c for d in per.values() for c in d})}
    wc = mean.get("SQ_WAVE_CYCLES", 0.0) or 1.0
    out = {"kernel": kern, "dispatches": n, "source": f"rocprofv3 --pmc, {os.path.basename(path)}",
           "per_launch": {k: round(v) for k, v in mean.items()},
           "active_inst_frac": round(mean.get("SQ_ACTIVE_INST_ANY", 0) / wc, 4),
           "valu_active_frac": round(mean.get("SQ_ACTIVE_INST_VALU", 0) / wc, 4),
           "wait_any_frac": round(mean.get("SQ_WAIT_ANY", 0) / wc, 4),
           "wait_inst_any_frac": round(mean.get("SQ_WAIT_INST_ANY", 0) / wc, 4)}
    g = mean.get("GRBM_GUI_ACTIVE", 0.0)
    if g:
        # MFMA pipe utilisation: busy cycles over (kernel cycles x SIMDs)
        out["mfma_busy_frac"] = round(mean.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0) / (g * cus * 4), 4)
    out["valu_insts_per_mfma"] = round(mean.get("SQ_INSTS_VALU", 0.0) / max(mean.get("SQ_INSTS_MFMA", 0.0), 1.0), 2)
    json.dump(out, open(os.path.join(ROOT, "profiles", "score_issue.json"), "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
