"""Which inter-kernel gaps are the host's: joins a rocprofv3 --kernel-trace --hip-trace run's
kernel and HIP API traces by correlation id and, over the last N scoring rounds, reports per
kernel pair the GPU gap (next start - previous end) and how late the host's launch call
returned relative to the previous kernel's end (> 0: the GPU waited for the host to enqueue).

    python tools/host_gaps.py <dir with run_kernel_trace.csv, run_hip_api_trace.csv> [rounds]
"""
import collections
import csv
import glob
import os
import re
import sys


def nm(x):
    m = re.search(r'(k_\w+|fill\w*|copy\w*|trampoline)', x)
    return m.group(1) if m else x[:30]


def main():
    d = sys.argv[1]
    rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    kt = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)[0]
    ht = glob.glob(os.path.join(d, "**", "*hip_api_trace.csv"), recursive=True)[0]
    ks = list(csv.DictReader(open(kt)))
    ks.sort(key=lambda x: int(x["Start_Timestamp"]))
    api = {}
    for x in csv.DictReader(open(ht)):
        if "Launch" in x.get("Function", "") or "launch" in x.get("Function", ""):
            api[x["Correlation_Id"]] = (int(x["Start_Timestamp"]), int(x["End_Timestamp"]), x["Function"])
    idx = [i for i, x in enumerate(ks) if "k_score_tiles" in x["Kernel_Name"]]
    seg = ks[idx[-rounds] - 2:]
    g = collections.defaultdict(list)
    for a, b in zip(seg, seg[1:]):
        gap = (int(b["Start_Timestamp"]) - int(a["End_Timestamp"])) / 1e3
        call = api.get(b["Correlation_Id"])
        late = (call[1] - int(a["End_Timestamp"])) / 1e3 if call else float("nan")
        lead = (int(b["Start_Timestamp"]) - call[1]) / 1e3 if call else float("nan")
        g[(nm(a["Kernel_Name"]), nm(b["Kernel_Name"]))].append((gap, late, lead, call[2] if call else "?"))
    print(f"{'pair':48s} {'n':>3} {'gap':>7} {'host late':>9} {'start-after-call':>16}  api")
    for k, v in sorted(g.items(), key=lambda kv: -sum(t[0] for t in kv[1])):
        n = len(v)
        print(f"{k[0] + ' -> ' + k[1]:48s} {n:3d} {sum(t[0] for t in v) / n:7.1f} "
              f"{sum(t[1] for t in v) / n:9.1f} {sum(t[2] for t in v) / n:16.1f}  {v[0][3]}")


if __name__ == "__main__":
    main()
