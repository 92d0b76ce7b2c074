"""Per-kernel summary of a rocprofv3 --kernel-trace --stats directory: calls, average and total
time, share of GPU time (the *_kernel_stats.csv), short kernel names.
Usage: python tools/kstats.py <rocprofv3 output dir> [top]"""
import csv
import glob
import os
import re
import sys


def short(name):
    name = name.replace("dlg::(anonymous namespace)::", "")
    name = re.sub(r"\(.*", "", name)
    name = re.sub(r"^void ", "", name)
    return name[:60]


def main():
    d = sys.argv[1]
    top = int(sys.argv[2]) if len(sys.argv) > 2 else 24
    f = glob.glob(os.path.join(d, "**", "*kernel_stats.csv"), recursive=True)[0]
    rows = list(csv.DictReader(open(f)))
    print(f"{'kernel':60s} {'calls':>6s} {'avg_us':>9s} {'total_ms':>9s} {'%':>6s}")
    for r in rows[:top]:
        print(f"{short(r['Name']):60s} {int(r['Calls']):6d} {float(r['AverageNs']) / 1e3:9.2f} "
              f"{float(r['TotalDurationNs']) / 1e6:9.3f} {float(r['Percentage']):6.2f}")


if __name__ == "__main__":
    main()
