"""Summarise tools/gap_probe's kernel trace: per launch pair, the median gap between the first
kernel's end and the second's start (and between pairs).
    python tools/gap_probe.py <run_kernel_trace.csv>"""
import csv
import statistics
import sys

NAMES = ["baseline 256->256", "256 -> 1024-thread WG", "256 -> 64 KB LDS", "256 -> 132 KB LDS x1024",
         "2048 WGs -> 2048 WGs", "ticket kernel -> small", "small -> ext launch",
         "small -> 1600 x 64-thread WGs", "scorer-shaped -> small", "611 x 1024 -> 611 x 1024"]


def main():
    r = [x for x in csv.DictReader(open(sys.argv[1])) if "k_probe" in x["Kernel_Name"]]
    r.sort(key=lambda x: int(x["Start_Timestamp"]))
    for p, name in enumerate(NAMES):
        seg = r[100 * p:100 * (p + 1)]
        within = [(int(seg[2 * k + 1]["Start_Timestamp"]) - int(seg[2 * k]["End_Timestamp"])) / 1e3
                  for k in range(len(seg) // 2)]
        across = [(int(seg[2 * k + 2]["Start_Timestamp"]) - int(seg[2 * k + 1]["End_Timestamp"])) / 1e3
                  for k in range(len(seg) // 2 - 1)]
        dur_b = [(int(seg[2 * k + 1]["End_Timestamp"]) - int(seg[2 * k + 1]["Start_Timestamp"])) / 1e3
                 for k in range(len(seg) // 2)]
        print(f"{p} {name:32s} gap a->b {statistics.median(within):6.2f} us   b->next a "
              f"{statistics.median(across):6.2f} us   b runs {statistics.median(dur_b):6.2f} us")


if __name__ == "__main__":
    main()
