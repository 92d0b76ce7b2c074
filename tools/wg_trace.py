"""Summarise the scoring launch's per-workgroup trace (A/B build with -DDLG_WG_TRACE: every
workgroup of k_score_tiles_ex prints "WGT <block> <start> <end> <items claimed>", 100 MHz ticks).

    DLG_EXTRA_CXXFLAGS=-DDLG_WG_TRACE bash tools/build_ab.sh wgtrace HEAD spatial.hip
    KERNELS=2 PRUNE_STATS=1 python tools/with_lib.py ab_libs/wgtrace.so tools/score_ab.py 1500000 4096 1 > log
    python tools/wg_trace.py log

Per launch (launches are sequential on one stream: workgroups sorted by start, 256 a launch):
the launch's span, the workgroups' start skew, end times (mean / p90 / max) from the first start,
per XCD (block & 7) the mean and latest end, and the claims of the latest-ending workgroups.
(A per-item printf was tried and dropped: at 1.5M points it stretched one launch to minutes.)
"""
import json
import sys

import numpy as np


def main():
    rows = []
    for line in open(sys.argv[1], errors="replace"):
        p = line.split()
        if len(p) == 5 and p[0] == "WGT":
            rows.append((int(p[1]), int(p[2]), int(p[3]), int(p[4])))
    g = int(sys.argv[2]) if len(sys.argv) > 2 else 256
    rows.sort(key=lambda r: r[1])
    out = []
    for k in range(0, len(rows) - g + 1, g):
        a = np.array(rows[k:k + g], dtype=np.int64)
        b, t0, t1, cl = a[:, 0], a[:, 1], a[:, 2], a[:, 3]
        z = t0.min()
        end = (t1 - z) / 100.0
        start = (t0 - z) / 100.0
        span = (t1 - t0) / 100.0
        x = b & 7
        late = np.argsort(-end)[:5]
        out.append(dict(
            launch=k // g, span_us=round(float(end.max()), 1), start_skew_us=round(float(start.max()), 1),
            end_mean=round(float(end.mean()), 1), end_p90=round(float(np.percentile(end, 90)), 1),
            wg_span_mean=round(float(span.mean()), 1),
            xcd_end_mean=[round(float(end[x == i].mean()), 1) for i in range(8)],
            xcd_end_max=[round(float(end[x == i].max()), 1) for i in range(8)],
            claims_mean=round(float(cl.mean()), 1), claims_min=int(cl.min()), claims_max=int(cl.max()),
            latest=[dict(block=int(b[i]), start=round(float(start[i]), 1), end=round(float(end[i]), 1),
                         claims=int(cl[i])) for i in late]))
    for o in out:
        print(json.dumps(o))


if __name__ == "__main__":
    main()
