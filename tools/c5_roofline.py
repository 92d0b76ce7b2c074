"""Rooflines of the C5 kernels from a kernel-trace profile of tools/c5_kernels.py (tools/gpu.sh
c5prof) and the work counts of tools/c5_counts.py (profiles/c5_counts.json).

  k_nbr_fused (radius 0.1 normals, one pass): ops view.  Per query: FLANN's d2 over every
    candidate of the 27 cells (3 sub + 3 mul + 3 add, the compare: 10 lane-ops) and the nine
    float chains over the neighbours (mul + add: 18 lane-ops); against the f32 VALU peak (78.6 T
    lane-ops/s without FMA).  Its HBM view (12 B per point read once, 16 B written) beside it.
  k_normals_knn (k = 20, all levels): HBM view (12 B read + 16 B written per query) and time per
    query.
  k_bfs2_claim (RegulateNormal): HBM view per reached node (its point and normal read, 28 B).

usage: python tools/c5_roofline.py <kernel_stats.csv> [c5_kernels.log] > profiles/<tag>_c5_rooflines.json
"""
from __future__ import annotations

import csv
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
VALU_PEAK = 256 * 4 * 32 * 2.4e9  # f32 lane-ops/s, non-FMA (bench.py VALU_PEAK_TOPS)
HBM_PEAK = 8.0e12


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    counts = json.load(open(os.path.join(ROOT, "profiles", "c5_counts.json")))
    wall = {}
    if len(sys.argv) > 2:
        for ln in open(sys.argv[2]):
            if ln.startswith("{"):
                wall = json.loads(ln)
    n = int(wall.get("n", 10_000_000))

    def kern(pat):
        sel = [r for r in rows if pat in r["Name"]]
        calls = sum(int(r["Calls"]) for r in sel)
        tot = sum(float(r["TotalDurationNs"]) for r in sel)
        return calls, tot

    out = {"source": os.path.relpath(sys.argv[1], ROOT), "points": n, "stage_wall_ms": wall}
    # each stage runs twice in c5_kernels.py (warm + timed): per-stage time = total / 2
    c, t = kern("k_nbr_fused")
    if c:
        ms = t / 2 / 1e6
        cand, nb = counts["candidates_per_query_mean"], counts["neighbours_per_query_mean"]
        ops = n * (10.0 * cand + 18.0 * nb)
        out["k_nbr_fused"] = {
            "launches_per_stage": c // 2, "ms_per_stage": round(ms, 3), "bound": "valu (ops view)",
            "ops_per_query": round(10.0 * cand + 18.0 * nb, 1),
            "achieved": round(ops / (ms / 1e3) / 1e12, 3), "peak": round(VALU_PEAK / 1e12, 2),
            "unit": "T lane-ops/s", "frac": round(ops / (ms / 1e3) / VALU_PEAK, 4),
            "hbm_view": {"alg_bytes": 28 * n, "achieved_GBs": round(28 * n / (ms / 1e3) / 1e9, 1),
                         "frac": round(28 * n / (ms / 1e3) / HBM_PEAK, 5)},
            "counts": "profiles/c5_counts.json (candidates %.0f, neighbours %.0f per query)" % (cand, nb)}
    c, t = kern("k_normals_knn")
    if c:
        ms = t / 2 / 1e6
        out["k_normals_knn"] = {
            "launches_per_stage": c // 2, "ms_per_stage": round(ms, 3),
            "bound": "latency (candidate scan, top-k network); hbm view",
            "ns_per_query": round(ms * 1e6 / n, 2),
            "achieved": round(28 * n / (ms / 1e3) / 1e9, 1), "peak": HBM_PEAK / 1e9, "unit": "GB/s",
            "frac": round(28 * n / (ms / 1e3) / HBM_PEAK, 5)}
    c, t = kern("k_bfs2_claim")
    if c:
        ms = t / 2 / 1e6
        reached = int(wall.get("regulate_reached", 0)) or n
        out["k_bfs2_claim"] = {
            "launches_per_stage": c // 2, "ms_per_stage": round(ms, 3),
            "us_per_level": round(ms * 1e3 / max(c // 2, 1), 2),
            "bound": "latency (level-synchronous BFS); hbm view",
            "achieved": round(28 * reached / (ms / 1e3) / 1e9, 1), "peak": HBM_PEAK / 1e9,
            "unit": "GB/s", "frac": round(28 * reached / (ms / 1e3) / HBM_PEAK, 5)}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
