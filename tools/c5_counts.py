"""Per-query work of the C5 radius-normal pass (r = 0.1, grid cell = r) on the bench's C5 cloud,
from a random sample of queries (CPU, numpy + scipy): the candidates a query scans (the points
of the 27 cells around its own) and its neighbours (d2 < r^2).  These are the work counts behind
the fused kernel's ops roofline (tools/c5_roofline.py); the kernel visits exactly these
candidates (its nine row ranges are the 27 cells).  Writes profiles/c5_counts.json.

usage: python tools/c5_counts.py [sample]
"""
from __future__ import annotations

import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    from scipy.spatial import cKDTree
    from dialog_amd.synth import SEED_BASE, plane_cloud
    sample = int(sys.argv[1]) if len(sys.argv) > 1 else 100_000
    r = 0.1
    pts, _, _ = plane_cloud(10_000_000, 20, seed=SEED_BASE + 5)
    lo = pts.min(axis=0)
    cell = np.floor((pts - lo) / r).astype(np.int64)
    g = cell.max(axis=0) + 1
    key = (cell[:, 2] * g[1] + cell[:, 1]) * g[0] + cell[:, 0]
    uk, cnt = np.unique(key, return_counts=True)
    rng = np.random.default_rng(7)
    qi = rng.choice(len(pts), sample, replace=False)
    qc = cell[qi]
    cand = np.zeros(sample, np.int64)
    for dz in (-1, 0, 1):
        for dy in (-1, 0, 1):
            for dx in (-1, 0, 1):
                c = qc + np.array([dx, dy, dz])
                ok = np.all((c >= 0) & (c < g), axis=1)
                k = (c[:, 2] * g[1] + c[:, 1]) * g[0] + c[:, 0]
                pos = np.searchsorted(uk, k)
                pos = np.minimum(pos, len(uk) - 1)
                hit = ok & (uk[pos] == k)
                cand += np.where(hit, cnt[pos], 0)
    tree = cKDTree(pts)
    nb = tree.query_ball_point(pts[qi], r, return_length=True, workers=8)
    out = {"cloud": "bench C5: plane_cloud(10M, 20 planes, seed SEED_BASE + 5)", "radius": r,
           "sample_queries": sample,
           "candidates_per_query_mean": float(cand.mean()),
           "neighbours_per_query_mean": float(nb.mean()),
           "neighbours_pct": {str(p): float(v) for p, v in
                              zip((50, 90, 99, 99.9), np.percentile(nb, (50, 90, 99, 99.9)))},
           "frac_over_256": float((nb > 256).mean()), "frac_over_512": float((nb > 512).mean())}
    os.makedirs(os.path.join(ROOT, "profiles"), exist_ok=True)
    with open(os.path.join(ROOT, "profiles", "c5_counts.json"), "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
