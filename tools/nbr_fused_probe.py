"""Radius-0.1 PCL-float normals on the C5 cloud (10M points): fused pass vs chunked pipeline, wall
time per call, and the fused pass's overflow counts (queries with > 256 / > 1024 neighbours).
Usage: python tools/nbr_fused_probe.py [n] [reps]"""
import json
import sys
import time

import numpy as np

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
import dialog_amd as D  # noqa: E402
from dialog_amd.synth import SEED_BASE, plane_cloud  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000_000
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 2
p, lab, planes = plane_cloud(n, 20, seed=SEED_BASE + 5)
res = {"n": n}
out = {}
for fused in (1, 0):
    ctx = D.Context(0)
    ctx.set_option(D.DLG_OPT_NORMALS_FUSED, fused)
    g = D.estimate_normals(p, radius=0.1, ctx=ctx)
    t0 = time.perf_counter()
    for _ in range(reps):
        g = D.estimate_normals(p, radius=0.1, ctx=ctx)
    res[f"fused{fused}_ms"] = round((time.perf_counter() - t0) / reps * 1e3, 2)
    out[fused] = g
    ctx.close()
a, b = out[1], out[0]
res["equal"] = bool(np.array_equal(np.isnan(a), np.isnan(b)) and
                    np.array_equal(a[~np.isnan(b[:, 0])].view(np.uint32), b[~np.isnan(b[:, 0])].view(np.uint32)))
print(json.dumps(res), flush=True)
