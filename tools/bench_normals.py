"""Normals-path timing on the C5 shape (10M points, 20 planes): radius normals, k = 20 normals and
RegulateNormal, wall time per call (host buffers in and out, as the C ABI takes them)."""
import json
import sys
import time

import numpy as np

sys.path.insert(0, ".")
import dialog_amd as D  # noqa: E402
from dialog_amd.synth import SEED_BASE, plane_cloud  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000_000
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
p, lab, planes = plane_cloud(n, 20, seed=SEED_BASE + 5)
ctx = D.Context(0)
res = {"n": n}


def timed(name, f):
    f()
    t0 = time.perf_counter()
    for _ in range(reps):
        out = f()
    res[name + "_ms"] = round((time.perf_counter() - t0) / reps * 1e3, 2)
    return out


g = timed("radius_r0.05", lambda: D.estimate_normals(p, radius=0.05, ctx=ctx))
res["radius_nan_frac"] = float(np.isnan(g[:, 0]).mean())
m = lab >= 0
res["radius_inlier_median_absdot"] = float(np.nanmedian(
    np.abs(np.sum(g[m, :3] * planes[lab[m], :3], axis=1))))
k = timed("knn20", lambda: D.estimate_normals(p, k=20, ctx=ctx))
res["knn_inlier_median_absdot"] = float(np.median(
    np.abs(np.sum(k[m, :3] * planes[lab[m], :3], axis=1))))
r = timed("regulate_r0.05", lambda: D.regulate_normals(p, g, 0, True, 0.05, ctx=ctx))
res["regulate_processed"] = r[2]
print(json.dumps(res))
ctx.close()
