"""Config C5 (BASELINE.json configs[4]): 10M-point 20-plane cloud, k = 20 normals on the GPU, then
SACMODEL_NORMAL_PLANE extract-and-remove (weight 0.1, threshold 0.02, 4096 hypotheses per round,
<= 20 planes, min 500 inliers, fast refit).  Prints one JSON line with the stage timings."""
import json
import sys
import time

import numpy as np

sys.path.insert(0, ".")
import dialog_amd as D  # noqa: E402
from dialog_amd.synth import SEED_BASE, plane_cloud  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000_000
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 2
p, lab, planes = plane_cloud(n, 20, seed=SEED_BASE + 5)
ctx = D.Context(0)
ctx.set_profiling(True)
res = {"n": n}
t0 = time.perf_counter()
nrm = D.estimate_normals(p, k=20, ctx=ctx)
res["normals_knn20_s"] = round(time.perf_counter() - t0, 3)
t0 = time.perf_counter()
nrm = D.estimate_normals(p, k=20, ctx=ctx)
res["normals_knn20_warm_s"] = round(time.perf_counter() - t0, 3)
cloud = D.Cloud(ctx, p)
cloud.set_normals(nrm)
prm = D.make_params(0.02, max_iterations=4095, probability=1.0, refit_mode=D.DLG_REFIT_FAST,
                    hypotheses_per_launch=4096, gather_inliers=False,
                    model=D.SACMODEL_NORMAL_PLANE, normal_distance_weight=0.1)
for _ in range(1):
    cloud.reset()
    D.extract_planes(cloud, prm, max_planes=20, min_inliers=500, capacity=n)
ctx.synchronize()
t0 = time.perf_counter()
tests = score_ms = 0
for _ in range(steps):
    cloud.reset()
    e = D.extract_planes(cloud, prm, max_planes=20, min_inliers=500, capacity=n)
    tests += e["stats"]["tests"]
    score_ms += e["stats"]["score_ms"]
ctx.synchronize()
dt = (time.perf_counter() - t0) / steps
res.update({"np_extract_ms": round(dt * 1e3, 2), "np_planes": e["n_planes"],
            "np_tests_per_s": round(tests / steps / dt / 1e9, 3),
            "np_score_ms_per_step": round(score_ms / steps, 2),
            "np_kernel_tests_per_s": round(e["stats"]["tests_scored"] / (e["stats"]["score_ms"] / 1e3) / 1e9, 3)})
print(json.dumps(res))
cloud.close()
ctx.close()
