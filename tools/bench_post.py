"""postProcessPlanes timing (Dialog/PlaneDetect.h:1454-1579) on a C5-sized scene: 10M points,
20 planes, 70% of each plane's points already in its points_set, concave star borders of
`n_border` vertices; wall time per call (host buffers in and out, as the C ABI takes them) plus
the work counts that size the absorption kernel (candidates x 10 rays x border edges)."""
import json
import sys
import time

import numpy as np

sys.path.insert(0, ".")
import dialog_amd as D  # noqa: E402
from dialog_amd.synth import SEED_BASE, postprocess_scene  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000_000
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
nb = int(sys.argv[3]) if len(sys.argv) > 3 else 1000
t0 = time.perf_counter()
cloud, planes = postprocess_scene(n, 20, n_border=nb, seed=SEED_BASE + 5)
res = {"n": n, "planes": 20, "border_vertices": nb, "gen_s": round(time.perf_counter() - t0, 2)}
ctx = D.Context(0)
prm = D.PostProcessParams(t_dist_point_plane=0.1, radius_local=0.1, t_cluster_num=500,
                          plane_start_index=0, rand_seed=12345)
out = D.post_process_planes(cloud, planes, prm, ctx=ctx)
t0 = time.perf_counter()
for _ in range(reps):
    out = D.post_process_planes(cloud, planes, prm, ctx=ctx)
res["post_process_ms"] = round((time.perf_counter() - t0) / reps * 1e3, 2)
co, ab, rem = out
res["absorbed"] = int(sum(a.size for a in ab))
res["remaining"] = int(rem.size)
t0 = time.perf_counter()
for _ in range(reps):
    D.refit_planes(planes)
res["refit_host_ms"] = round((time.perf_counter() - t0) / reps * 1e3, 2)
t0 = time.perf_counter()
for _ in range(reps):
    D.cluster_filter(cloud[rem], 0.1, 500, ctx=ctx)
res["cluster_filter_ms"] = round((time.perf_counter() - t0) / reps * 1e3, 2)
print(json.dumps(res))
ctx.close()
