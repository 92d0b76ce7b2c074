"""The C5 stages once each, warm, for a kernel-trace profile (tools/gpu.sh c5prof): k = 20 and
radius 0.1 normals on a cloud's device copy, RegulateNormal on the device copy (after the k = 20
normals) and (r 0.1, seed 0) from host records.
Prints the stage wall times as one JSON line.

usage: python tools/c5_kernels.py [points]
"""
import json
import os
import sys
import time

sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(
    os.path.abspath(__file__)))))
import dialog_amd as D  # noqa: E402
from dialog_amd.synth import SEED_BASE, plane_cloud  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000_000
p, _, _ = plane_cloud(n, 20, seed=SEED_BASE + 5)
ctx = D.Context(0)
cloud = D.Cloud(ctx, p)
res = {"n": n}


def timed(name, f):
    f()  # (warm: buffers allocated, code loaded)
    ctx.synchronize()
    t0 = time.perf_counter()
    r = f()
    ctx.synchronize()
    res[name] = round((time.perf_counter() - t0) * 1e3, 2)
    return r


timed("cloud_normals_knn20_ms", lambda: cloud.estimate_normals(k=20))
timed("cloud_regulate_r0.1_ms", lambda: cloud.regulate_normals(0, True, 0.1))
rn = timed("cloud_normals_radius0.1_ms", lambda: cloud.estimate_normals(radius=0.1, copy_out=True))
res["regulate_reached"] = timed("regulate_r0.1_ms",
                                lambda: D.regulate_normals(p, rn, 0, True, 0.1, ctx=ctx))[2]
cloud.close()
ctx.close()
print(json.dumps(res))
