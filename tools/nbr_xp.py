import sys, time, json
sys.path.insert(0, __import__("os").environ.get("GRAFT_REPO_ROOT", "."))
import numpy as np
import dialog_amd as D
from dialog_amd.synth import SEED_BASE, plane_cloud
p, lab, planes = plane_cloud(10_000_000, 20, seed=SEED_BASE + 5)
res = {}
for v in (1, 11, 12, 14, 13, 17):
    ctx = D.Context(0); ctx.set_option(D.DLG_OPT_NORMALS_FUSED, v)
    D.estimate_normals(p, radius=0.1, ctx=ctx)
    t0 = time.perf_counter(); D.estimate_normals(p, radius=0.1, ctx=ctx); res[v] = round((time.perf_counter()-t0)*1e3, 1)
    ctx.close()
print(json.dumps(res))
