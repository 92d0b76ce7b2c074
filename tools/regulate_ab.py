"""A/B of RegulateNormal's claim pass (DLG_OPT_REGULATE_WAVE 1 / 0) on the C5 cloud (10M points,
radius-0.1 PCL normals, r 0.1, seed 0): wall ms per call, results checked equal.
usage: python tools/regulate_ab.py [reps]"""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import dialog_amd as D  # noqa: E402
from dialog_amd.synth import SEED_BASE, plane_cloud  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
p, _, _ = plane_cloud(10_000_000, 20, seed=SEED_BASE + 5)
ctx = D.Context(0)
nrm = D.estimate_normals(p, radius=0.1, ctx=ctx)
res = {1: [], 0: []}
ref = None
for r in range(reps + 1):
    for v in (1, 0):
        ctx.set_option(D.DLG_OPT_REGULATE_WAVE, v)
        t0 = time.perf_counter()
        g, proc, cnt = D.regulate_normals(p, nrm, 0, True, 0.1, ctx=ctx)
        if r:
            res[v].append((time.perf_counter() - t0) * 1e3)
        if ref is None:
            ref = (g, proc, cnt)
        assert cnt == ref[2] and np.array_equal(proc, ref[1]) and \
            np.array_equal(g.view(np.uint32), ref[0].view(np.uint32)), "claim passes differ"
print(json.dumps({f"regulate_wave={v}_ms": round(sorted(x)[len(x) // 2], 2) for v, x in res.items()}
                 | {"reached": int(ref[2])}))
