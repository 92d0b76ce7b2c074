"""One k = 20 normal estimation of the C5 cloud (10M points), for PMC passes on k_normals_knn."""
import sys

sys.path.insert(0, ".")
import dialog_amd as D  # noqa: E402
from dialog_amd.synth import SEED_BASE, plane_cloud  # noqa: E402

p, lab, planes = plane_cloud(10_000_000, 20, seed=SEED_BASE + 5)
ctx = D.Context(0)
D.estimate_normals(p, k=20, ctx=ctx)
ctx.close()
