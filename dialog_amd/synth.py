"""Seeded synthetic plane clouds (BASELINE.md §3 "Shared generator").

P planes with normals uniform on S^2 and offsets U[-5, 5]; points uniform on a 10 x 10 patch of
each plane around the plane's foot point, N(0, sigma) noise along the normal; a fraction of
uniform outliers in the bounding box; float32; the point order is randomly permuted so that any
contiguous shard (multi-GPU) sees every plane.  Generator seed = 0xD1A106 + config_id.
"""
from __future__ import annotations

import numpy as np

SEED_BASE = 0xD1A106


def plane_cloud(n_points: int, n_planes: int, outlier_frac: float = 0.1, sigma: float = 0.005,
                seed: int = SEED_BASE, shares=None, patch: float = 10.0, shuffle: bool = True,
                shard: int | None = None):
    """Returns (points float32 [n,3], labels int32 [n] (-1 = outlier), planes float32 [P,4]).

    shard=None: one cloud from `seed`.  shard=r: the planes still come from `seed` but the points
    from an independent stream (seed, r) -- rank r's shard of a weak-scaled multi-GPU cloud.
    """
    rng = np.random.default_rng(seed)
    normals = rng.normal(size=(n_planes, 3))
    normals /= np.linalg.norm(normals, axis=1, keepdims=True)
    offsets = rng.uniform(-5.0, 5.0, size=n_planes)
    if shard is not None:
        rng = np.random.default_rng((seed, int(shard)))
    n_out = int(round(n_points * outlier_frac))
    n_in = n_points - n_out
    if shares is None:
        shares = np.full(n_planes, 1.0 / n_planes)
    shares = np.asarray(shares, np.float64)
    shares = shares / shares.sum()
    counts = np.floor(shares * n_in).astype(np.int64)
    counts[: n_in - counts.sum()] += 1
    pts = np.empty((n_points, 3), np.float32)
    labels = np.empty(n_points, np.int32)
    pos = 0
    for p in range(n_planes):
        nrm = normals[p]
        a = np.array([1.0, 0.0, 0.0]) if abs(nrm[0]) < 0.9 else np.array([0.0, 1.0, 0.0])
        u = np.cross(nrm, a)
        u /= np.linalg.norm(u)
        v = np.cross(nrm, u)
        c = -offsets[p] * nrm
        k = int(counts[p])
        st = rng.uniform(-patch / 2, patch / 2, size=(k, 2))
        eps = rng.normal(0.0, sigma, size=k)
        blk = c + st[:, :1] * u + st[:, 1:] * v + eps[:, None] * nrm
        pts[pos:pos + k] = blk.astype(np.float32)
        labels[pos:pos + k] = p
        pos += k
    if n_out:
        lo = pts[:pos].min(axis=0) if pos else np.full(3, -5.0, np.float32)
        hi = pts[:pos].max(axis=0) if pos else np.full(3, 5.0, np.float32)
        pts[pos:] = rng.uniform(lo, hi, size=(n_out, 3)).astype(np.float32)
        labels[pos:] = -1
    if shuffle:
        perm = rng.permutation(n_points)
        pts, labels = pts[perm], labels[perm]
    planes = np.concatenate([normals, offsets[:, None]], axis=1).astype(np.float32)
    return np.ascontiguousarray(pts), labels, planes


CONFIGS = {
    # id: (n_points, n_planes, shares, ransac kwargs)
    2: dict(n_points=1_000_000, n_planes=3, shares=[1, 1, 1]),
    3: dict(n_points=10_000_000, n_planes=20, shares=None),
    4: dict(n_points=100_000_000, n_planes=20, shares=None),
    5: dict(n_points=10_000_000, n_planes=20, shares=None),
}


def config_cloud(config_id: int, n_points: int | None = None, seed_offset: int = 0):
    c = CONFIGS[config_id]
    return plane_cloud(n_points or c["n_points"], c["n_planes"], shares=c["shares"],
                       seed=SEED_BASE + config_id + seed_offset)


def postprocess_scene(n_points: int, n_planes: int, keep_frac: float = 0.7, n_border: int = 40,
                      seed: int = SEED_BASE + 6, outlier_frac: float = 0.1, sigma: float = 0.005):
    """A cloud plus the plane list postProcessPlanes receives (Dialog/PlaneDetect.h:1454).

    points_set of plane p = a random keep_frac of its points (the rest stays unclaimed in the
    cloud); border = a concave star polygon (n_border vertices, radii alternating 4.6 / 3.2 around
    the patch centre, counter-clockwise about the normal), lying on the plane; coeff = the plane
    normal with a random sign (postProcessPlanes re-orients the refit normal by it).
    Returns (cloud float32 [n, 3], planes: list of dict(coeff, points, border)).
    """
    pts, lab, planes = plane_cloud(n_points, n_planes, outlier_frac=outlier_frac, sigma=sigma,
                                   seed=seed)
    rng = np.random.default_rng((seed, 99))
    out = []
    for p in range(n_planes):
        nrm = planes[p, :3].astype(np.float64)
        a = np.array([1.0, 0.0, 0.0]) if abs(nrm[0]) < 0.9 else np.array([0.0, 1.0, 0.0])
        u = np.cross(nrm, a)
        u /= np.linalg.norm(u)
        v = np.cross(nrm, u)
        c = -float(planes[p, 3]) * nrm
        th = np.arange(n_border) * (2.0 * np.pi / n_border)
        r = np.where(np.arange(n_border) % 2 == 0, 4.6, 3.2)
        border = (c + (r * np.cos(th))[:, None] * u + (r * np.sin(th))[:, None] * v)
        ids = np.nonzero(lab == p)[0]
        keep = np.sort(rng.choice(ids, size=int(round(keep_frac * ids.size)), replace=False))
        sign = 1.0 if rng.random() < 0.5 else -1.0
        out.append(dict(coeff=(sign * planes[p, :3]).astype(np.float32), points=pts[keep].copy(),
                        border=border.astype(np.float32)))
    return pts, out
