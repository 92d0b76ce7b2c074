"""Alpha-shape fixtures for the plane borders (dlg_plane_border / dialog_amd/csrc/alpha_shape.hpp),
generated with qhull through scipy.spatial.Delaunay(points, qhull_options="QJ") -- the same
library and option string ("d QJ") pcl::ConcaveHull hands its projected points to
(polyPointCloud, Dialog/PlaneDetect.h:1399-1405).  scipy's qhull is not PCL 1.8.1's qhull 2015.2
and the joggle is seeded differently; for points in general position the Delaunay
triangulation is unique, so the triangles, the alpha filter and the boundary are pinned by it.

Per case (2-D): the points, alpha, qhull's triangles (sorted vertex triples), which of them the
alpha filter keeps (circumradius <= alpha, measured from the circumcentre to the first vertex as
ConcaveHull measures it), the boundary edges (a kept triangle's edge whose other side is not a
kept triangle) and the boundary's connected components as vertex sets (PCL's polygons, up to
walk order).  Cases whose circumradii come within 1e-9 (relative) of alpha are re-drawn, so
rounding cannot move a triangle across the filter.  Per 3-D case: plane points for the
end-to-end dlg_plane_border test, with the boundary vertex set of the largest polygon computed
through a float64 restatement of ConcaveHull's projection (PCA frame).

Usage: python tests/golden/make_alpha.py   -> tests/golden/alpha_shapes.npz
"""
import os

import numpy as np
from scipy.spatial import Delaunay

HERE = os.path.dirname(os.path.abspath(__file__))


def alpha_complex(xy, alpha):
    d = Delaunay(xy, qhull_options="QJ")
    s = d.simplices
    a, b, c = xy[s[:, 0]], xy[s[:, 1]], xy[s[:, 2]]
    dx, dy = b[:, 0] - a[:, 0], b[:, 1] - a[:, 1]
    ex, ey = c[:, 0] - a[:, 0], c[:, 1] - a[:, 1]
    bl, cl = dx * dx + dy * dy, ex * ex + ey * ey
    dd = 0.5 / (dx * ey - dy * ex)
    ux, uy = (ey * bl - dy * cl) * dd, (dx * cl - ex * bl) * dd
    r = np.sqrt(ux * ux + uy * uy)
    kept = r <= alpha
    near = np.abs(r - alpha) <= 1e-9 * alpha
    # boundary: edges of kept triangles not shared with another kept triangle
    cnt = {}
    for t in np.nonzero(kept)[0]:
        v = s[t]
        for i in range(3):
            e = tuple(sorted((int(v[i]), int(v[(i + 1) % 3]))))
            cnt[e] = cnt.get(e, 0) + 1
    bedges = sorted(e for e, k in cnt.items() if k == 1)
    # components of the boundary graph
    adj = {}
    for a_, b_ in bedges:
        adj.setdefault(a_, []).append(b_)
        adj.setdefault(b_, []).append(a_)
    comps, seen = [], set()
    for v in sorted(adj):
        if v in seen:
            continue
        st, comp = [v], []
        seen.add(v)
        while st:
            u = st.pop()
            comp.append(u)
            for w in adj[u]:
                if w not in seen:
                    seen.add(w)
                    st.append(w)
        comps.append(sorted(comp))
    tri = np.sort(s, axis=1)
    order = np.lexsort((tri[:, 2], tri[:, 1], tri[:, 0]))
    return tri[order], kept[order], np.array(bedges, np.int32).reshape(-1, 2), comps, bool(near.any())


def shape(rng, kind, n):
    if kind == "square":
        return rng.uniform(0, 10, (n, 2))
    if kind == "L":
        p = rng.uniform(0, 10, (3 * n, 2))
        return p[(p[:, 0] < 5) | (p[:, 1] < 5)][:n]
    if kind == "annulus":  # a hole: two boundary polygons
        p = rng.uniform(-5, 5, (3 * n, 2))
        r = np.hypot(p[:, 0], p[:, 1])
        return p[(r < 5) & (r > 2)][:n]
    if kind == "blobs":  # two separate pieces
        a = rng.normal(0, 1.0, (n // 2, 2))
        b = rng.normal(0, 1.0, (n - n // 2, 2)) + [8.0, 1.0]
        return np.vstack([a, b])
    if kind == "graded":  # density falling off: the alpha filter cuts the sparse fringe
        r = rng.exponential(2.0, n)
        t = rng.uniform(0, 2 * np.pi, n)
        return np.stack([r * np.cos(t), r * np.sin(t)], 1)
    raise ValueError(kind)


def frame3(n):
    n = np.asarray(n, np.float64)
    n = n / np.linalg.norm(n)
    u = np.cross(n, [1.0, 0, 0] if abs(n[0]) < 0.9 else [0, 1.0, 0])
    u /= np.linalg.norm(u)
    return n, u, np.cross(n, u)


def main():
    out = {}
    cases2 = [("square", 800, 0.5), ("L", 3000, 0.5), ("annulus", 4000, 0.4), ("blobs", 2000, 0.6),
              ("graded", 3000, 0.5)]
    names = []
    for k, (kind, n, alpha) in enumerate(cases2):
        for seed in range(100):
            rng = np.random.default_rng(1000 * k + seed)
            xy = shape(rng, kind, n)
            tri, kept, be, comps, near = alpha_complex(xy, alpha)
            if not near:
                break
        name = f"c2_{kind}"
        names.append(name)
        out[f"{name}_xy"] = xy
        out[f"{name}_alpha"] = np.float64(alpha)
        out[f"{name}_tri"] = tri.astype(np.int32)
        out[f"{name}_kept"] = kept
        out[f"{name}_bedges"] = be
        out[f"{name}_comp_sizes"] = np.array([len(c) for c in comps], np.int32)
        out[f"{name}_comp_verts"] = np.array([v for c in comps for v in c], np.int32)
    # 3-D plane patches for dlg_plane_border (float32 points, alpha_poly-like alpha)
    cases3 = [("square", (0.3, -0.5, 0.8), 2.0, 6000, 0.5), ("L", (1, 2, -0.5), 0.5, 8000, 0.5)]
    for k, (kind, normal, off, n, alpha) in enumerate(cases3):
        for seed in range(100):
            rng = np.random.default_rng(77 + 1000 * k + seed)
            st = shape(rng, kind, n)
            nrm, u, v = frame3(normal)
            p = (off * nrm + st[:, :1] * u + st[:, 1:] * v +
                 rng.normal(0, 0.003, (len(st), 1)) * nrm).astype(np.float32)
            # ConcaveHull's frame in float64: PCA of the points (the projection onto the LS plane
            # only moves points along the normal, which the frame's z absorbs)
            q = p.astype(np.float64)
            c = q.mean(0)
            w, V = np.linalg.eigh(np.cov((q - c).T, bias=True))
            xy = (q - c) @ V[:, [2, 1]]
            tri, kept, be, comps, near = alpha_complex(xy, alpha)
            if not near:
                break
        big = max(comps, key=len)
        name = f"c3_{kind}"
        names.append(name)
        out[f"{name}_pts"] = p
        out[f"{name}_normal"] = nrm.astype(np.float32)
        out[f"{name}_alpha"] = np.float64(alpha)
        out[f"{name}_outer"] = np.array(big, np.int32)
    out["names"] = np.array(names)
    np.savez_compressed(os.path.join(HERE, "alpha_shapes.npz"), **out)
    print("written", os.path.join(HERE, "alpha_shapes.npz"), names)


if __name__ == "__main__":
    main()
