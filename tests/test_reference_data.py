"""The reference's own data files as fixtures (tests/golden/import_reference_data.py copied them):

* Dialog/dataForPlane/{source,target}_plane_registration.{pcd,txt} -- real plane-border polygons
  (the plane stage's hand-off output, read by Registration.h:356-420): the reader's polygon split,
  and the postProcessPlanes absorption (isPointInPoly over these concave many-vertex borders) on
  the GPU against the oracle, bit for bit;
* Dialog/result_pcd/filed_OM.pcd -- a real 147,486-point scan: GPU segment / extract-and-remove
  (PCL and fast refit), preProcess, normals and RegulateNormal against the oracle, bit for bit.

The reference holds no RANSAC outputs, so these pin the GPU path to the oracle on real geometry;
the PCL arithmetic itself stays "parity unpinned" (DESIGN.md §2).
"""
import os

import numpy as np
import pytest

from oracle import oracle as O

HERE = os.path.dirname(os.path.abspath(__file__))
DFP = os.path.join(HERE, "golden", "dataForPlane")


def polygons(side):
    from dialog_amd.polyio import read_polygon_pair
    return read_polygon_pair(os.path.join(DFP, f"{side}_plane_registration.pcd"),
                             os.path.join(DFP, f"{side}_plane_registration.txt"))


def filed_om():
    return np.load(os.path.join(HERE, "golden", "filed_OM.npz"))["points"]


# ---------------------------------------------------------------------------------------------
# CPU: the reader and the oracle on the real borders

@pytest.mark.parametrize("side,sizes", [
    ("source", [337, 194, 242, 182, 229, 154, 124, 212, 120, 89, 77]),
    ("target", [315, 213, 239, 162, 246, 128, 188, 199, 87, 112, 74]),
])
def test_polygon_pair_split(side, sizes):
    polys = polygons(side)
    assert [p.shape[0] for p in polys] == sizes
    from dialog_amd.pcd import read_pcd
    allv = read_pcd(os.path.join(DFP, f"{side}_plane_registration.pcd"))
    assert np.array_equal(np.concatenate(polys), allv)
    for p in polys:  # each border lies in a plane (ConcaveHull of projected inliers)
        c = p.astype(np.float64).mean(0)
        w = np.linalg.eigvalsh(np.cov((p - c).T))
        assert w[0] < 1e-6 * w[2]


def test_polygon_pair_malformed(tmp_path):
    from dialog_amd.pcd import write_pcd_ascii
    from dialog_amd.polyio import read_polygon_pair
    pcd = str(tmp_path / "v.pcd")
    write_pcd_ascii(pcd, np.zeros((10, 3), np.float32))
    (tmp_path / "ok.txt").write_text("4\n6\n99\n")  # later entries are never read
    assert [p.shape[0] for p in read_polygon_pair(pcd, str(tmp_path / "ok.txt"))] == [4, 6]
    (tmp_path / "short.txt").write_text("4\n3\n")
    with pytest.raises(ValueError):
        read_polygon_pair(pcd, str(tmp_path / "short.txt"))
    (tmp_path / "over.txt").write_text("4\n7\n")
    with pytest.raises(ValueError):
        read_polygon_pair(pcd, str(tmp_path / "over.txt"))


def plane_frame(border):
    b = border.astype(np.float64)
    c = b.mean(0)
    w, v = np.linalg.eigh(np.cov((b - c).T))
    n = v[:, 0]
    u = (b[0] - c) / np.linalg.norm(b[0] - c)
    u = u - (u @ n) * n
    u /= np.linalg.norm(u)
    return c, n, u, np.cross(n, u)


def even_odd(q2, poly2):
    x, y = q2[:, 0:1], q2[:, 1:2]
    a, b = poly2, np.roll(poly2, -1, axis=0)
    cond = (a[:, 1] > y) != (b[:, 1] > y)
    xi = a[:, 0] + (y - a[:, 1]) * (b[:, 0] - a[:, 0]) / np.where(b[:, 1] != a[:, 1],
                                                                   b[:, 1] - a[:, 1], 1.0)
    return (np.sum(cond & (x < xi), axis=1) % 2) == 1


def border_scene(side, per_poly=1500, seed=0, keep=0.6):
    """A cloud sampled on each real border's plane (inside and around the polygon, N(0, 5 mm)
    off-plane), each plane's points_set = `keep` of its inside samples (cloud points)."""
    rng = np.random.default_rng(seed)
    clouds, planes, info = [], [], []
    base = 0
    for k, b in enumerate(polygons(side)):
        c, n, u, v = plane_frame(b)
        b2 = np.c_[(b - c) @ u, (b - c) @ v]
        lo, hi = b2.min(0), b2.max(0)
        pad = 0.1 * (hi - lo)
        st = rng.uniform(lo - pad, hi + pad, (per_poly, 2))
        q = (c + st[:, :1] * u + st[:, 1:] * v + rng.normal(0, 0.005, (per_poly, 1)) * n)
        q = q.astype(np.float32)
        inside = even_odd(st, b2)
        idx = np.flatnonzero(inside)
        keep_idx = idx[rng.random(idx.size) < keep]
        clouds.append(q)
        planes.append(dict(coeff=np.r_[n, -n @ c].astype(np.float32), points=q[keep_idx],
                           border=b))
        info.append((base, st, b2))
        base += per_poly
    return np.concatenate(clouds), planes, info


def test_oracle_point_in_poly_on_real_borders():
    """The oracle's 10-ray vote (isPointInPoly, PlaneDetect.h:1891-1964) agrees with exact
    even-odd containment on the reference's concave borders, away from the border."""
    rng = np.random.default_rng(1)
    for b in polygons("source")[:4]:
        c, n, u, v = plane_frame(b)
        b2 = np.c_[(b - c) @ u, (b - c) @ v]
        lo, hi = b2.min(0), b2.max(0)
        st = rng.uniform(lo, hi, (150, 2))
        q = (c + st[:, :1] * u + st[:, 1:] * v).astype(np.float32)
        a, bb = b2, np.roll(b2, -1, axis=0)
        ab = bb - a
        t = np.clip(((st[:, None, :] - a) * ab).sum(-1) / (ab * ab).sum(-1), 0, 1)
        dd = st[:, None, :] - (a + t[..., None] * ab)
        far = np.sqrt((dd * dd).sum(-1)).min(1) > 0.02
        coeff = np.r_[n, -n @ c].astype(np.float32)
        got = np.array([O.is_point_in_poly(x, coeff, b, 0.1, 4242) for x in q])
        assert np.array_equal(got[far], even_odd(st, b2)[far])


# ---------------------------------------------------------------------------------------------
# GPU: post-process on the real borders; the RANSAC path, preProcess and normals on filed_OM

@pytest.mark.gpu
@pytest.mark.parametrize("side,seed", [("source", 0), ("target", 1)])
def test_gpu_post_process_real_borders(gpu_ctx, side, seed):
    import dialog_amd as D
    cloud, planes, _ = border_scene(side, seed=seed)
    prm = D.PostProcessParams(0.1, 0.05, 10, 0, 1700000000 + seed)
    g = D.post_process_planes(cloud, planes, prm, ctx=gpu_ctx)
    co = np.array([np.r_[p["coeff"][:3], 0.0] for p in planes], np.float32)
    o = O.post_process_planes(cloud, co, [p["points"] for p in planes],
                              [p["border"] for p in planes], 0.1, 0, 1700000000 + seed, 0.05, 10)
    assert np.array_equal(g[0].view(np.uint32), o[0].view(np.uint32))
    assert len(g[1]) == len(o[1]) == len(planes)
    for a, b in zip(g[1], o[1]):
        assert np.array_equal(a, b)
    assert np.array_equal(g[2], o[2])
    assert sum(a.size for a in g[1]) > 1000  # the borders did absorb points


@pytest.mark.gpu
@pytest.mark.parametrize("refit", ["pcl", "fast"])
def test_gpu_filed_om_extract(gpu_ctx, refit):
    """Extract-and-remove on the real scan (PCL-default-like RANSAC budget and the C3 budget)."""
    import dialog_amd as D
    p = filed_om()
    mode = D.DLG_REFIT_PCL if refit == "pcl" else D.DLG_REFIT_FAST
    for thr, kw in ((0.05, dict(max_iterations=50, probability=0.99)),
                    (0.02, dict(max_iterations=4095, probability=1.0))):
        cloud = D.Cloud(gpu_ctx, p)
        e = D.extract_planes(cloud, D.make_params(thr, refit_mode=mode, **kw), max_planes=12,
                             min_inliers=200)
        cloud.close()
        r = O.extract_planes(p, thr, max_planes=12, min_inliers=200, refit=refit, **kw)
        assert e["n_planes"] == r["n_planes"] >= 3
        assert np.array_equal(e["coeffs"].view(np.uint32), r["coeffs"].view(np.uint32))
        assert np.array_equal(e["offsets"], r["offsets"])
        assert np.array_equal(e["inliers"], r["inliers"])


@pytest.mark.gpu
def test_gpu_filed_om_segment(gpu_ctx):
    import dialog_amd as D
    p = filed_om()
    for thr, kw in ((0.005, dict()), (0.02, dict(max_iterations=1023, probability=1.0))):
        r = O.sac_segment(p, thr, **kw)
        cloud = D.Cloud(gpu_ctx, p)
        inl, coeff, st = D.segment_cloud(cloud, D.make_params(thr, **kw))
        cloud.close()
        assert st["iterations"] == r["iterations"] and st["draws"] == r["draws"]
        assert list(st["best_sample"]) == list(r["best_sample"])
        assert np.array_equal(coeff.view(np.uint32), r["coeff"].view(np.uint32))
        assert np.array_equal(inl, r["inliers"])


@pytest.mark.gpu
def test_gpu_filed_om_preprocess(gpu_ctx):
    """preProcess (PlaneDetect.h:448-512) with the reference's min_dist_between_points
    (config.txt:3, 0.001) and a coarser 0.02."""
    import dialog_amd as D
    p = filed_om()
    for md in (0.001, 0.02):
        xyz, idx, tr = D.preprocess(p, md, ctx=gpu_ctx)
        oxyz, oidx, otr = O.preprocess(p, md)
        assert np.array_equal(idx, oidx)
        assert np.array_equal(xyz.view(np.uint32), oxyz.view(np.uint32))
        assert np.array_equal(np.asarray(tr, np.float32).view(np.uint32),
                              np.asarray(otr, np.float32).view(np.uint32))


@pytest.mark.gpu
def test_gpu_filed_om_regulate(gpu_ctx):
    """RegulateNormal BFS on the real scan from the oracle's normals (radius r_for_estimate_normal
    / r_for_regulate_normal of config.txt scaled to this scan's spacing)."""
    import dialog_amd as D
    p = filed_om()
    nrm = O.estimate_normals(p, 0.1)
    reg, proc, n = D.regulate_normals(p, nrm, 0, False, 0.08, ctx=gpu_ctx)
    oreg, oproc, on = O.regulate_normals(p, nrm, 0, False, 0.08)
    assert n == on > 1000
    assert np.array_equal(proc.astype(bool), oproc.astype(bool))
    assert np.array_equal(reg[:, :3].view(np.uint32), oreg[:, :3].view(np.uint32))
