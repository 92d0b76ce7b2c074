"""Plane borders (dlg_plane_border): polyPlanes / polyPointCloud (Dialog/PlaneDetect.h:1358-1440)
so the four-file polygon hand-off (PCLViewer.cpp:1341-1396) runs from RANSAC output alone.

The reference's border is polygons[0] of pcl::ConcaveHull (qhull alpha shape, alpha_poly = 0.5,
config.txt); qhull is absent from this image, so the border here is the outer boundary of the
projected points' alpha occupancy -- PARITY UNPINNED: these tests check the contract the
reference's consumers rely on, not qhull's facets:
  * every vertex is one of the plane's points projected as projPoint2Plane projects it (on the
    least-squares plane of pcl::computePointNormal, within float rounding);
  * the polygon is closed, has no repeated vertex, encloses the point set's occupied area (area
    close to the patch's), and is oriented as the reference orients it: the normal of its first
    three vertices points along the given outward normal;
  * an L-shaped plane gets a concave border (area well below its convex hull's).
CPU (host arithmetic, no device); the GPU test runs extract -> borders -> write_polygons ->
read_polygons -> dlg_post_process_planes.
"""
import numpy as np
import pytest

import dialog_amd as D
from dialog_amd.postprocess import plane_border


def frame(n):
    n = np.asarray(n, np.float64)
    n = n / np.linalg.norm(n)
    u = np.cross(n, [1.0, 0, 0] if abs(n[0]) < 0.9 else [0, 1.0, 0])
    u /= np.linalg.norm(u)
    return n, u, np.cross(n, u)


def patch(rng, n, normal, off, shape="square", size=10.0, noise=0.003):
    nrm, u, v = frame(normal)
    st = rng.uniform(0, size, (n * 3, 2))
    if shape == "L":
        st = st[(st[:, 0] < size / 2) | (st[:, 1] < size / 2)]
    st = st[:n]
    p = off * nrm + st[:, :1] * u + st[:, 1:] * v + rng.normal(0, noise, (len(st), 1)) * nrm
    return p.astype(np.float32), nrm, u, v


def area3(b, nrm):
    c = np.zeros(3)
    for k in range(len(b)):
        c += np.cross(b[k].astype(np.float64), b[(k + 1) % len(b)].astype(np.float64))
    return 0.5 * float(np.dot(c, nrm))


@pytest.mark.parametrize("shape,normal,off", [("square", (0.3, -0.5, 0.8), 2.0),
                                              ("square", (0, 0, 1), -3.0),
                                              ("L", (1, 2, -0.5), 0.5)])
def test_border_contract(shape, normal, off):
    rng = np.random.default_rng(hash(shape) % 1000 + int(off * 10))
    p, nrm, u, v = patch(rng, 40000, normal, off, shape)
    b = plane_border(p, nrm, 0.5)
    assert b.shape[0] >= 8
    # vertices: projected plane points (distance to the LS plane ~ float rounding)
    co = D.refit_planes([dict(points=p, border=p[:3], coeff=nrm)])[0]
    d = b.astype(np.float64) @ co[:3].astype(np.float64) + co[3]
    assert np.abs(d).max() < 1e-4
    # every vertex is (the projection of) a distinct plane point
    assert len({tuple(x) for x in b.tolist()}) == b.shape[0]
    # oriented as the reference orients it (the turn of the first three vertices along the
    # outward normal), which here is the polygon's own orientation: counter-clockwise about the
    # outward normal, enclosing the occupied area (signed area ~ the patch's)
    v01, v12 = b[1] - b[0], b[2] - b[1]
    assert np.dot(np.cross(v01, v12), nrm) >= 0
    full = 100.0 if shape == "square" else 75.0
    a = area3(b, nrm)
    assert 0.85 * full < a < 1.1 * full, a
    if shape == "L":
        assert abs(a) < 0.85 * 100.0  # concave: well below the bounding square


def test_border_reversed_normal_reverses_order():
    rng = np.random.default_rng(3)
    p, nrm, _, _ = patch(rng, 20000, (0.2, 0.1, 1.0), 1.0)
    b1 = plane_border(p, nrm, 0.5)
    b2 = plane_border(p, -nrm, 0.5)
    # the same cycle of vertices, traversed the other way round
    r = b1[::-1]
    k = int(np.nonzero((r == b2[0]).all(axis=1))[0][0])
    assert np.array_equal(np.roll(r, -k, axis=0), b2)


def test_border_degenerate():
    assert plane_border(np.zeros((2, 3), np.float32), (0, 0, 1)).shape[0] == 0
    with pytest.raises(Exception):
        plane_border(np.zeros((10, 3), np.float32), (0, 0, 1), alpha=0.0)


@pytest.mark.gpu
def test_gpu_extract_borders_polygon_files_post_process(gpu_ctx, tmp_path):
    """RANSAC output alone drives the hand-off: extract (GPU) -> plane borders -> the four files
    (write_polygons) -> read_polygons -> dlg_post_process_planes absorbs leftover points."""
    from dialog_amd.polyio import read_polygons, write_polygons
    from dialog_amd.postprocess import PostProcessParams, post_process_planes
    from dialog_amd.synth import plane_cloud
    p, lab, planes = plane_cloud(200000, 4, seed=4242, outlier_frac=0.05)
    cl = D.Cloud(gpu_ctx, p)
    e = D.extract_planes(cl, D.make_params(0.02, max_iterations=1023, probability=1.0),
                         max_planes=4, min_inliers=500)
    cl.close()
    assert e["n_planes"] == 4
    offs, inl = e["offsets"], e["inliers"]
    borders, normals = [], []
    for k in range(4):
        pts = p[inl[offs[k]:offs[k + 1]]]
        c = e["coeffs"][k]
        b = plane_border(pts, c[:3], 0.5)
        assert b.shape[0] >= 8
        borders.append(b)
        normals.append(c[:3])
    stem = str(tmp_path / "planes")
    write_polygons(stem + ".pcd", borders, normals, 0.5)
    rb, rn, rs = read_polygons(stem + ".pcd")
    assert len(rb) == 4 and all(np.allclose(a, b) for a, b in zip(rb, borders))
    # post-process: each plane keeps 70 % of its inliers; the rest must come back via the borders
    keep, rest = [], []
    for k in range(4):
        ids = inl[offs[k]:offs[k + 1]]
        keep.append(ids[: int(0.7 * ids.size)])
        rest.append(ids[int(0.7 * ids.size):])
    # (the plane points are copies of cloud points, as in the reference: each marks itself)
    planes_in = [dict(points=p[keep[k]], border=rb[k], coeff=np.append(rn[k], 0.0))
                 for k in range(4)]
    co, absorbed, remaining = post_process_planes(p, planes_in,
                                                  PostProcessParams(0.1, 0.1, 500, 0, 12345),
                                                  ctx=gpu_ctx)
    for k in range(4):
        assert np.dot(co[k][:3], rn[k]) > 0.99
        got = np.intersect1d(absorbed[k], rest[k]).size
        assert got >= 0.9 * rest[k].size, (k, got, rest[k].size)
