"""Plane borders (dlg_plane_border): polyPlanes / polyPointCloud (Dialog/PlaneDetect.h:1358-1440)
so the four-file polygon hand-off (PCLViewer.cpp:1341-1396) runs from RANSAC output alone.

The reference's border is polygons[0] of pcl::ConcaveHull (qhull "d QJ" Delaunay + alpha test,
alpha_poly = 0.5, config.txt).  dialog_amd/csrc/alpha_shape.hpp restates ConcaveHull's steps with
its own Delaunay triangulation; these tests pin it to qhull itself (scipy.spatial.Delaunay with
"QJ", committed fixtures tests/golden/alpha_shapes.npz from tests/golden/make_alpha.py):
  * the triangulation equals qhull's triangle for triangle (points in general position), the
    alpha filter keeps the same triangles, and the boundary edges and their components (PCL's
    polygons, as vertex sets) are qhull's;
  * on 3-D plane patches, dlg_plane_border's vertices are exactly the fixture's outer-boundary
    vertex set (each vertex mapped back to its plane point);
  * the contract the reference's consumers rely on: vertices on the least-squares plane, a closed
    polygon without repeated vertices enclosing the patch's area, the reference's orientation
    rule, a concave border for an L-shaped patch.
Parity unpinned: qhull's version and joggle seed, the facet order that decides where PCL's walk
starts and which polygon is polygons[0] (the border here is the largest polygon), and qhull's
joggled output coordinates.
CPU (host arithmetic, no device); the GPU test runs extract -> borders -> write_polygons ->
read_polygons -> dlg_post_process_planes.
"""
import ctypes
import os
import subprocess

import numpy as np
import pytest

import dialog_amd as D
from dialog_amd.postprocess import plane_border

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLD = os.path.join(ROOT, "tests", "golden", "alpha_shapes.npz")
VP = ctypes.c_void_p


@pytest.fixture(scope="module")
def ah(tmp_path_factory):
    so = tmp_path_factory.mktemp("alpha") / "libalpha_host.so"
    subprocess.run(["g++", "-std=c++17", "-O2", "-ffp-contract=off", "-shared", "-fPIC",
                    os.path.join(ROOT, "tests", "cpp", "alpha_host.cpp"), "-o", str(so)], check=True)
    L = ctypes.CDLL(str(so))
    L.alpha_delaunay.restype = ctypes.c_int64
    L.alpha_boundary.restype = ctypes.c_int64
    return L


def delaunay(L, xy):
    xy = np.ascontiguousarray(xy, np.float64)
    out = np.zeros((2 * xy.shape[0] + 8, 3), np.int32)
    nt = L.alpha_delaunay(VP(xy.ctypes.data), ctypes.c_int64(xy.shape[0]), VP(out.ctypes.data),
                          ctypes.c_int64(out.shape[0]))
    assert nt <= out.shape[0]
    return out[:nt]


def boundary(L, xy, alpha):
    xy = np.ascontiguousarray(xy, np.float64)
    n = xy.shape[0]
    kept = np.zeros(2 * n + 8, np.uint8)
    verts, order, poly = (np.zeros(n + 1, np.int32) for _ in range(3))
    nv = L.alpha_boundary(VP(xy.ctypes.data), ctypes.c_int64(n), ctypes.c_double(alpha),
                          VP(kept.ctypes.data), ctypes.c_int64(kept.size), VP(verts.ctypes.data),
                          VP(order.ctypes.data), VP(poly.ctypes.data), ctypes.c_int64(n + 1))
    nt = delaunay(L, xy).shape[0]
    polys = {}
    for v, pid in zip(order[:nv], poly[:nv]):
        if pid >= 0:
            polys.setdefault(int(pid), []).append(int(v))
    return kept[:nt].astype(bool), verts[:nv], [polys[k] for k in sorted(polys)]


def sorted_tris(t):
    t = np.sort(t, axis=1)
    return t[np.lexsort((t[:, 2], t[:, 1], t[:, 0]))]


def names(prefix):
    z = np.load(GOLD)
    return [str(x) for x in z["names"] if str(x).startswith(prefix)]


@pytest.mark.parametrize("name", names("c2_"))
def test_alpha_shape_equals_qhull_fixture(ah, name):
    """Triangles, alpha filter, boundary edges and boundary components equal qhull's (scipy
    Delaunay "QJ") on the committed fixtures: square, L, annulus (a hole), two blobs, graded
    density."""
    z = np.load(GOLD)
    xy, alpha = z[f"{name}_xy"], float(z[f"{name}_alpha"])
    tri = delaunay(ah, xy)
    st = sorted_tris(tri)
    assert np.array_equal(st, z[f"{name}_tri"])
    kept, verts, polys = boundary(ah, xy, alpha)
    order = np.lexsort((np.sort(tri, 1)[:, 2], np.sort(tri, 1)[:, 1], np.sort(tri, 1)[:, 0]))
    assert np.array_equal(kept[order], z[f"{name}_kept"])
    # boundary edges: the kept triangles' edges not shared with another kept triangle
    cnt = {}
    for t in tri[kept]:
        for i in range(3):
            e = tuple(sorted((int(t[i]), int(t[(i + 1) % 3]))))
            cnt[e] = cnt.get(e, 0) + 1
    be = sorted(e for e, k in cnt.items() if k == 1)
    assert be == [tuple(e) for e in z[f"{name}_bedges"].tolist()]
    sizes, cv = z[f"{name}_comp_sizes"], z[f"{name}_comp_verts"]
    comps = [frozenset(x.tolist()) for x in np.split(cv, np.cumsum(sizes)[:-1])]
    assert set(verts.tolist()) == set(cv.tolist())
    deg = {}
    for a, b in be:
        deg[a] = deg.get(a, 0) + 1
        deg[b] = deg.get(b, 0) + 1
    if max(deg.values()) == 2:  # simple boundaries: PCL's walk yields exactly the components
        assert {frozenset(p) for p in polys} == set(comps)
        for p in polys:  # consecutive walk vertices are boundary edges
            for k in range(len(p)):
                assert tuple(sorted((p[k], p[(k + 1) % len(p)]))) in cnt


def delaunay_valid(xy, tri):
    """every triangle counter-clockwise and no point strictly inside its circumcircle"""
    a, b, c = xy[tri[:, 0]], xy[tri[:, 1]], xy[tri[:, 2]]
    o = (b[:, 0] - a[:, 0]) * (c[:, 1] - a[:, 1]) - (b[:, 1] - a[:, 1]) * (c[:, 0] - a[:, 0])
    assert (o > 0).all()
    for k in range(tri.shape[0]):
        rows = []
        for v in (a[k], b[k], c[k]):
            d = v[None, :] - xy
            rows.append((d[:, 0], d[:, 1], d[:, 0] ** 2 + d[:, 1] ** 2))
        (ax, ay, al), (bx, by, bl), (cx, cy, cl) = rows
        det = ax * (by * cl - bl * cy) - ay * (bx * cl - bl * cx) + al * (bx * cy - by * cx)
        scale = (np.abs(ax) + np.abs(ay) + 1e-300) ** 4
        assert (det <= 1e-9 * scale.max()).all(), k


@pytest.mark.parametrize("case", ["random", "grid", "collinear", "duplicates", "tiny", "far"])
def test_delaunay_degenerate_inputs(ah, case):
    """Degenerate inputs (cocircular grids, collinear sets, duplicates, tiny / offset coordinates)
    triangulate without error into a valid Delaunay triangulation (for general-position input:
    qhull's, live through scipy)."""
    from scipy.spatial import Delaunay
    rng = np.random.default_rng(11)
    if case == "random":
        xy = rng.uniform(-3, 3, (1500, 2))
    elif case == "grid":
        g = np.arange(20.0)
        xy = np.stack(np.meshgrid(g, g), -1).reshape(-1, 2)
    elif case == "collinear":  # exactly collinear (integer coordinates): no triangle
        t = rng.permutation(200).astype(np.float64)
        xy = np.stack([t, 2 * t + 1], 1)
    elif case == "duplicates":
        xy = np.repeat(rng.uniform(0, 1, (300, 2)), 3, axis=0)
    elif case == "tiny":
        xy = rng.uniform(0, 1e-6, (500, 2))
    else:
        xy = rng.uniform(0, 1, (500, 2)) + 1e4
    tri = delaunay(ah, xy)
    if case == "collinear":
        assert tri.shape[0] == 0
        return
    delaunay_valid(xy, tri)
    if case in ("random", "tiny", "far"):
        # (qhull's joggle scales with the coordinates' magnitude: far from the origin it flips
        # near-cocircular pairs, so qhull is run on the centred points -- ConcaveHull demeans
        # before qhull as well)
        d = Delaunay(xy - xy.mean(0), qhull_options="QJ")
        assert np.array_equal(sorted_tris(tri), sorted_tris(d.simplices))
    if case == "duplicates":  # each distinct point used once
        assert np.unique(xy[np.unique(tri)], axis=0).shape[0] == np.unique(tri).size


@pytest.mark.parametrize("name", names("c3_"))
def test_plane_border_vertex_set_pinned(name):
    """dlg_plane_border on 3-D plane patches: its vertices, mapped back to the plane points, are
    exactly the outer boundary of qhull's alpha shape (fixture)."""
    z = np.load(GOLD)
    p, nrm, alpha = z[f"{name}_pts"], z[f"{name}_normal"], float(z[f"{name}_alpha"])
    b = plane_border(p, nrm, alpha)
    q = p.astype(np.float64)
    c = q.mean(0)
    _, V = np.linalg.eigh(np.cov((q - c).T, bias=True))
    pq, bq = (q - c) @ V[:, [2, 1]], (b.astype(np.float64) - c) @ V[:, [2, 1]]
    d2 = ((bq[:, None, :] - pq[None, :, :]) ** 2).sum(-1)
    idx = d2.argmin(1)
    assert np.sqrt(d2[np.arange(len(idx)), idx]).max() < 1e-4
    assert len(set(idx.tolist())) == len(idx)
    assert set(idx.tolist()) == set(z[f"{name}_outer"].tolist())


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


def _outer_vertex_set(pts, alpha):
    """The fixture logic of make_alpha.py for one plane: ConcaveHull's PCA frame in float64, qhull
    ("QJ") Delaunay, the alpha filter, the largest boundary component's vertex set."""
    import sys
    sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
    from make_alpha import alpha_complex
    q = pts.astype(np.float64)
    c = q.mean(0)
    _, V = np.linalg.eigh(np.cov((q - c).T, bias=True))
    xy = (q - c) @ V[:, [2, 1]]
    _, _, _, comps, near = alpha_complex(xy, alpha)
    return set(max(comps, key=len)), near, xy, c, V


def _patch_cloud():
    """Two plane patches of the fixtures' kinds (a square and an L), far enough from each other's
    planes that RANSAC's inliers of one never reach into the other, plus sparse outliers."""
    rng = np.random.default_rng(2024)
    a, na, _, _ = patch(rng, 6000, (0.3, -0.5, 0.8), 2.0, "square")
    b, nb, _, _ = patch(rng, 8000, (1, 2, -0.5), 0.5, "L")
    b = b + (20.0 * na).astype(np.float32)  # (B's plane stays B's: shifted along A's normal)
    out = rng.uniform(-15, 25, (100, 3)).astype(np.float32)
    return np.vstack([a, b, out]).astype(np.float32)


@pytest.mark.gpu
def test_cpp_poly_planes_on_ransac_planes(tmp_path):
    """the reference's polyPlanes() with dialog::polyPlanes (the shim's
    polyPointCloud over dlg_plane_border) in place of pcl::ConcaveHull, compiled as a C++ adapter
    with the reference's struct Plane, on planes RANSAC extracted on the GPU.  Every border's
    vertices are distinct points of its plane's projected points_set, and they are exactly the
    outer boundary of qhull's alpha shape of those points (test_plane_border_vertex_set_pinned's
    fixture logic, computed here with scipy's qhull); a second polyPlanes() call keeps them."""
    lib = os.path.dirname(D.LIB_PATH)
    exe = tmp_path / "poly_planes_glue"
    subprocess.run(["g++", "-std=c++17", "-O1", "-I", os.path.join(ROOT, "include"),
                    os.path.join(ROOT, "tests", "cpp", "poly_planes_glue.cpp"), "-o", str(exe),
                    "-L", lib, "-ldialog_amd", f"-Wl,-rpath,{lib}"], check=True)
    cloud = _patch_cloud()
    fin, fout = tmp_path / "cloud.bin", tmp_path / "planes.bin"
    cloud.tofile(fin)
    r = subprocess.run([str(exe), str(fin), str(fout)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, (r.stdout, r.stderr)
    assert r.stdout.strip() == "planes 2 built 2 again 0", r.stdout
    raw = fout.read_bytes()
    off = 0

    def take():
        nonlocal off
        k = int(np.frombuffer(raw, np.int64, 1, off)[0])
        off += 8
        a = np.frombuffer(raw, np.float32, 3 * k, off).reshape(k, 3)
        off += 12 * k
        return a

    assert int(np.frombuffer(raw, np.int64, 1, 0)[0]) == 2
    off = 8
    for _ in range(2):
        pts, border = take(), take()
        assert pts.shape[0] > 5000 and border.shape[0] >= 8
        want, near, xy, c, V = _outer_vertex_set(pts, 0.5)
        assert not near  # (no circumradius within 1e-9 of alpha: the filter is decided)
        bq = (border.astype(np.float64) - c) @ V[:, [2, 1]]
        d2 = ((bq[:, None, :] - xy[None, :, :]) ** 2).sum(-1)
        idx = d2.argmin(1)
        assert np.sqrt(d2[np.arange(len(idx)), idx]).max() < 1e-4
        assert len(set(idx.tolist())) == len(idx)
        assert set(idx.tolist()) == want
