"""Normals path: estimateNormal() (PlaneDetect.h:515-545, radius; PCLViewer.cpp:507-522, k = 20)
and regulateNormal() (PlaneDetect.h:547-665).

CPU tests pin the oracle (oracle/pcl_oracle.c) against an independent float64 numpy restatement
and the committed fixture; GPU tests compare libdialog_amd.so against both:
  * neighbour sets are exact (same float d2 test as KdTreeFLANN): the NaN mask (< 3 neighbours)
    must match the oracle exactly;
  * normals / curvature, mode "pcl" (the default, PCL's float arithmetic: single-pass float sums
    over the (d2, index)-ordered neighbours, eigen33 in float): bit-exact with the oracle, for
    radius neighbourhoods of every size class of the device sort (<= 64 ... > 1024) and k-NN;
  * mode "double" (centred double moments): the float64 restatement at 1e-5 rad / 1e-5 relative
    curvature where the eigenproblem is well conditioned;
  * RegulateNormal is bit-exact: same processed set, same count, identical normals.
"""
import json
import os

import numpy as np
import pytest
from scipy.spatial import cKDTree

from oracle import oracle as O

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")

RADIUS = 0.1


def small_cloud(n=12000, seed=7, planes=3, patch=2.0, outliers=0.05):
    from dialog_amd.synth import plane_cloud
    return plane_cloud(n, planes, outlier_frac=outliers, seed=seed, patch=patch)


def flann_radius_sets(p, r):
    """exact KdTreeFLANN radius sets: float d2 = ((0 + dx^2) + dy^2) + dz^2 < float(r*r)."""
    r2 = np.float32(float(r) * float(r))
    tree = cKDTree(p.astype(np.float64))
    cand = tree.query_ball_point(p.astype(np.float64), r * 1.001)
    out = []
    for i, c in enumerate(cand):
        c = np.asarray(c, np.int64)
        d = p[i][None, :] - p[c]
        d2 = ((np.float32(0) + d[:, 0] * d[:, 0]) + d[:, 1] * d[:, 1]) + d[:, 2] * d[:, 2]
        out.append(np.sort(c[d2 < r2]))
    return out


def knn_sets(p, k):
    """FLANN kNN sets: the k smallest (float d2, index) among the points (query included)."""
    tree = cKDTree(p.astype(np.float64))
    _, cand = tree.query(p.astype(np.float64), k=min(k + 8, len(p)))
    out = []
    for i, c in enumerate(cand):
        d = p[i][None, :] - p[c]
        d2 = ((np.float32(0) + d[:, 0] * d[:, 0]) + d[:, 1] * d[:, 1]) + d[:, 2] * d[:, 2]
        o = np.lexsort((c, d2))[:k]
        out.append(np.sort(c[o]))
    return out


def f64_normals(p, sets, vp=(0.0, 0.0, 0.0)):
    """float64 restatement: covariance, eigh, curvature, viewpoint flip; + eigen-gap quality."""
    n = p.shape[0]
    out = np.full((n, 4), np.nan)
    gap = np.zeros(n)
    P = p.astype(np.float64)
    for i, s in enumerate(sets):
        if len(s) < 3:
            continue
        q = P[s]
        c = np.cov(q.T, bias=True)
        w, v = np.linalg.eigh(c)
        nv = v[:, 0]
        if np.dot(np.asarray(vp) - P[i], nv) < 0:
            nv = -nv
        tr = w.sum()
        out[i, :3] = nv
        out[i, 3] = abs(w[0] / tr) if tr != 0 else 0.0
        gap[i] = (w[1] - w[0]) / max(w[2], 1e-300)
    return out, gap


def angle(a, b):
    """unsigned angle between the lines of two normal sets, robust near 0 (float32 unit vectors
    are only unit to ~6e-8, which arccos of the dot product would turn into ~3e-4 rad)."""
    a = a[:, :3].astype(np.float64)
    b = b[:, :3].astype(np.float64)
    return np.arctan2(np.linalg.norm(np.cross(a, b), axis=1), np.abs(np.sum(a * b, axis=1)))


# ------------------------------------------------------------------------------------- CPU tests
def test_oracle_radius_normals_match_f64_restatement():
    p, _, _ = small_cloud(4000)
    o = O.estimate_normals(p, RADIUS)
    sets = flann_radius_sets(p, RADIUS)
    ref, gap = f64_normals(p, sets)
    assert np.array_equal(np.isnan(o[:, 0]), np.isnan(ref[:, 0]))
    ok = ~np.isnan(ref[:, 0]) & (gap > 1e-2)
    a = angle(o[ok], ref[ok])
    assert np.percentile(a, 99) < 2e-3 and a.max() < 2e-2
    # flip towards the origin agrees wherever the direction is not ~perpendicular to the view ray
    s = np.sign(np.sum(o[ok, :3] * ref[ok, :3], axis=1))
    view = np.abs(np.sum(-p[ok] * ref[ok, :3], axis=1)) / np.linalg.norm(p[ok], axis=1)
    assert np.all(s[view > 1e-2] > 0)


def test_oracle_knn_normals_match_f64_restatement():
    p, _, _ = small_cloud(3000, seed=11)
    o = O.estimate_normals_knn(p, 20)
    ref, gap = f64_normals(p, knn_sets(p, 20))
    ok = gap > 1e-2
    a = angle(o[ok], ref[ok])
    assert np.percentile(a, 99) < 2e-3 and a.max() < 2e-2
    assert not np.isnan(o).any()


def test_oracle_regulate_is_bfs_over_radius_graph():
    """processed set = connected component of the seed in the r-graph (PlaneDetect.h:620-640)."""
    p, _, _ = small_cloud(3000, seed=5)
    nrm = O.estimate_normals(p, RADIUS)
    reg, proc, cnt = O.regulate_normals(p, nrm, 17, True, 0.08)
    sets = flann_radius_sets(p, 0.08)
    seen = np.zeros(len(p), bool)
    seen[17] = True
    st = [17]
    while st:
        u = st.pop()
        for v in sets[u]:
            if not seen[v]:
                seen[v] = True
                st.append(v)
    assert np.array_equal(proc, seen) and cnt == seen.sum()
    # untouched points keep their normals; touched ones only change sign
    assert np.array_equal(reg[~proc], nrm[~proc], equal_nan=True)
    same = np.all(reg[:, :3] == nrm[:, :3], axis=1) | np.all(reg[:, :3] == -nrm[:, :3], axis=1)
    assert np.all(same | np.isnan(nrm[:, 0]))


def test_oracle_normals_fixture():
    path = os.path.join(GOLDEN, "normals_small.npz")
    f = np.load(path)
    p = f["points"]
    np.testing.assert_array_equal(O.estimate_normals(p, float(f["radius"])), f["radius_normals"])
    np.testing.assert_array_equal(O.estimate_normals_knn(p, int(f["k"])), f["knn_normals"])
    reg, proc, cnt = O.regulate_normals(p, f["radius_normals"], int(f["seed_idx"]), False,
                                        float(f["r_regulate"]))
    np.testing.assert_array_equal(reg, f["regulated"])
    np.testing.assert_array_equal(proc, f["processed"])


# ------------------------------------------------------------------------------------- GPU tests
@pytest.fixture(scope="module")
def cloud():
    return small_cloud(12000, seed=3)


@pytest.mark.gpu
def test_gpu_radius_normals(gpu_ctx, cloud):
    import dialog_amd as D
    p, _, _ = cloud
    g = D.estimate_normals(p, radius=RADIUS, ctx=gpu_ctx, mode="double")
    o = O.estimate_normals(p, RADIUS)
    assert np.array_equal(np.isnan(g[:, 0]), np.isnan(o[:, 0]))  # exact neighbour counts
    ref, gap = f64_normals(p, flann_radius_sets(p, RADIUS))
    ok = ~np.isnan(ref[:, 0]) & (gap > 1e-3)
    a = angle(g[ok], ref[ok])
    assert a.max() < 1e-5, a.max()
    np.testing.assert_allclose(g[ok, 3], ref[ok, 3], rtol=1e-4, atol=1e-7)
    # same viewpoint-flip decision as the float64 restatement (away from perpendicular views)
    s = np.sum(g[ok, :3] * ref[ok, :3], axis=1)
    view = np.abs(np.sum(-p[ok] * ref[ok, :3], axis=1)) / np.linalg.norm(p[ok], axis=1)
    assert np.all(s[view > 1e-3] > 0)
    # and against the PCL-float oracle at the float-cancellation bound
    ok2 = ~np.isnan(o[:, 0]) & (gap > 1e-2)
    a2 = angle(g[ok2], o[ok2])
    assert np.percentile(a2, 99) < 2e-3 and a2.max() < 2e-2


@pytest.mark.gpu
def test_gpu_knn_normals(gpu_ctx, cloud):
    import dialog_amd as D
    p, _, _ = cloud
    for k in (3, 20, 64):
        g = D.estimate_normals(p, k=k, ctx=gpu_ctx, mode="double")
        ref, gap = f64_normals(p, knn_sets(p, k))
        ok = gap > 1e-3
        assert not np.isnan(g).any()
        a = angle(g[ok], ref[ok])
        assert a.max() < 1e-5, (k, a.max())
        np.testing.assert_allclose(g[ok, 3], ref[ok, 3], rtol=1e-4, atol=1e-7)
    o = O.estimate_normals_knn(p[:3000], 20)
    g = D.estimate_normals(p[:3000], k=20, ctx=gpu_ctx, mode="double")
    _, gap = f64_normals(p[:3000], knn_sets(p[:3000], 20))
    ok = gap > 1e-2
    a = angle(g[ok], o[ok])
    assert np.percentile(a, 99) < 2e-3


@pytest.mark.gpu
@pytest.mark.parametrize("n,patch,r,seed", [
    (12000, 2.0, 0.1, 3),     # ~30 neighbours: one-register sort
    (12000, 2.0, 0.2, 4),     # ~100-200: 2-4 keys per lane
    (6000, 1.0, 0.3, 5),      # ~500-1000: 8-16 keys per lane
    (3000, 0.5, 0.45, 6),     # > 1024 neighbours: the heapsort path
])
def test_gpu_radius_normals_pcl_bit_exact(gpu_ctx, n, patch, r, seed):
    """PCL-float mode (dlg_estimate_normals): bit-identical to the oracle's computePointNormal
    restatement, NaN mask included, viewpoint flip included."""
    import dialog_amd as D
    p, _, _ = small_cloud(n, seed=seed, patch=patch)
    p[::97] = np.nan
    for vp in ((0.0, 0.0, 0.0), (3.0, -1.0, 2.0)):
        g = D.estimate_normals(p, radius=r, viewpoint=vp, ctx=gpu_ctx)
        o = O.estimate_normals(p, r, viewpoint=vp)
        assert np.array_equal(np.isnan(g), np.isnan(o))
        ok = ~np.isnan(o[:, 0])
        assert np.array_equal(g[ok].view(np.uint32), o[ok].view(np.uint32)), \
            int((g[ok] != o[ok]).any(axis=1).sum())


@pytest.mark.gpu
def test_gpu_radius_normals_fused_ties_and_chunked(gpu_ctx):
    """The fused radius pass (DLG_OPT_NORMALS_FUSED = 1, default) on a quantised cloud, where
    many neighbours tie in d2 and FLANN's order falls back to the point index: bit-identical to
    the oracle; and on a larger cloud bit-identical to the chunked pipeline (option 0)."""
    import dialog_amd as D
    p, _, _ = small_cloud(8000, seed=21, patch=1.5)
    q = (np.round(p * 64) / 64).astype(np.float32)
    g = D.estimate_normals(q, radius=0.12, ctx=gpu_ctx)
    o = O.estimate_normals(q, 0.12)
    assert np.array_equal(np.isnan(g), np.isnan(o))
    ok = ~np.isnan(o[:, 0])
    assert np.array_equal(g[ok].view(np.uint32), o[ok].view(np.uint32))
    big, _, _ = small_cloud(200000, seed=22, patch=6.0)
    ctx = D.Context(0)
    try:
        f = D.estimate_normals(big, radius=0.1, ctx=ctx)
        ctx.set_option(D.DLG_OPT_NORMALS_FUSED, 0)
        c = D.estimate_normals(big, radius=0.1, ctx=ctx)
    finally:
        ctx.close()
    assert np.array_equal(np.isnan(f), np.isnan(c))
    ok = ~np.isnan(c[:, 0])
    assert np.array_equal(f[ok].view(np.uint32), c[ok].view(np.uint32))


@pytest.mark.gpu
@pytest.mark.parametrize("k", [3, 20, 33, 64])
def test_gpu_knn_normals_pcl_bit_exact(gpu_ctx, k):
    """k-NN normals bit for bit, with sparse outliers that defer to coarser levels."""
    import dialog_amd as D
    p, _, _ = small_cloud(3000, seed=9)
    rng = np.random.default_rng(19)
    far = rng.uniform(-6.0, 6.0, size=(300, 3)).astype(np.float32)
    p = np.concatenate([p, far])
    o = O.estimate_normals_knn(p, k)
    g = D.estimate_normals(p, k=k, ctx=gpu_ctx)
    assert np.array_equal(g.view(np.uint32), o.view(np.uint32)), int((g != o).any(axis=1).sum())


@pytest.mark.gpu
def test_gpu_normals_pcl_layout_viewpoint_and_edges(gpu_ctx, cloud):
    import dialog_amd as D
    p, _, _ = cloud
    vp = (1.0, -2.0, 3.0)
    g4 = D.estimate_normals(p, radius=RADIUS, viewpoint=vp, ctx=gpu_ctx)
    g8 = D.estimate_normals(np.c_[p, np.ones(len(p), np.float32)], radius=RADIUS, viewpoint=vp,
                            ctx=gpu_ctx, layout="pcl")
    np.testing.assert_array_equal(g8[:, :3], g4[:, :3])
    np.testing.assert_array_equal(g8[:, 4], g4[:, 3])
    assert np.all(g8[:, [3, 5, 6, 7]] == 0)
    ok = ~np.isnan(g4[:, 0])
    cosv = np.sum((np.asarray(vp, np.float32) - p[ok]) * g4[ok, :3], axis=1)
    assert np.all(cosv >= -1e-6)
    # a NaN point: NaN normal for it, invisible to the others
    q = p.copy()
    q[5] = np.nan
    gq = D.estimate_normals(q, radius=RADIUS, ctx=gpu_ctx)
    keep = np.arange(len(p)) != 5
    gk = D.estimate_normals(p[keep], radius=RADIUS, ctx=gpu_ctx)
    assert np.isnan(gq[5]).all()
    np.testing.assert_array_equal(gq[keep], gk)
    # isolated points (< 3 neighbours) -> NaN; empty input; bad arguments fail loudly
    iso = np.array([[0, 0, 0], [10, 0, 0], [0, 10, 0], [0, 0, 10]], np.float32)
    assert np.isnan(D.estimate_normals(iso, radius=1.0, ctx=gpu_ctx)).all()
    assert D.estimate_normals(np.zeros((0, 3), np.float32), radius=1.0, ctx=gpu_ctx).shape == (0, 4)
    with pytest.raises(D.DialogError):
        D.estimate_normals(p, ctx=gpu_ctx)  # neither radius nor k
    with pytest.raises(D.DialogError):
        D.estimate_normals(p, k=65, ctx=gpu_ctx)


@pytest.mark.gpu
@pytest.mark.parametrize("wave", [1, 0])
@pytest.mark.parametrize("seed_idx,outward,r", [(0, True, 0.08), (123, False, 0.08),
                                                (4567, True, 0.15), (11000, False, 0.05)])
def test_gpu_regulate_bit_exact(gpu_ctx, cloud, seed_idx, outward, r, wave):
    """Both claim passes (DLG_OPT_REGULATE_WAVE 1: a wave per frontier node, default; 0: a
    thread per (node, cell)) against the oracle's BFS, bit for bit."""
    import dialog_amd as D
    p, _, _ = cloud
    nrm = O.estimate_normals(p, RADIUS)
    # scramble the signs so the BFS has work to do
    rng = np.random.default_rng(seed_idx)
    nrm[:, :3] *= np.where(rng.random(len(p)) < 0.5, -1.0, 1.0).astype(np.float32)[:, None]
    o_reg, o_proc, o_cnt = O.regulate_normals(p, nrm, seed_idx, outward, r)
    gpu_ctx.set_option(D.DLG_OPT_REGULATE_WAVE, wave)
    try:
        g_reg, g_proc, g_cnt = D.regulate_normals(p, nrm, seed_idx, outward, r, ctx=gpu_ctx)
    finally:
        gpu_ctx.set_option(D.DLG_OPT_REGULATE_WAVE, 1)
    assert g_cnt == o_cnt
    assert np.array_equal(g_proc, o_proc)
    np.testing.assert_array_equal(g_reg, o_reg)  # NaN-aware, bit-exact
    # curvature column untouched
    np.testing.assert_array_equal(g_reg[:, 3], nrm[:, 3])


@pytest.mark.gpu
@pytest.mark.parametrize("seed_idx,outward,r", [(0, True, 0.08), (4567, False, 0.15)])
def test_gpu_cloud_regulate_bit_exact(gpu_ctx, cloud, seed_idx, outward, r):
    """dlg_cloud_regulate_normals: the BFS on the cloud's device copy and its attached normals
    (no host round trip) equals the oracle's BFS bit for bit; the regulated normals replace the
    attached ones (raw, as read back, and the curvature untouched)."""
    import dialog_amd as D
    p, _, _ = cloud
    nrm = O.estimate_normals(p, RADIUS)
    rng = np.random.default_rng(seed_idx + 7)
    nrm[:, :3] *= np.where(rng.random(len(p)) < 0.5, -1.0, 1.0).astype(np.float32)[:, None]
    o_reg, o_proc, o_cnt = O.regulate_normals(p, nrm, seed_idx, outward, r)
    cl = D.Cloud(gpu_ctx, p)
    try:
        cl.set_normals(nrm)
        g_proc, g_cnt, g_reg = cl.regulate_normals(seed_idx, outward, r, copy_out=True)
        assert g_cnt == o_cnt
        assert np.array_equal(g_proc, o_proc)
        np.testing.assert_array_equal(g_reg[:, :3], o_reg[:, :3])  # NaN-aware, bit-exact
        np.testing.assert_array_equal(g_reg[:, 3], nrm[:, 3])
        # a second call sees the regulated normals (they replaced the attached ones): with the
        # seed confirmed outward nothing flips any more
        g2_proc, g2_cnt, g2_reg = cl.regulate_normals(seed_idx, True, r, copy_out=True)
        o2_reg, o2_proc, o2_cnt = O.regulate_normals(p, o_reg, seed_idx, True, r)
        assert g2_cnt == o2_cnt and np.array_equal(g2_proc, o2_proc)
        np.testing.assert_array_equal(g2_reg[:, :3], o2_reg[:, :3])
        # invalid seed: nothing changes; out of range / no normals: errors
        pr, cnt, _ = cl.regulate_normals(-1, True, r)
        assert cnt == 0 and not pr.any()
        with pytest.raises(D.DialogError):
            cl.regulate_normals(len(p), True, r)
    finally:
        cl.close()
    bare = D.Cloud(gpu_ctx, p)
    try:
        with pytest.raises(D.DialogError):
            bare.regulate_normals(0, True, r)
    finally:
        bare.close()


@pytest.mark.gpu
def test_gpu_regulate_edges(gpu_ctx, cloud):
    import dialog_amd as D
    p, _, _ = cloud
    nrm = O.estimate_normals(p, RADIUS)
    reg, proc, cnt = D.regulate_normals(p, nrm, -1, True, 0.1, ctx=gpu_ctx)
    assert cnt == 0 and not proc.any()
    np.testing.assert_array_equal(reg, nrm)
    with pytest.raises(D.DialogError):
        D.regulate_normals(p, nrm, len(p), True, 0.1, ctx=gpu_ctx)
    # isolated seed: only itself, flipped when not outward
    iso = np.array([[0, 0, 0], [10, 0, 0], [0, 10, 0]], np.float32)
    n3 = np.array([[0, 0, 1, 0.5], [0, 1, 0, 0], [1, 0, 0, 0]], np.float32)
    reg, proc, cnt = D.regulate_normals(iso, n3, 0, False, 1.0, ctx=gpu_ctx)
    assert cnt == 1 and proc.tolist() == [True, False, False]
    np.testing.assert_array_equal(reg[0], [0, 0, -1, 0.5])


@pytest.mark.gpu
def test_gpu_normals_large_cloud_properties(gpu_ctx):
    """1M points on 3 planes: inlier normals are the generating plane normals."""
    import time

    import dialog_amd as D
    from dialog_amd.synth import plane_cloud
    p, lab, planes = plane_cloud(1_000_000, 3, outlier_frac=0.0, seed=99, patch=10.0)
    t0 = time.perf_counter()
    g = D.estimate_normals(p, radius=0.15, ctx=gpu_ctx)
    dt = time.perf_counter() - t0
    for k in range(3):
        m = lab == k
        d = np.abs(g[m, :3] @ planes[k, :3])
        good = ~np.isnan(d)
        assert good.mean() > 0.99
        assert np.median(d[good]) > 0.999
    gk = D.estimate_normals(p, k=20, ctx=gpu_ctx)
    for k in range(3):
        m = lab == k
        assert np.median(np.abs(gk[m, :3] @ planes[k, :3])) > 0.99
    print(json.dumps({"normals_1M_radius_s": round(dt, 3)}))


def test_oracle_orient_nn_semantics():
    """later-round branch: normal flips iff its dot with the nearest backup normal is < 0."""
    p, _, _ = small_cloud(1500, seed=21)
    nrm = O.estimate_normals(p, RADIUS)
    ref = p[::3] + np.float32(1e-3)
    rn = O.estimate_normals(ref, 0.2)
    out = O.orient_normals_nn(p, nrm, ref, rn)
    d2 = ((p[:, None, :].astype(np.float64) - ref[None, :, :]) ** 2).sum(-1)
    j = d2.argmin(1)
    dot = np.sum(nrm[:, :3] * rn[j, :3], axis=1)
    flip = dot < 0
    np.testing.assert_array_equal(out[flip, :3], -nrm[flip, :3])
    np.testing.assert_array_equal(out[~flip], nrm[~flip])


@pytest.mark.gpu
def test_gpu_orient_nn_bit_exact(gpu_ctx, cloud):
    import dialog_amd as D
    p, _, _ = cloud
    nrm = O.estimate_normals(p, RADIUS)
    rng = np.random.default_rng(4)
    nrm[:, :3] *= np.where(rng.random(len(p)) < 0.5, -1.0, 1.0).astype(np.float32)[:, None]
    # backup: a perturbed, subsampled copy with its own normals (the previous round's cloud)
    ref = (p[::2] + rng.normal(0, 0.003, size=(len(p[::2]), 3))).astype(np.float32)
    rn = O.estimate_normals(ref, 0.15)
    rn[np.isnan(rn)] = 0.0
    o = O.orient_normals_nn(p, nrm, ref, rn)
    g = D.orient_normals_nn(p, nrm, ref, rn, ctx=gpu_ctx)
    np.testing.assert_array_equal(g, o)
    # pcl::Normal stride (8 floats) in and out
    n8 = np.zeros((len(p), 8), np.float32)
    n8[:, :3] = nrm[:, :3]
    n8[:, 4] = nrm[:, 3]
    g8 = D.orient_normals_nn(np.c_[p, np.ones(len(p), np.float32)], n8, ref, rn, ctx=gpu_ctx)
    np.testing.assert_array_equal(g8[:, :3], o[:, :3])
    np.testing.assert_array_equal(g8[:, 4], nrm[:, 3])

