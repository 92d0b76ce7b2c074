"""preProcess() (Dialog/PlaneDetect.h:448-512) and removeRedundantPoints (PCLViewer.cpp:781-805).

Oracle: the reference loop restated literally (oracle/pcl_oracle.c orc_preprocess: NaN removal,
float centroid in index order, radiusSearch sorted by (dist2, index) with indices[0] skipped).
CPU tests pin it against the independent characterisation -- kept = the index-ordered maximal
independent set of the radius graph -- and the GPU (dlg_preprocess: parallel rounds of that MIS)
must equal it bit-for-bit: same kept indices, same translated coordinates, same translation.
Exact duplicates (distance 0 ties) follow the (dist2, index) order; FLANN leaves their order
unspecified, so results on clouds with exact duplicates are "parity unpinned" against PCL itself.
"""
import numpy as np
import pytest
from scipy.spatial import cKDTree

from oracle import oracle as O


def cloud(n, seed, nan_every=0, quantise=0.0):
    from dialog_amd.synth import plane_cloud
    p, _, _ = plane_cloud(n, 3, seed=seed, patch=2.0)
    if quantise:
        p = (np.round(p / quantise) * quantise).astype(np.float32)
    if nan_every:
        p[::nan_every, seed % 3] = np.nan
    return p


def mis_reference(p, r):
    """index-ordered MIS of {d2 < float(r*r)} (FLANN distance), brute force over a kd-tree."""
    r2 = np.float32(float(r) * float(r))
    tree = cKDTree(p.astype(np.float64))
    kept = np.zeros(len(p), bool)
    removed = np.zeros(len(p), bool)
    for i in range(len(p)):
        if removed[i]:
            continue
        kept[i] = True
        for j in tree.query_ball_point(p[i].astype(np.float64), r * 1.001):
            d = p[i] - p[j]
            d2 = ((np.float32(0) + d[0] * d[0]) + d[1] * d[1]) + d[2] * d[2]
            if j != i and d2 < r2:
                removed[j] = True
    return np.flatnonzero(kept)


def test_oracle_preprocess_is_index_ordered_mis():
    p = cloud(6000, 1, nan_every=101)
    out, idx, tr = O.preprocess(p, 0.03, translate=False)
    fin = np.flatnonzero(np.isfinite(p).all(1))
    ref = fin[mis_reference(p[fin], 0.03)]
    np.testing.assert_array_equal(idx, ref.astype(np.int32))
    np.testing.assert_array_equal(out, p[idx])
    # translation: float sums in index order / float(n)
    out2, idx2, tr2 = O.preprocess(p, 0.03, translate=True)
    q = p[fin]
    s = np.zeros(3, np.float32)
    for v in q:
        s = (s + v).astype(np.float32)
    np.testing.assert_array_equal(tr2, (s / np.float32(len(q))).astype(np.float32))
    np.testing.assert_array_equal(out2, (p[idx2] - tr2).astype(np.float32))


# ------------------------------------------------------------------------------------- GPU tests
@pytest.mark.gpu
@pytest.mark.parametrize("n,seed,r,translate,nan_every,quantise",
                         [(20000, 1, 0.02, True, 0, 0.0), (20000, 2, 0.05, False, 37, 0.0),
                          (50000, 3, 0.01, True, 0, 0.005), (3000, 4, 0.0, True, 7, 0.0),
                          (7, 5, 10.0, True, 0, 0.0)])
def test_gpu_preprocess_bit_exact(gpu_ctx, n, seed, r, translate, nan_every, quantise):
    import dialog_amd as D
    p = cloud(n, seed, nan_every, quantise)
    o_out, o_idx, o_tr = O.preprocess(p, r, translate)
    g_out, g_idx, g_tr = D.preprocess(p, r, translate, ctx=gpu_ctx)
    np.testing.assert_array_equal(g_idx, o_idx)
    np.testing.assert_array_equal(g_tr, o_tr)
    np.testing.assert_array_equal(g_out, o_out)


@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["offset", "centred", "quantised"])
def test_gpu_preprocess_centroid_large(gpu_ctx, kind):
    """The translation at sizes past fsum's chunk / unit / window boundaries (PlaneDetect.h:463-471:
    p.x += x_i in index order, then / float(n)); np.cumsum is the literal sequential float loop.
    'centred' makes the chains hover around zero (the walk's slow, start-dependent windows)."""
    import dialog_amd as D
    rng = np.random.default_rng({"offset": 11, "centred": 12, "quantised": 13}[kind])
    n = {"offset": 1_000_003, "centred": 2_000_000, "quantised": 1_500_001}[kind]
    p = rng.normal(0.0, 3.0, (n, 3)).astype(np.float32)
    if kind == "offset":
        p += np.float32([120.0, -45.0, 7.5])
    elif kind == "quantised":
        p = (np.round(p / 0.001) * 0.001 + 2.0).astype(np.float32)
    p[rng.choice(n, 97, replace=False), 1] = np.nan  # dropped before the sums
    _, g_idx, g_tr = D.preprocess(p, 0.0, True, ctx=gpu_ctx)
    q = p[np.all(np.isfinite(p), axis=1)]
    assert 0 < len(g_idx) <= len(q)  # (the translation comes before redundancy removal)
    want = np.array([np.cumsum(q[:, k], dtype=np.float32)[-1] for k in range(3)], np.float32)
    want = (want / np.float32(len(q))).astype(np.float32)
    np.testing.assert_array_equal(np.asarray(g_tr, np.float32).view(np.uint32), want.view(np.uint32))


@pytest.mark.gpu
def test_gpu_preprocess_edges(gpu_ctx):
    import dialog_amd as D
    # all NaN, empty, PointXYZ stride, capacity error
    allnan = np.full((10, 3), np.nan, np.float32)
    out, idx, tr = D.preprocess(allnan, 0.1, ctx=gpu_ctx)
    assert len(idx) == 0
    out, idx, tr = D.preprocess(np.zeros((0, 3), np.float32), 0.1, ctx=gpu_ctx)
    assert len(idx) == 0
    p = cloud(5000, 6)
    a, ia, ta = D.preprocess(p, 0.03, ctx=gpu_ctx)
    b, ib, tb = D.preprocess(np.c_[p, np.ones(len(p), np.float32)], 0.03, ctx=gpu_ctx)
    np.testing.assert_array_equal(ia, ib)
    np.testing.assert_array_equal(a, b)
    assert np.array_equal(D.remove_redundant_points(p, 0.03, ctx=gpu_ctx),
                          O.preprocess(p, 0.03, translate=False)[1])


@pytest.mark.gpu
def test_gpu_preprocess_large_properties(gpu_ctx):
    """2M points: kept points are pairwise >= r apart and every dropped point is within r of a
    kept point of lower index (the defining properties), checked on a sample."""
    import dialog_amd as D
    from dialog_amd.synth import plane_cloud
    p, _, _ = plane_cloud(2_000_000, 5, seed=8, patch=10.0)
    r = 0.02
    out, idx, tr = D.preprocess(p, r, translate=False, ctx=gpu_ctx)
    assert 0 < len(idx) < len(p)
    kept = p[idx].astype(np.float64)
    tree = cKDTree(kept)
    pairs = tree.query_pairs(r * 0.999)
    assert len(pairs) == 0
    dropped = np.setdiff1d(np.arange(len(p)), idx)
    rng = np.random.default_rng(0)
    sample = rng.choice(dropped, 2000, replace=False)
    d, j = tree.query(p[sample].astype(np.float64))
    assert np.all(d < r * 1.001)
