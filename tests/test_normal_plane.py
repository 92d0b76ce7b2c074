"""SACMODEL_NORMAL_PLANE (SACSegmentationFromNormals; BASELINE config C5).

The reference does not call this model; PCL 1.8's SampleConsensusModelNormalPlane is restated in
oracle/pcl_oracle.c (orc_normal_plane_dist) and cross-checked here by an independent numpy
restatement.  "Parity unpinned" as the rest of the PCL arithmetic (no PCL build here), and the
exact getAngle3D form (n.normalized().dot(coeff.normalized()), clamped, acos) is taken from the
PCL 1.8 sources as published.  GPU results must equal the oracle bit-for-bit (PCL float refit):
same iterations, same winning sample, same coefficients bits, same inlier lists.
"""
import os
import threading

import numpy as np
import pytest

from oracle import oracle as O

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def np_twin_dist(c, p, nrm, lam):
    """numpy restatement of the NORMAL_PLANE point distance (float32 ops in Eigen's order)."""
    c = np.asarray(c, np.float32)
    p = np.asarray(p, np.float32)
    n = np.asarray(nrm, np.float32)
    f = np.float32
    de = np.abs(((c[0] * p[:, 0] + c[2] * p[:, 2]) + (c[1] * p[:, 1] + f(0) * f(0))) + c[3])

    def normalized(v0, v1, v2):
        z = (v0 * v0 + v2 * v2) + (v1 * v1 + f(0) * f(0))
        s = np.sqrt(z)
        ok = z > 0
        with np.errstate(invalid="ignore", divide="ignore"):
            return (np.where(ok, v0 / s, v0), np.where(ok, v1 / s, v1), np.where(ok, v2 / s, v2))

    nx, ny, nz = normalized(n[:, 0], n[:, 1], n[:, 2])
    cx, cy, cz = normalized(np.full(1, c[0]), np.full(1, c[1]), np.full(1, c[2]))
    rad = ((nx * cx + nz * cz) + (ny * cy + f(0) * f(0))).astype(np.float64)
    rad = np.where(rad < -1.0, -1.0, np.where(rad > 1.0, 1.0, rad))
    dn = np.abs(np.arccos(rad))
    alt = np.pi - dn
    dn = np.where(alt < dn, alt, dn)
    w = lam * (1.0 - n[:, 3].astype(np.float64))
    return np.abs(w * dn + (1.0 - w) * de.astype(np.float64))


def cloud_with_normals(n=8192, seed=6, outliers=0.1):
    from dialog_amd.synth import plane_cloud
    p, lab, pl = plane_cloud(n, 3, outlier_frac=outliers, seed=seed, patch=2.0)
    return p, O.estimate_normals(p, 0.1), lab, pl


# ------------------------------------------------------------------------------------- CPU tests
def test_oracle_np_distance_matches_numpy_twin():
    p, nrm, _, _ = cloud_with_normals(3000, seed=2)
    rng = np.random.default_rng(0)
    for t in range(20):
        i = rng.choice(len(p), 3, replace=False)
        c = np.zeros(4, np.float32)
        # a plane through three of the points
        v1, v2 = p[i[1]] - p[i[0]], p[i[2]] - p[i[0]]
        nn = np.cross(v1.astype(np.float64), v2.astype(np.float64))
        nn /= np.linalg.norm(nn)
        c[:3] = nn
        c[3] = -np.dot(nn, p[i[0]])
        lam = [0.0, 0.1, 0.5, 1.0][t % 4]
        ok = ~np.isnan(nrm[:, 0])
        twin = np_twin_dist(c, p[ok], nrm[ok], lam)
        orc = np.array([O.normal_plane_dist(c, p[k], nrm[k], lam) for k in np.flatnonzero(ok)[:400]])
        np.testing.assert_allclose(orc, twin[:400], rtol=1e-14, atol=1e-15)
        for thr in (0.01, 0.05, 0.2):
            assert O.count_within_np(p, nrm, c, thr, lam) == int((twin < thr).sum())


def test_oracle_np_prefilter_any_curvature():
    """The oracle's countWithinDistance shortcut ((1 - w) d >= threshold decides "out" without the
    acos, for w in [0, 1]) gives the twin's counts also for weights outside [0, 1] (curvature
    above 1 or below 0), NaN curvature and NaN / zero normals, where it must not apply."""
    p, nrm, _, _ = cloud_with_normals(4000, seed=9)
    rng = np.random.default_rng(9)
    nrm = nrm.copy()
    nrm[:, 3] = rng.uniform(-0.5, 1.5, len(nrm)).astype(np.float32)
    nrm[::37, 3] = np.nan
    nrm[5::53, :3] = np.nan
    nrm[7::61, :3] = 0.0
    for t in range(12):
        i = rng.choice(len(p), 3, replace=False)
        nn = np.cross((p[i[1]] - p[i[0]]).astype(np.float64), (p[i[2]] - p[i[0]]).astype(np.float64))
        nn /= np.linalg.norm(nn)
        c = np.array([*nn, -np.dot(nn, p[i[0]])], np.float32)
        lam = [0.1, 0.7, 1.0, 2.0][t % 4]
        twin = np_twin_dist(c, p, nrm, lam)
        for thr in (0.01, 0.05, 0.3):
            assert O.count_within_np(p, nrm, c, thr, lam) == int((twin < thr).sum())


def test_oracle_np_segment_properties():
    p, nrm, lab, pl = cloud_with_normals()
    r = O.sac_segment(p, 0.05, max_iterations=200, normals=nrm, normal_distance_weight=0.1)
    assert r["ok"]
    d = np_twin_dist(r["coeff"], p, nrm, 0.1)
    ok = np.flatnonzero(d < 0.05)
    assert np.array_equal(ok.astype(np.int32), r["inliers"])
    # the plane found is one of the generator's planes
    k = np.argmax(np.abs(pl[:, :3] @ r["coeff"][:3]))
    assert abs(abs(pl[k, :3] @ r["coeff"][:3]) - 1) < 1e-3
    # the RNG stream does not depend on the model: same draws as the plane model
    r0 = O.sac_segment(p, 0.05, max_iterations=3, probability=1.0, normals=nrm)
    rp = O.sac_segment(p, 0.05, max_iterations=3, probability=1.0)
    assert r0["draws"] == rp["draws"]


def test_oracle_np_fixture():
    z = np.load(os.path.join(GOLDEN, "normal_plane_small.npz"))
    r = O.sac_segment(z["points"], float(z["seg_threshold"]),
                      max_iterations=int(z["seg_max_iterations"]),
                      probability=float(z["seg_probability"]), normals=z["normals"],
                      normal_distance_weight=float(z["seg_lambda"]))
    assert r["iterations"] == int(z["seg_iterations"])
    assert np.array_equal(r["coeff"].view(np.uint32), z["seg_coeff"].view(np.uint32))
    assert np.array_equal(r["inliers"], z["seg_inliers"])


# ------------------------------------------------------------------------------------- GPU tests
@pytest.mark.gpu
@pytest.mark.parametrize("pruned", ["none", "before", "after"])
def test_gpu_np_segment_golden(gpu_ctx, pruned):
    """pruned: the Morton-ordered copy (pruned NORMAL_PLANE scoring, spatial.hip) built before
    or after the normals are attached (normals gathered into it either way)."""
    import dialog_amd as D
    z = np.load(os.path.join(GOLDEN, "normal_plane_small.npz"))
    cloud = D.Cloud(gpu_ctx, z["points"])
    if pruned == "before":
        cloud.build_spatial()
    cloud.set_normals(z["normals"])
    if pruned == "after":
        cloud.build_spatial()
    prm = D.make_params(float(z["seg_threshold"]), max_iterations=int(z["seg_max_iterations"]),
                        probability=float(z["seg_probability"]), model=D.SACMODEL_NORMAL_PLANE,
                        normal_distance_weight=float(z["seg_lambda"]))
    inl, coeff, st = D.segment_cloud(cloud, prm)
    assert st["iterations"] == int(z["seg_iterations"])
    assert np.array_equal(st["best_sample"], z["seg_best_sample"])
    assert np.array_equal(coeff.view(np.uint32), z["seg_coeff"].view(np.uint32))
    assert np.array_equal(inl, z["seg_inliers"])
    cloud.close()


@pytest.mark.gpu
@pytest.mark.parametrize("pruned", [False, True])
def test_gpu_np_extract_golden(gpu_ctx, pruned):
    import dialog_amd as D
    z = np.load(os.path.join(GOLDEN, "normal_plane_small.npz"))
    cloud = D.Cloud(gpu_ctx, z["points"])
    if pruned:  # the Morton copy is compacted with the list (normals included) every round
        cloud.build_spatial()
    # pcl::Normal records (stride 32) must give the same result as (n, curvature) float4
    rec = np.zeros((z["normals"].shape[0], 8), np.float32)
    rec[:, :3] = z["normals"][:, :3]
    rec[:, 4] = z["normals"][:, 3]
    cloud.set_normals(rec)
    prm = D.make_params(float(z["ex_threshold"]), max_iterations=int(z["ex_max_iterations"]),
                        probability=1.0, model=D.SACMODEL_NORMAL_PLANE,
                        normal_distance_weight=float(z["ex_lambda"]))
    e = D.extract_planes(cloud, prm, max_planes=int(z["ex_max_planes"]),
                         min_inliers=int(z["ex_min_inliers"]))
    assert np.array_equal(e["offsets"], z["ex_offsets"])
    assert np.array_equal(e["coeffs"].view(np.uint32), z["ex_coeffs"].view(np.uint32))
    assert np.array_equal(e["inliers"], z["ex_inliers"])
    cloud.close()


@pytest.mark.gpu
@pytest.mark.parametrize("pruned", [False, True, "rl"])
@pytest.mark.parametrize("seed,lam,thr", [(1, 0.1, 0.05), (2, 0.5, 0.1), (3, 0.0, 0.02),
                                          (4, 1.0, 0.3), (5, 0.2, 0.05)])
def test_gpu_np_random_vs_oracle(gpu_ctx, seed, lam, thr, pruned):
    """pruned: the Morton copy with the default tile scorer (lanes as planes), or "rl" with
    DLG_TILE_BF16 (round 4's lanes-as-points NORMAL_PLANE scorer)."""
    import dialog_amd as D
    p, nrm, _, _ = cloud_with_normals(int(2000 + 3000 * seed), seed=seed, outliers=0.2)
    if seed == 5:  # NaN normals (isolated points) and a zero normal
        nrm[::97] = np.nan
        nrm[5, :3] = 0.0
    idx = None
    if seed == 2:  # setIndices subset, unsorted
        idx = np.random.default_rng(seed).permutation(len(p))[: len(p) // 2].astype(np.int32)
    r = O.sac_segment(p, thr, indices=idx, max_iterations=300, normals=nrm,
                      normal_distance_weight=lam)
    cloud = D.Cloud(gpu_ctx, p, indices=idx)
    if pruned:  # (lam = 1 with zero curvatures: w reaches 1, the exhaustive kernel runs)
        cloud.build_spatial()
    cloud.set_normals(nrm)
    prm = D.make_params(thr, max_iterations=300, model=D.SACMODEL_NORMAL_PLANE,
                        normal_distance_weight=lam)
    if pruned == "rl":
        gpu_ctx.set_option(D.DLG_OPT_PRUNE_TILE_SCORER, D.DLG_TILE_BF16)
    try:
        inl, coeff, st = D.segment_cloud(cloud, prm)
    finally:
        gpu_ctx.set_option(D.DLG_OPT_PRUNE_TILE_SCORER, D.DLG_TILE_EXACT)
    assert st["has_model"] == r["ok"]
    assert st["iterations"] == r["iterations"]
    assert np.array_equal(st["best_sample"], r["best_sample"])
    assert np.array_equal(coeff.view(np.uint32), r["coeff"].view(np.uint32))
    assert np.array_equal(inl, r["inliers"])
    cloud.close()


@pytest.mark.gpu
def test_gpu_np_requires_normals_and_fast_refit(gpu_ctx):
    import dialog_amd as D
    p, nrm, _, _ = cloud_with_normals(6000, seed=9)
    cloud = D.Cloud(gpu_ctx, p)
    prm = D.make_params(0.05, max_iterations=100, model=D.SACMODEL_NORMAL_PLANE)
    with pytest.raises(D.DialogError):
        D.segment_cloud(cloud, prm)
    with pytest.raises(D.DialogError):
        cloud.set_normals(nrm[:-1])  # one record per point
    cloud.set_normals(nrm)
    prm_f = D.make_params(0.05, max_iterations=100, model=D.SACMODEL_NORMAL_PLANE,
                          refit_mode=D.DLG_REFIT_FAST)
    inl, coeff, st = D.segment_cloud(cloud, prm_f)
    r = O.sac_segment(p, 0.05, max_iterations=100, normals=nrm, refit="fast")
    assert np.array_equal(coeff.view(np.uint32), r["coeff"].view(np.uint32))
    rd = O.sac_segment(p, 0.05, max_iterations=100, normals=nrm, refit="double")
    sg = 1.0 if coeff[:3] @ rd["coeff"][:3] > 0 else -1.0  # (the double twin is not oriented)
    assert np.abs(coeff - sg * rd["coeff"]).max() < 1e-5
    d = np_twin_dist(coeff, p, nrm, 0.1)
    assert np.array_equal(inl, np.flatnonzero(d < 0.05).astype(np.int32))
    # the PCL mirror
    seg = D.SACSegmentationFromNormals(gpu_ctx)
    seg.setModelType(D.SACMODEL_NORMAL_PLANE)
    seg.setMethodType(D.SAC_RANSAC)
    seg.setDistanceThreshold(0.05)
    seg.setMaxIterations(100)
    seg.setNormalDistanceWeight(0.1)
    seg.setInputCloud(p)
    seg.setInputNormals(nrm)
    i2, c2 = seg.segment()
    r2 = O.sac_segment(p, 0.05, max_iterations=100, normals=nrm)
    assert np.array_equal(i2, r2["inliers"])
    assert np.array_equal(c2.view(np.uint32), r2["coeff"].view(np.uint32))
    cloud.close()


@pytest.mark.gpu
@pytest.mark.parametrize("world", [2, 3])
def test_gpu_np_loopback_sharded(gpu_ctx, world):
    import dialog_amd as D
    p, nrm, _, _ = cloud_with_normals(20000, seed=12)
    prm = D.make_params(0.05, max_iterations=255, probability=1.0,
                        model=D.SACMODEL_NORMAL_PLANE, normal_distance_weight=0.2)
    cloud = D.Cloud(gpu_ctx, p)
    cloud.set_normals(nrm)
    ref = D.extract_planes(cloud, prm, max_planes=4, min_inliers=200)
    cloud.close()
    ctxs = D.Context.loopback_group(world, 0)
    bounds = np.linspace(0, p.shape[0], world + 1).astype(np.int64)
    out = [None] * world
    errs = []

    def run(r):
        try:
            c = D.Cloud(ctxs[r], p[bounds[r]:bounds[r + 1]], id_base=int(bounds[r]))
            c.set_normals(nrm[bounds[r]:bounds[r + 1]])
            out[r] = D.extract_planes(c, prm, max_planes=4, min_inliers=200, capacity=p.shape[0])
            c.close()
        except Exception as e:  # pragma: no cover
            errs.append(e)

    th = [threading.Thread(target=run, args=(r,)) for r in range(world)]
    [t.start() for t in th]
    [t.join() for t in th]
    assert not errs, errs
    for r in range(world):
        assert np.array_equal(out[r]["offsets"], ref["offsets"])
        assert np.array_equal(out[r]["coeffs"].view(np.uint32), ref["coeffs"].view(np.uint32))
        assert np.array_equal(out[r]["inliers"], ref["inliers"])
    for c in ctxs:
        c.close()


@pytest.mark.gpu
def test_gpu_cloud_normals_refused_on_a_shard():
    """dlg_cloud_estimate_normals on one rank's shard (world > 1) is refused: points near the
    cut would lose their neighbours on other ranks.  The whole cloud's normals, attached per
    shard with set_normals, are the supported path (test_gpu_np_loopback_sharded)."""
    import dialog_amd as D
    p, _, _, _ = cloud_with_normals(4000, seed=5)
    ctxs = D.Context.loopback_group(2, 0)
    try:
        c = D.Cloud(ctxs[0], p[:2000], id_base=0)
        with pytest.raises(D.DialogError):
            c.estimate_normals(radius=0.1)
        c.close()
    finally:
        for x in ctxs:
            x.close()


# ------------------------------------------------------------------------------------- C5 chain
@pytest.mark.gpu
@pytest.mark.parametrize("nmode,refit", [("radius", "pcl"), ("knn", "pcl"), ("knn", "fast")])
def test_gpu_c5_chain_vs_oracle_chain(gpu_ctx, nmode, refit):
    """BASELINE configs[4] (C5) end to end at test size: GPU normals (PCL-float mode) ->
    GPU SACMODEL_NORMAL_PLANE extract-and-remove equals oracle normals -> oracle extract, bit for
    bit (the normals are bit-identical, so every normal-plane distance is too)."""
    import dialog_amd as D
    from dialog_amd.synth import plane_cloud
    p, _, _ = plane_cloud(30000, 5, outlier_frac=0.1, seed=55, patch=2.0)
    if nmode == "radius":
        g = D.estimate_normals(p, radius=0.1, ctx=gpu_ctx)
        o = O.estimate_normals(p, 0.1)
    else:
        g = D.estimate_normals(p, k=20, ctx=gpu_ctx)
        o = O.estimate_normals_knn(p, 20)
    assert np.array_equal(g.view(np.uint32), o.view(np.uint32))
    kw = dict(max_iterations=255, probability=1.0)
    mode = D.DLG_REFIT_PCL if refit == "pcl" else D.DLG_REFIT_FAST
    prm = D.make_params(0.05, model=D.SACMODEL_NORMAL_PLANE, normal_distance_weight=0.1,
                        refit_mode=mode, **kw)
    r = O.extract_planes(p, 0.05, max_planes=6, min_inliers=200, normals=o,
                         normal_distance_weight=0.1, refit=refit, **kw)
    # host hand-off (normals out, then back in) and the device-resident chain
    # (dlg_cloud_estimate_normals: the normals never leave the device)
    for resident in (False, True):
        cloud = D.Cloud(gpu_ctx, p)
        if resident:
            gd = cloud.estimate_normals(radius=0.1 if nmode == "radius" else 0.0,
                                        k=0 if nmode == "radius" else 20, copy_out=True)
            assert np.array_equal(gd.view(np.uint32), o.view(np.uint32))
        else:
            cloud.set_normals(g)
        e = D.extract_planes(cloud, prm, max_planes=6, min_inliers=200)
        cloud.close()
        assert e["n_planes"] == r["n_planes"] >= 4
        assert np.array_equal(e["coeffs"].view(np.uint32), r["coeffs"].view(np.uint32))
        assert np.array_equal(e["offsets"], r["offsets"])
        assert np.array_equal(e["inliers"], r["inliers"])


@pytest.mark.gpu
@pytest.mark.parametrize("refit", ["pcl", "fast"])
def test_gpu_c5_regulate_chain_vs_oracle_chain(gpu_ctx, refit):
    """The reference's order end to end at test size, all on the device copy: k = 20 normals
    (dlg_cloud_estimate_normals) -> RegulateNormal (dlg_cloud_regulate_normals, BFS r 0.1 from
    point 0) -> SACMODEL_NORMAL_PLANE extract-and-remove, equal to the oracle's chain (k-NN
    normals -> regulate_normals -> extract) bit for bit."""
    import dialog_amd as D
    from dialog_amd.synth import plane_cloud
    p, _, _ = plane_cloud(30000, 5, outlier_frac=0.1, seed=56, patch=2.0)
    o = O.estimate_normals_knn(p, 20)
    o_reg, _, o_cnt = O.regulate_normals(p, o, 0, False, 0.1)
    kw = dict(max_iterations=255, probability=1.0)
    mode = D.DLG_REFIT_PCL if refit == "pcl" else D.DLG_REFIT_FAST
    prm = D.make_params(0.05, model=D.SACMODEL_NORMAL_PLANE, normal_distance_weight=0.1,
                        refit_mode=mode, **kw)
    r = O.extract_planes(p, 0.05, max_planes=6, min_inliers=200, normals=o_reg,
                         normal_distance_weight=0.1, refit=refit, **kw)
    cloud = D.Cloud(gpu_ctx, p)
    try:
        cloud.estimate_normals(k=20)
        _, cnt, g_reg = cloud.regulate_normals(0, False, 0.1, copy_out=True)
        assert cnt == o_cnt
        assert np.array_equal(g_reg.view(np.uint32), o_reg.view(np.uint32))
        e = D.extract_planes(cloud, prm, max_planes=6, min_inliers=200)
    finally:
        cloud.close()
    assert e["n_planes"] == r["n_planes"] >= 4
    assert np.array_equal(e["coeffs"].view(np.uint32), r["coeffs"].view(np.uint32))
    assert np.array_equal(e["offsets"], r["offsets"])
    assert np.array_equal(e["inliers"], r["inliers"])


@pytest.mark.gpu
def test_gpu_cloud_normals_index_subset(gpu_ctx):
    """dlg_cloud_estimate_normals on a cloud uploaded with an index subset (and a non-zero id
    base): the normals of the subset cloud itself, == dlg_estimate_normals on those points."""
    import dialog_amd as D
    from dialog_amd.synth import plane_cloud
    p, _, _ = plane_cloud(40000, 4, outlier_frac=0.1, seed=77, patch=2.0)
    idx = np.sort(np.random.default_rng(1).choice(p.shape[0], 25000, replace=False)).astype(np.int32)
    cloud = D.Cloud(gpu_ctx, p, indices=idx, id_base=1000)
    gd = cloud.estimate_normals(k=12, copy_out=True)
    cloud.close()
    ref = D.estimate_normals(p[idx], k=12, ctx=gpu_ctx)
    assert np.array_equal(gd.view(np.uint32), ref.view(np.uint32))


@pytest.mark.gpu
@pytest.mark.slow
def test_gpu_c5_full_size_properties(gpu_ctx):
    """C5 at its quoted size (10M points, k = 20 PCL-float normals, NORMAL_PLANE w = 0.1, 4096
    hypotheses per round): every extracted inlier passes PCL's normal-plane test (numpy
    restatement on a sample), planes disjoint and ascending, deterministic across runs."""
    import dialog_amd as D
    from dialog_amd.synth import SEED_BASE, plane_cloud
    p, _, _ = plane_cloud(10_000_000, 20, seed=SEED_BASE + 5)
    cloud = D.Cloud(gpu_ctx, p)
    nrm = cloud.estimate_normals(k=20, copy_out=True)  # (device-resident: attached on the GPU)
    assert np.isfinite(nrm).all()
    prm = D.make_params(0.02, max_iterations=4095, probability=1.0, refit_mode=D.DLG_REFIT_FAST,
                        hypotheses_per_launch=4096, model=D.SACMODEL_NORMAL_PLANE,
                        normal_distance_weight=0.1)
    e = D.extract_planes(cloud, prm, max_planes=20, min_inliers=500, capacity=p.shape[0])
    cloud.reset()
    e2 = D.extract_planes(cloud, prm, max_planes=20, min_inliers=500, capacity=p.shape[0])
    cloud.close()
    assert e["n_planes"] >= 18
    assert np.array_equal(e["inliers"], e2["inliers"])
    assert np.array_equal(e["coeffs"].view(np.uint32), e2["coeffs"].view(np.uint32))
    inl, offs = e["inliers"], e["offsets"]
    assert np.unique(inl).size == inl.size
    rng = np.random.default_rng(0)
    for k in range(e["n_planes"]):
        ids = inl[offs[k]:offs[k + 1]]
        assert np.all(np.diff(ids) > 0)
        s = ids[rng.choice(ids.size, min(2000, ids.size), replace=False)]
        d = np_twin_dist(e["coeffs"][k], p[s], nrm[s], 0.1)
        assert np.all(d < 0.02)


@pytest.mark.gpu
@pytest.mark.parametrize("lam", [0.1, 0.7])
def test_gpu_np_tile_scorers_agree(gpu_ctx, lam):
    """The pruned NORMAL_PLANE scorers (default: lanes as planes with the prefilter verdicts as
    bits, spatial.hip k_score_tiles_ex<NPM>; DLG_TILE_BF16: k_score_tiles_rl<NPM>, lanes as
    points) and the exhaustive kernel (DLG_OPT_PRUNE_NP 0) extract the same planes bit for bit
    from a 300k-point cloud with synthetic normals (tilted, NaN, zero and high-curvature ones)."""
    import dialog_amd as D
    from dialog_amd.synth import plane_cloud
    p, lab, pl = plane_cloud(300_000, 6, outlier_frac=0.15, seed=31)
    rng = np.random.default_rng(31)
    nrm = np.zeros((p.shape[0], 4), np.float32)
    for k in range(len(pl)):
        nrm[lab == k, :3] = np.asarray(pl[k][:3], np.float32)
    out = lab < 0
    nrm[out, :3] = rng.normal(size=(int(out.sum()), 3)).astype(np.float32)
    nrm[:, :3] += rng.normal(scale=0.05, size=(p.shape[0], 3)).astype(np.float32)
    nrm[:, :3] /= np.linalg.norm(nrm[:, :3], axis=1, keepdims=True)
    nrm[:, 3] = rng.uniform(0.0, 0.3, p.shape[0]).astype(np.float32)
    nrm[::101] = np.nan
    nrm[7::997, :3] = 0.0
    nrm[11::503, 3] = 1.5  # (w < 0: the prefilter does not apply)
    prm = D.make_params(0.03, max_iterations=1023, probability=1.0,
                        model=D.SACMODEL_NORMAL_PLANE, normal_distance_weight=lam)
    res = {}
    for name, opts in (("ex", {}), ("rl", {D.DLG_OPT_PRUNE_TILE_SCORER: D.DLG_TILE_BF16}),
                       ("exhaustive", {D.DLG_OPT_PRUNE_NP: 0})):
        for k, v in opts.items():
            gpu_ctx.set_option(k, v)
        try:
            cloud = D.Cloud(gpu_ctx, p)
            cloud.set_normals(nrm)
            if name != "exhaustive":
                cloud.build_spatial()
            res[name] = D.extract_planes(cloud, prm, max_planes=6, min_inliers=500)
            cloud.close()
        finally:
            gpu_ctx.set_option(D.DLG_OPT_PRUNE_TILE_SCORER, D.DLG_TILE_EXACT)
            gpu_ctx.set_option(D.DLG_OPT_PRUNE_NP, 1)
    ref = res["exhaustive"]
    assert len(ref["offsets"]) > 2
    for name in ("ex", "rl"):
        assert np.array_equal(res[name]["offsets"], ref["offsets"]), name
        assert np.array_equal(res[name]["coeffs"].view(np.uint32), ref["coeffs"].view(np.uint32)), name
        assert np.array_equal(res[name]["inliers"], ref["inliers"]), name
