"""GPU: the pruned scoring path (spatial.hpp -- Morton-ordered copy, tile / super-tile bounding
spheres, k_score_pruned) against the oracle and against the exhaustive kernels.

Clouds of >= 131072 points get the spatial copy at upload; here it is forced on small clouds
(Cloud.build_spatial) so that every case the exhaustive path is checked on is also checked with
pruned scoring: bit-exact best sample / iterations / coefficients / inlier lists against the
PCL restatement, extract-and-remove (the spatial copy is compacted with the list every round),
reset, non-finite points, and counts equal to the exhaustive kernels' on band-loaded clouds.
"""
import json
import os
import threading

import numpy as np
import pytest

import dialog_amd as D
from dialog_amd.pcd import read_pcd
from dialog_amd.synth import SEED_BASE, plane_cloud
from oracle import oracle as O

pytestmark = pytest.mark.gpu


def seg(ctx, pts, thr, indices=None, **kw):
    cloud = D.Cloud(ctx, pts, indices=indices)
    try:
        cloud.build_spatial()
        return D.segment_cloud(cloud, D.make_params(thr, **kw))
    finally:
        cloud.close()


def same(inl, coeff, st, r):
    assert st["has_model"] == r["ok"]
    assert (st["iterations"], st["draws"]) == (r["iterations"], r["draws"])
    if not r["ok"]:
        assert inl.size == 0
        return
    assert list(st["best_sample"]) == list(r["best_sample"])
    assert st["n_unrefined"] == r["n_unrefined"]
    assert np.array_equal(coeff.view(np.uint32), r["coeff"].view(np.uint32))
    assert np.array_equal(inl, r["inliers"])


@pytest.mark.parametrize("seed", range(12))
def test_pruned_random_clouds_vs_oracle(gpu_ctx, seed):
    rng = np.random.default_rng(5000 + seed)
    n = int(rng.choice([3, 5, 100, 1000, 5000, 20000, 60000]))
    p, _, _ = plane_cloud(n, int(rng.integers(1, 5)), seed=seed + 77,
                          outlier_frac=float(rng.uniform(0, 0.5)))
    if seed % 3 == 0:  # quantised: duplicates, ties, collinear draws
        p = (np.round(p * 2) / 2).astype(np.float32)
    if seed % 4 == 1 and n > 10:  # non-finite points (never inliers; not in the spatial copy)
        p[::7, 0] = np.nan
        p[3::11, 2] = np.inf
    thr = float(rng.choice([0.005, 0.02, 0.1, 0.25]))
    mi = int(rng.choice([10, 50, 300, 1000, 4095]))
    pr = float(rng.choice([0.9, 0.99, 1.0]))
    r = O.sac_segment(p, thr, max_iterations=mi, probability=pr)
    same(*seg(gpu_ctx, p, thr, max_iterations=mi, probability=pr), r)


@pytest.mark.parametrize("name", ["pcl_defaults", "h4096", "pcl_defaults_t02"])
def test_pruned_double_shadow(gpu_ctx, golden_dir, name):
    pts = read_pcd(os.path.join(golden_dir, "double_shadow.pcd"))
    g = json.load(open(os.path.join(golden_dir, "double_shadow.json")))["configs"][name]
    kw = {k: g[k] for k in ("max_iterations", "probability") if k in g}
    inl, coeff, st = seg(gpu_ctx, pts, g["threshold"], **kw)
    assert st["iterations"] == g["iterations"] and list(st["best_sample"]) == g["best_sample"]
    assert list(coeff.view(np.uint32)) == g["coeff_bits"]
    assert list(inl) == g["inliers"]


def test_pruned_extract_golden_and_reset(gpu_ctx, golden_dir):
    z = np.load(os.path.join(golden_dir, "synth_c3_small.npz"))
    cloud = D.Cloud(gpu_ctx, z["points"])
    cloud.build_spatial()
    prm = D.make_params(float(z["threshold"]), max_iterations=int(z["max_iterations"]),
                        probability=float(z["probability"]))
    for _ in range(2):  # second pass after reset: the pristine spatial copy is back
        e = D.extract_planes(cloud, prm, max_planes=int(z["max_planes"]),
                             min_inliers=int(z["min_inliers"]))
        assert np.array_equal(e["offsets"], z["offsets"])
        assert np.array_equal(e["inliers"], z["inliers"])
        assert np.array_equal(e["coeffs"].view(np.uint32), z["coeffs"].view(np.uint32))
        cloud.reset()
    cloud.close()


def test_pruned_extract_nonfinite_vs_oracle(gpu_ctx):
    p, _, _ = plane_cloud(30000, 5, seed=31)
    p[::13, 1] = np.nan
    p[5::101] = np.inf
    kw = dict(max_iterations=300, probability=0.99)
    ref = O.extract_planes(p, 0.02, max_planes=6, min_inliers=100, **kw)
    cloud = D.Cloud(gpu_ctx, p)
    cloud.build_spatial()
    e = D.extract_planes(cloud, D.make_params(0.02, **kw), max_planes=6, min_inliers=100)
    assert e["n_planes"] == ref["n_planes"] >= 4
    assert np.array_equal(e["coeffs"].view(np.uint32), ref["coeffs"].view(np.uint32))
    assert np.array_equal(e["inliers"], ref["inliers"])
    cloud.close()


def test_pruned_after_normal_plane_round(gpu_ctx):
    """A SACMODEL_NORMAL_PLANE round compacts only the list: the spatial copy is dropped (the
    exhaustive kernel takes over) until reset restores it; results stay exact."""
    p, _, _ = plane_cloud(20000, 3, seed=8)
    nrm = np.zeros((p.shape[0], 4), np.float32)
    nrm[:, 2] = 1.0
    cloud = D.Cloud(gpu_ctx, p)
    cloud.build_spatial()
    cloud.set_normals(nrm)
    npp = D.make_params(0.05, max_iterations=100, model=D.SACMODEL_NORMAL_PLANE,
                        normal_distance_weight=0.1)
    e1 = D.extract_planes(cloud, npp, max_planes=1, min_inliers=10)
    assert e1["n_planes"] == 1
    rem = np.setdiff1d(np.arange(p.shape[0]), e1["inliers"])
    prm = D.make_params(0.02, max_iterations=200)
    e2 = D.extract_planes(cloud, prm, max_planes=2, min_inliers=10)
    r = O.sac_segment(p, 0.02, indices=rem.astype(np.int32), max_iterations=200)
    assert np.array_equal(e2["inliers"][:e2["offsets"][1]], r["inliers"])
    cloud.reset()
    e3 = D.extract_planes(cloud, prm, max_planes=2, min_inliers=10)
    ref = O.extract_planes(p, 0.02, max_planes=2, min_inliers=10, max_iterations=200)
    assert np.array_equal(e3["inliers"], ref["inliers"])
    cloud.close()


def test_pruned_loopback_sharded(gpu_ctx):
    p, _, _ = plane_cloud(40000, 6, seed=99)
    prm = D.make_params(0.02, max_iterations=511, probability=1.0)
    ref = O.extract_planes(p, 0.02, max_planes=6, min_inliers=200, max_iterations=511,
                           probability=1.0)
    world = 2
    ctxs = D.Context.loopback_group(world, 0)
    bounds = [0, 17000, p.shape[0]]
    out, errs = [None] * world, []

    def run(r):
        try:
            c = D.Cloud(ctxs[r], p[bounds[r]:bounds[r + 1]], id_base=int(bounds[r]))
            c.build_spatial()
            out[r] = D.extract_planes(c, prm, max_planes=6, min_inliers=200, capacity=p.shape[0])
            c.close()
        except Exception as e:  # pragma: no cover
            errs.append(e)

    th = [threading.Thread(target=run, args=(r,)) for r in range(world)]
    [t.start() for t in th]
    [t.join() for t in th]
    assert not errs, errs
    for r in range(world):
        assert np.array_equal(out[r]["coeffs"].view(np.uint32), ref["coeffs"].view(np.uint32))
        assert np.array_equal(out[r]["inliers"], ref["inliers"])
    for c in ctxs:
        c.close()


@pytest.mark.slow
def test_pruned_counts_c3_full_size(gpu_ctx):
    """10M-point C3 cloud (spatial copy built at upload), 4096 random hypotheses: the pruned
    kernel's counts equal the exhaustive exact kernel's."""
    from test_score_variants import counts
    p, _, _ = plane_cloud(10_000_000, 20, seed=SEED_BASE + 3)
    cloud = D.Cloud(gpu_ctx, p)
    try:
        for thr in (0.02, 0.2):
            ref = counts(gpu_ctx, cloud, 4096, 1, thr)
            got = counts(gpu_ctx, cloud, 4096, 2, thr)
            assert ref.sum() > 0 and np.array_equal(got, ref), int((got != ref).sum())
    finally:
        cloud.close()


@pytest.mark.parametrize("optimize", [False, True])
def test_lean_list_continue_segment_and_normal_plane(gpu_ctx, optimize):
    """Lean-list rounds (the Morton copy decides the inliers, the list keeps pristine indices)
    run whenever the refit stays on the device: optimize=False here (bit-exact against the
    oracle's optimize-off extraction), and optimize=True with PCL's float refit on the device
    (the unrefined inliers from the pristine-index bitmap).  Extraction continued over several calls equals one call; a plain
    segment and a SACMODEL_NORMAL_PLANE round afterwards read the materialised list; all
    against the oracle."""
    p, _, _ = plane_cloud(40000, 6, seed=41)
    p[::17, 2] = np.nan
    kw = dict(max_iterations=255, probability=1.0, optimize=optimize)
    prm = D.make_params(0.02, **kw)
    ref = O.extract_planes(p, 0.02, max_planes=5, min_inliers=50, **kw)
    cloud = D.Cloud(gpu_ctx, p)
    cloud.build_spatial()
    got = []
    lean = 0
    for k in (2, 2, 1):  # 5 planes over three calls
        e = D.extract_planes(cloud, prm, max_planes=k, min_inliers=50)
        got.append(e["inliers"].copy())
        lean += e["stats"]["lean_rounds"]
    assert lean == 5
    assert np.array_equal(np.concatenate(got), ref["inliers"])
    taken = np.concatenate(got)
    rem = np.setdiff1d(np.arange(p.shape[0]), taken).astype(np.int32)
    # plain segment over the remaining (lean) list: materialised from the pristine copy
    inl, coeff, st = D.segment_cloud(cloud, prm)
    r = O.sac_segment(p, 0.02, indices=rem, **kw)
    same(inl, coeff, st, r)
    # a NORMAL_PLANE round on the same list
    nrm = np.zeros((p.shape[0], 4), np.float32)
    nrm[:, 2] = 1.0
    cloud.set_normals(nrm)  # (resets the cloud)
    e = D.extract_planes(cloud, prm, max_planes=2, min_inliers=50)
    assert np.array_equal(e["inliers"], ref["inliers"][:ref["offsets"][2]])
    npp = D.make_params(0.05, max_iterations=100, model=D.SACMODEL_NORMAL_PLANE,
                        normal_distance_weight=0.1, optimize=optimize)
    e2 = D.extract_planes(cloud, npp, max_planes=1, min_inliers=10)
    # (round 5: a NORMAL_PLANE round is lean too when the pruned NP scorer applies and the list is
    # still lean; either way its inliers are the oracle's)
    assert e2["stats"]["lean_rounds"] in (0, 1)
    rem2 = np.setdiff1d(np.arange(p.shape[0]), e["inliers"]).astype(np.int32)
    r2 = O.sac_segment(p, 0.05, indices=rem2, max_iterations=100, normals=nrm,
                       normal_distance_weight=0.1, optimize=optimize)
    assert np.array_equal(e2["inliers"][:e2["offsets"][1]], r2["inliers"])
    cloud.close()


@pytest.mark.parametrize("optimize", [False, True])
def test_lean_list_indexed_cloud(gpu_ctx, optimize):
    """setIndices clouds: the list's pristine indices differ from the point ids (and from list
    order of the ids when the indices are unsorted); lean rounds with or without the (device) PCL
    refit."""
    p, _, _ = plane_cloud(50000, 5, seed=43)
    rng = np.random.default_rng(9)
    idx = rng.choice(p.shape[0], 30000, replace=False).astype(np.int32)  # unsorted
    kw = dict(max_iterations=200, probability=1.0, optimize=optimize)
    cloud = D.Cloud(gpu_ctx, p, indices=idx)
    cloud.build_spatial()
    e = D.extract_planes(cloud, D.make_params(0.02, **kw), max_planes=4, min_inliers=50)
    ref = O.extract_planes(p[idx], 0.02, max_planes=4, min_inliers=50, **kw)
    assert e["stats"]["lean_rounds"] == e["stats"]["rounds"]
    assert e["n_planes"] == ref["n_planes"] >= 3
    assert np.array_equal(e["coeffs"].view(np.uint32), ref["coeffs"].view(np.uint32))
    assert np.array_equal(e["inliers"], idx[ref["inliers"]])
    cloud.close()


@pytest.mark.parametrize("seed", range(4))
def test_path_options_identical(gpu_ctx, seed):
    """Every execution-path option (dlg_ctx_set_option) gives the same planes and inliers: lean
    vs two-pass selects, speculative vs host pick, pruned vs exhaustive bf16 vs exact VALU
    scoring, Hilbert vs Morton order of the spatial copy -- each against the oracle's optimize-off
    extraction (the paths lean rounds take)."""
    rng = np.random.default_rng(900 + seed)
    p, _, _ = plane_cloud(int(rng.integers(20000, 80000)), int(rng.integers(2, 7)),
                          seed=seed + 300, outlier_frac=float(rng.uniform(0.05, 0.4)))
    if seed % 2:
        p[::29, 1] = np.nan
    kw = dict(max_iterations=int(rng.choice([63, 255, 1023])), probability=1.0, optimize=False)
    ref = O.extract_planes(p, 0.02, max_planes=6, min_inliers=50, **kw)
    prm = D.make_params(0.02, **kw)
    combos = [dict(), {D.DLG_OPT_LEAN_ROUNDS: 0}, {D.DLG_OPT_SPEC_PICK: 0},
              {D.DLG_OPT_PRUNE: 0}, {D.DLG_OPT_PRUNE: 0, D.DLG_OPT_SCORE_KERNEL: D.DLG_SCORE_EXACT},
              {D.DLG_OPT_SELECT_TILE: 4096}, {D.DLG_OPT_SELECT_TILE: 8192},
              {D.DLG_OPT_SELECT_TILE: 16384},
              {D.DLG_OPT_PRUNE_TILE_SCORER: D.DLG_TILE_BF16},
              {D.DLG_OPT_SPATIAL_CURVE: 0}]  # (Morton-ordered copy; the default is Hilbert)
    for opts in combos:
        ctx = D.Context(0)
        try:
            ctx.set_option(D.DLG_OPT_PRUNE, 1)
            for k, v in opts.items():
                ctx.set_option(k, v)
            cloud = D.Cloud(ctx, p)
            e = D.extract_planes(cloud, prm, max_planes=6, min_inliers=50)
            cloud.close()
        finally:
            ctx.close()
        assert e["n_planes"] == ref["n_planes"], opts
        assert np.array_equal(e["coeffs"].view(np.uint32), ref["coeffs"].view(np.uint32)), opts
        assert np.array_equal(e["offsets"], ref["offsets"]) and np.array_equal(e["inliers"], ref["inliers"]), opts
        lean_expected = opts.get(D.DLG_OPT_LEAN_ROUNDS, 1) and opts.get(D.DLG_OPT_PRUNE, 1)
        assert (e["stats"]["lean_rounds"] > 0) == bool(lean_expected), (opts, e["stats"])
