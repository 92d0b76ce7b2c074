"""GPU: DLG_REFIT_PCL with PCL's float sums on the device (fsum.hip) against the oracle, bit for bit.

The oracle (oracle/pcl_oracle.c) refits with the literal single-pass float loop of
computeMeanAndCovarianceMatrix (list order) and PCL's float eigen33.  The device takes the
unrefined inliers in list order (lean rounds: a bitmap over pristine indices; otherwise the
two-pass select), evaluates the nine sequential sums by the fan/translation hierarchy of fsum.hpp
and runs eigen33 on the device.  Cases:
  * extract-and-remove over random clouds above and below the Morton-copy threshold, with the
    lean rounds on and off, the host-sum path (DLG_OPT_PCL_REFIT_DEVICE 0), the host
    verification of every refit tail (2) and the forced redo of every select (3);
  * clouds whose sums hover around zero (planes through the origin), far from the origin
    (large sums), quantised coordinates (rounding ties), NaN points;
  * a single segment() with > 524288 inliers, so the records take a third level (k_fs_level);
  * SACMODEL_NORMAL_PLANE with the PCL refit (the non-lean device path).
"""
import numpy as np
import pytest

import dialog_amd as D
from dialog_amd.synth import plane_cloud
from oracle import oracle as O

pytestmark = pytest.mark.gpu


def bits(a):
    return np.ascontiguousarray(a, np.float32).view(np.uint32)


def extract(p, prm, opts, max_planes, min_inliers, prune=None):
    ctx = D.Context(0)
    try:
        if prune is not None:
            ctx.set_option(D.DLG_OPT_PRUNE, prune)
        for k, v in opts.items():
            ctx.set_option(k, v)
        cl = D.Cloud(ctx, p)
        e = D.extract_planes(cl, prm, max_planes=max_planes, min_inliers=min_inliers)
        cl.close()
    finally:
        ctx.close()
    return e


def check(e, ref, tag):
    assert e["n_planes"] == ref["n_planes"], tag
    assert np.array_equal(bits(e["coeffs"]), bits(ref["coeffs"])), (tag, e["coeffs"], ref["coeffs"])
    assert np.array_equal(e["offsets"], ref["offsets"]), tag
    assert np.array_equal(e["inliers"], ref["inliers"]), tag


# (DLG_OPT_UNREFINED_LIST 0: the lean rounds' unrefined inliers from the Morton copy's stamps and
# the bitmap compaction instead of the default list pass)
OPTS = [dict(), {D.DLG_OPT_LEAN_ROUNDS: 0}, {D.DLG_OPT_PCL_REFIT_DEVICE: 0},
        {D.DLG_OPT_PCL_REFIT_DEVICE: 2}, {D.DLG_OPT_PCL_REFIT_DEVICE: 3},
        {D.DLG_OPT_UNREFINED_LIST: 0}]


@pytest.mark.parametrize("seed", range(4))
def test_extract_pcl_matches_oracle_every_path(seed):
    rng = np.random.default_rng(4100 + seed)
    n = int(rng.integers(150000, 400000)) if seed % 2 == 0 else int(rng.integers(20000, 90000))
    p, _, _ = plane_cloud(n, int(rng.integers(2, 8)), seed=seed + 880,
                          outlier_frac=float(rng.uniform(0.05, 0.3)))
    if seed == 3:
        p[::31, 2] = np.nan
    kw = dict(max_iterations=int(rng.choice([255, 1023])), probability=1.0)
    ref = O.extract_planes(p, 0.02, max_planes=8, min_inliers=100, **kw)
    prm = D.make_params(0.02, **kw)
    for opts in OPTS:
        e = extract(p, prm, opts, 8, 100, prune=1 if seed % 2 else None)
        check(e, ref, opts)
        st = e["stats"]
        lean = opts.get(D.DLG_OPT_LEAN_ROUNDS, 1) and opts.get(D.DLG_OPT_PCL_REFIT_DEVICE, 1)
        assert (st["lean_rounds"] >= e["n_planes"] > 0) == bool(lean), (opts, st)
        if opts.get(D.DLG_OPT_PCL_REFIT_DEVICE, 1) >= 2:
            assert e["n_planes"] <= st["pcl_host_checks"] <= st["rounds"], st


@pytest.mark.parametrize("case", ["origin", "far", "quantised", "tiny"])
def test_extract_pcl_adversarial_sums(case):
    """Sums that hover around zero and change binade often (planes through the origin), huge
    sums (a cloud 3000 units out), rounding ties on every step (coordinates on a 1/64 grid), and
    sub-millimetre scales."""
    rng = np.random.default_rng(77)
    p, _, planes = plane_cloud(300000, 5, seed=4242 + len(case), outlier_frac=0.05)
    if case == "origin":
        # move every plane's patch to pass through the origin: the x, y, z, xy, ... sums hover
        p64 = p.astype(np.float64)
        for k in range(5):
            nrm = planes[k, :3].astype(np.float64)
            d = p64 @ nrm + planes[k, 3]
            sel = np.abs(d) < 0.05
            p64[sel] += float(planes[k, 3]) * nrm  # (n.p + d = 0) -> (n.p' = 0)
        p = p64.astype(np.float32)
    elif case == "far":
        p = (p + np.float32(3000.0)).astype(np.float32)
    elif case == "quantised":
        p = (np.round(p * 64) / 64).astype(np.float32)
    else:
        p = (p * np.float32(1e-4)).astype(np.float32)
    thr = 2e-6 if case == "tiny" else 0.02
    kw = dict(max_iterations=511, probability=1.0)
    ref = O.extract_planes(p, thr, max_planes=6, min_inliers=200, **kw)
    assert ref["n_planes"] >= 2
    prm = D.make_params(thr, **kw)
    # (DLG_OPT_FS_POISON: the window tables hold garbage stamped for the next launch until the
    # clear after the scratch is laid out; results unchanged)
    for opts in (dict(), {D.DLG_OPT_LEAN_ROUNDS: 0}, {D.DLG_OPT_FS_POISON: 1},
                 {D.DLG_OPT_UNREFINED_LIST: 0}):
        check(extract(p, prm, opts, 6, 200), ref, (case, opts))


def test_segment_pcl_three_levels(gpu_ctx):
    """One segment() with ~1.4M inliers: more than 64 units of 4096 (the unit scans run over
    several windows) and ~22k chunk records per chain for the walk."""
    p, _, _ = plane_cloud(1_600_000, 1, seed=515, outlier_frac=0.1)
    kw = dict(max_iterations=255, probability=1.0)
    ref = O.sac_segment(p, 0.02, **kw)
    cl = D.Cloud(gpu_ctx, p)
    inl, coeff, st = D.segment_cloud(cl, D.make_params(0.02, **kw))
    cl.close()
    assert st["n_unrefined"] == ref["n_unrefined"] > 524288
    assert np.array_equal(bits(coeff), bits(ref["coeff"])), (coeff, ref["coeff"])
    assert np.array_equal(inl, ref["inliers"])


@pytest.mark.parametrize("world,lean,proto", [(2, 1, 0), (3, 1, 0), (3, 0, 0), (3, 1, 1),
                                              (3, 0, 1), (3, 1, 2), (3, 0, 2)])
def test_extract_pcl_sharded(world, lean, proto):
    """The PCL refit over in-process ranks (one shard empty in one case), every protocol of
    DLG_OPT_FS_ONE_WALK: 0 = walk from the guess, rebase on the propagated guess, walk again,
    repairs rank after rank; 1 = round 4's (no rebase); 2 = 0 with parallel repair iterations
    and host checks.  == the one-rank oracle."""
    import threading
    rng = np.random.default_rng(70 + world + lean)
    n = int(rng.integers(300000, 500000))
    p, _, _ = plane_cloud(n, 5, seed=world * 10 + lean, outlier_frac=0.15)
    kw = dict(max_iterations=511, probability=1.0)
    ref = O.extract_planes(p, 0.02, max_planes=6, min_inliers=200, **kw)
    cuts = sorted(rng.integers(150000, n - 150000, world - 1).tolist())
    if world == 3 and not lean:
        cuts = [cuts[0], cuts[0]]  # (an empty middle shard)
    b = [0, *cuts, n]
    ctxs = D.Context.loopback_group(world, 0)
    out, errs = [None] * world, []

    def run(r):
        try:
            ctxs[r].set_option(D.DLG_OPT_LEAN_ROUNDS, lean)
            ctxs[r].set_option(D.DLG_OPT_FS_ONE_WALK, proto)
            c = D.Cloud(ctxs[r], p[b[r]:b[r + 1]], id_base=b[r])
            out[r] = D.extract_planes(c, D.make_params(0.02, **kw), max_planes=6, min_inliers=200,
                                      capacity=n)
            c.close()
        except Exception as ex:  # pragma: no cover
            errs.append(ex)

    th = [threading.Thread(target=run, args=(r,)) for r in range(world)]
    [t.start() for t in th]
    [t.join() for t in th]
    for c in ctxs:
        c.close()
    assert not errs, errs
    for r in range(world):
        check(out[r], ref, (world, lean, proto, r))


def test_normal_plane_pcl_refit_device():
    """SACMODEL_NORMAL_PLANE extraction with the PCL refit: the two-pass select's inlier xyz feed
    the device sums (no host round trip); == the oracle, and == the host-sum path."""
    rng = np.random.default_rng(3)
    p, lab, planes = plane_cloud(60000, 3, seed=919, outlier_frac=0.1)
    nrm = np.zeros((p.shape[0], 4), np.float32)
    for k in range(3):
        nrm[lab == k, :3] = planes[k, :3]
    nrm[lab < 0, :3] = rng.normal(size=((lab < 0).sum(), 3))
    nrm[:, :3] /= np.linalg.norm(nrm[:, :3], axis=1, keepdims=True)
    nrm[:, 3] = np.abs(rng.normal(0, 0.01, p.shape[0]))
    kw = dict(max_iterations=255, probability=1.0)
    ref = O.extract_planes(p, 0.05, max_planes=3, min_inliers=100, normals=nrm, **kw)
    prm = D.make_params(0.05, model=D.SACMODEL_NORMAL_PLANE, **kw)
    for opts in (dict(), {D.DLG_OPT_PCL_REFIT_DEVICE: 0}):
        ctx = D.Context(0)
        for k, v in opts.items():
            ctx.set_option(k, v)
        cl = D.Cloud(ctx, p)
        cl.set_normals(nrm)
        e = D.extract_planes(cl, prm, max_planes=3, min_inliers=100)
        cl.close()
        ctx.close()
        check(e, ref, opts)
