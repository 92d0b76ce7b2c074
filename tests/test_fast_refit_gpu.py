"""GPU: DLG_REFIT_FAST (the exact-moment refit, dialog_amd/csrc/exact_refit.hpp) bit-exact against
the oracle's restatement (refit="fast") -- the mode the headline bench runs.

The moments are exact integers, so the refined plane depends only on the inlier set: the lean
rounds (moments over the Morton copy), the two-pass rounds (list order), any grid and any rank
count give the same bits.  Checked here: random clouds (segment and extract-and-remove), every
execution-path option, a 2- and 3-rank point-sharded group, NaN points, setIndices clouds.
"""
import threading

import numpy as np
import pytest

import dialog_amd as D
from dialog_amd.synth import plane_cloud
from oracle import oracle as O

pytestmark = pytest.mark.gpu


def same(e, r):
    assert e["n_planes"] == r["n_planes"]
    assert np.array_equal(e["coeffs"].view(np.uint32), r["coeffs"].view(np.uint32))
    assert np.array_equal(e["offsets"], r["offsets"])
    assert np.array_equal(e["inliers"], r["inliers"])


def cloud_case(seed):
    rng = np.random.default_rng(7000 + seed)
    n = int(rng.choice([1000, 20000, 60000, 150000, 300000]))
    p, _, _ = plane_cloud(n, int(rng.integers(2, 8)), seed=seed + 5,
                          outlier_frac=float(rng.uniform(0.0, 0.4)))
    if seed % 3 == 1:
        p[::13, 1] = np.nan
    if seed % 4 == 2:
        p = (p + np.float32(rng.uniform(-200, 200))).astype(np.float32)
    kw = dict(max_iterations=int(rng.choice([50, 255, 1023, 4095])),
              probability=float(rng.choice([0.99, 1.0])))
    thr = float(rng.choice([0.01, 0.02, 0.05]))
    return p, thr, kw


@pytest.mark.parametrize("seed", range(10))
def test_fast_segment_vs_oracle(gpu_ctx, seed):
    p, thr, kw = cloud_case(seed)
    r = O.sac_segment(p, thr, refit="fast", **kw)
    cloud = D.Cloud(gpu_ctx, p)
    inl, coeff, st = D.segment_cloud(cloud, D.make_params(thr, refit_mode=D.DLG_REFIT_FAST, **kw))
    cloud.close()
    assert st["has_model"] == r["ok"] and st["iterations"] == r["iterations"]
    assert list(st["best_sample"]) == list(r["best_sample"])
    assert np.array_equal(coeff.view(np.uint32), r["coeff"].view(np.uint32)), (coeff, r["coeff"])
    assert np.array_equal(inl, r["inliers"])


@pytest.mark.parametrize("seed", range(8))
def test_fast_extract_vs_oracle_all_paths(seed):
    p, thr, kw = cloud_case(100 + seed)
    r = O.extract_planes(p, thr, max_planes=8, min_inliers=30, refit="fast", **kw)
    combos = [dict(), {D.DLG_OPT_LEAN_ROUNDS: 0}, {D.DLG_OPT_SPEC_PICK: 0}, {D.DLG_OPT_PRUNE: 0},
              {D.DLG_OPT_PRUNE: 1}]
    for opts in combos:
        ctx = D.Context(0)
        try:
            for k, v in opts.items():
                ctx.set_option(k, v)
            cloud = D.Cloud(ctx, p)
            e = D.extract_planes(cloud, D.make_params(thr, refit_mode=D.DLG_REFIT_FAST, **kw),
                                 max_planes=8, min_inliers=30)
            cloud.close()
        finally:
            ctx.close()
        same(e, r)


@pytest.mark.parametrize("world", [2, 3])
def test_fast_extract_sharded_equals_oracle(world):
    """Point-sharded ranks (in-process group on one GPU): the int64 moment digits are summed
    across ranks, so the sharded fast refit equals the one-rank one and the oracle's."""
    p, _, _ = plane_cloud(90000 + world, 5, seed=31 + world, outlier_frac=0.2)
    kw = dict(max_iterations=511, probability=1.0)
    r = O.extract_planes(p, 0.02, max_planes=6, min_inliers=50, refit="fast", **kw)
    ctxs = D.Context.loopback_group(world, 0)
    bounds = np.linspace(0, p.shape[0], world + 1).astype(int)
    out, errs = [None] * world, []

    def run(k):
        try:
            lo, hi = bounds[k], bounds[k + 1]
            cloud = D.Cloud(ctxs[k], p[lo:hi], id_base=int(lo))
            prm = D.make_params(0.02, refit_mode=D.DLG_REFIT_FAST, **kw)
            out[k] = D.extract_planes(cloud, prm, max_planes=6, min_inliers=50,
                                      capacity=p.shape[0])
            cloud.close()
        except Exception as ex:  # pragma: no cover
            errs.append(ex)

    th = [threading.Thread(target=run, args=(k,)) for k in range(world)]
    [t.start() for t in th]
    [t.join() for t in th]
    for c in ctxs:
        c.close()
    assert not errs, errs
    for k in range(world):
        same(out[k], r)


def test_fast_indexed_cloud(gpu_ctx):
    """setIndices: the quantum comes from the indexed points (the uploaded cloud)."""
    p, _, _ = plane_cloud(80000, 4, seed=61)
    rng = np.random.default_rng(3)
    idx = rng.choice(p.shape[0], 50000, replace=False).astype(np.int32)
    kw = dict(max_iterations=300, probability=1.0)
    cloud = D.Cloud(gpu_ctx, p, indices=idx)
    e = D.extract_planes(cloud, D.make_params(0.02, refit_mode=D.DLG_REFIT_FAST, **kw),
                         max_planes=4, min_inliers=50)
    cloud.close()
    r = O.extract_planes(p[idx], 0.02, max_planes=4, min_inliers=50, refit="fast", **kw)
    assert e["n_planes"] == r["n_planes"] >= 3
    assert np.array_equal(e["coeffs"].view(np.uint32), r["coeffs"].view(np.uint32))
    assert np.array_equal(e["inliers"], idx[r["inliers"]])
