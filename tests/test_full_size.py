"""BASELINE.json full-size configurations on the GPU, checked through size-independent properties
(the oracle is too slow at 10M points x 4096 hypotheses x 20 rounds; bit parity with it is
established at the smaller sizes in test_gpu_parity.py / test_normal_plane.py).

C3: 10M points, 20 planes, 4096 hypotheses per round, extract-and-remove:
  * every extracted plane's inliers satisfy the exact PCL test |(c0 x + c2 z) + (c1 y + c3)| <
    thr (float32 op order) and every point left at the end fails it for every extracted plane
    (each round removed all inliers of its plane from the remaining list);
  * inlier id lists are disjoint, ascending within a plane, inside [0, N);
  * the run is deterministic and a 2-rank sharded run (loopback group) gives identical planes.
"""
import threading

import numpy as np
import pytest

THR = 0.02


def pcl_abs_dist(c, p):
    c = np.asarray(c, np.float32)
    return np.abs((c[0] * p[:, 0] + c[2] * p[:, 2]) + (c[1] * p[:, 1] + c[3] * np.float32(1)))


def cthr(thr):
    f = np.float32(thr)
    if float(f) < thr:
        f = np.nextafter(f, np.float32(np.inf))
    return f


@pytest.fixture(scope="module")
def c3_cloud():
    from dialog_amd.synth import SEED_BASE, plane_cloud
    p, lab, planes = plane_cloud(10_000_000, 20, seed=SEED_BASE + 3)
    return p


def extract(ctx, p, id_base=0, cap=None, fast=True):
    import dialog_amd as D
    cloud = D.Cloud(ctx, p, id_base=id_base)
    prm = D.make_params(THR, max_iterations=4095, probability=1.0,
                        refit_mode=D.DLG_REFIT_FAST if fast else D.DLG_REFIT_PCL,
                        hypotheses_per_launch=4096)
    e = D.extract_planes(cloud, prm, max_planes=20, min_inliers=500, capacity=cap)
    cloud.close()
    return e


@pytest.mark.gpu
@pytest.mark.slow
def test_c3_full_size_properties(gpu_ctx, c3_cloud):
    p = c3_cloud
    n = p.shape[0]
    e = extract(gpu_ctx, p)
    assert e["n_planes"] >= 18
    offs = e["offsets"]
    inl = e["inliers"]
    assert offs[0] == 0 and np.all(np.diff(offs) >= 500)
    assert inl.min() >= 0 and inl.max() < n
    assert np.unique(inl).size == inl.size  # disjoint
    t = cthr(THR)
    for k in range(e["n_planes"]):
        ids = inl[offs[k]:offs[k + 1]]
        assert np.all(np.diff(ids) > 0)  # list order of the remaining indices = ascending
        assert np.all(pcl_abs_dist(e["coeffs"][k], p[ids]) < t)
    left = np.ones(n, bool)
    left[inl] = False
    rest = p[left]
    for k in range(e["n_planes"]):
        assert not np.any(pcl_abs_dist(e["coeffs"][k], rest) < t)
    # deterministic
    e2 = extract(gpu_ctx, p)
    assert np.array_equal(e2["offsets"], offs) and np.array_equal(e2["inliers"], inl)
    assert np.array_equal(e2["coeffs"].view(np.uint32), e["coeffs"].view(np.uint32))


@pytest.mark.gpu
@pytest.mark.slow
def test_c3_full_size_two_rank_shards(gpu_ctx, c3_cloud):
    """The point-sharded path at full size (2 in-process ranks on one GPU), PCL-refit mode (its
    sums run in global list order whatever the sharding): bit-identical to the 1-rank run."""
    import dialog_amd as D
    p = c3_cloud
    ref = extract(gpu_ctx, p, fast=False)
    ctxs = D.Context.loopback_group(2, 0)
    half = p.shape[0] // 2
    out = [None, None]
    errs = []

    def run(r):
        try:
            lo, hi = (0, half) if r == 0 else (half, p.shape[0])
            cloud = D.Cloud(ctxs[r], p[lo:hi], id_base=lo)
            prm = D.make_params(THR, max_iterations=4095, probability=1.0,
                                refit_mode=D.DLG_REFIT_PCL, hypotheses_per_launch=4096)
            out[r] = D.extract_planes(cloud, prm, max_planes=20, min_inliers=500,
                                      capacity=p.shape[0])
            cloud.close()
        except Exception as ex:  # pragma: no cover
            errs.append(ex)

    th = [threading.Thread(target=run, args=(r,)) for r in range(2)]
    [t.start() for t in th]
    [t.join() for t in th]
    assert not errs, errs
    for r in range(2):
        assert np.array_equal(out[r]["offsets"], ref["offsets"])
        assert np.array_equal(out[r]["inliers"], ref["inliers"])
        assert np.array_equal(out[r]["coeffs"].view(np.uint32), ref["coeffs"].view(np.uint32))
    for c in ctxs:
        c.close()
