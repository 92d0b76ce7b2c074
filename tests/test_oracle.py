"""CPU: the oracle (PCL-1.8 restatement) against the golden vectors and its independent numpy twin.

Pinning: the RNG stream is pinned by two MT19937 implementations independent of the oracle
(tests/golden/rng_kat.json); the PCL arithmetic is cross-checked C-vs-numpy ("parity unpinned"
against PCL itself, which is not available -- see DESIGN.md).
"""
import json
import os

import numpy as np
import pytest
from hypothesis import given, settings
from hypothesis import strategies as st

from dialog_amd.pcd import read_pcd
from dialog_amd.synth import SEED_BASE, plane_cloud
from oracle import numpy_twin as T
from oracle import oracle as O


def test_rng_kat_matches_two_independent_mt19937(golden_dir):
    kat = json.load(open(os.path.join(golden_dir, "rng_kat.json")))
    n = len(kat["mt19937_raw"])
    assert [int(v) for v in O.mt_stream(n)] == kat["mt19937_raw"]
    assert [int(v) for v in O.rnd_stream(n)] == kat["rnd"]
    assert kat["rnd"][:5] == [1996335345, 1911592690, 679411342, 280691776, 394962642]
    r = T.Rnd(12345)
    assert [r() for _ in range(n)] == kat["rnd"]


@pytest.mark.parametrize("name", ["pcl_defaults", "h4096", "pcl_defaults_t02"])
def test_oracle_reproduces_double_shadow_golden(golden_dir, name):
    pts = read_pcd(os.path.join(golden_dir, "double_shadow.pcd"))
    g = json.load(open(os.path.join(golden_dir, "double_shadow.json")))["configs"][name]
    kw = {k: g[k] for k in ("max_iterations", "probability") if k in g}
    r = O.sac_segment(pts, g["threshold"], **kw)
    assert r["iterations"] == g["iterations"] and r["draws"] == g["draws"]
    assert list(r["best_sample"]) == g["best_sample"]
    assert list(r["coeff_unrefined"].view(np.uint32)) == g["coeff_unrefined_bits"]
    assert list(r["coeff"].view(np.uint32)) == g["coeff_bits"]
    assert list(r["inliers"]) == g["inliers"]
    rd = O.sac_segment(pts, g["threshold"], refit_double=True, **kw)
    assert list(rd["inliers"]) == g["inliers_double"]


def test_oracle_reproduces_synth_golden(golden_dir):
    z = np.load(os.path.join(golden_dir, "synth_c2_small.npz"))
    r = O.sac_segment(z["points"], float(z["threshold"]), max_iterations=int(z["max_iterations"]),
                      probability=float(z["probability"]))
    assert np.array_equal(r["best_sample"], z["best_sample"])
    assert np.array_equal(r["coeff"].view(np.uint32), z["coeff"].view(np.uint32))
    assert np.array_equal(r["inliers"], z["inliers"])
    z3 = np.load(os.path.join(golden_dir, "synth_c3_small.npz"))
    e = O.extract_planes(z3["points"], float(z3["threshold"]), max_planes=int(z3["max_planes"]),
                         min_inliers=int(z3["min_inliers"]), max_iterations=int(z3["max_iterations"]),
                         probability=float(z3["probability"]))
    assert np.array_equal(e["offsets"], z3["offsets"])
    assert np.array_equal(e["inliers"], z3["inliers"])
    assert np.array_equal(e["coeffs"].view(np.uint32), z3["coeffs"].view(np.uint32))


def test_synth_generator_is_deterministic(golden_dir):
    z = np.load(os.path.join(golden_dir, "synth_c2_small.npz"))
    p, _, _ = plane_cloud(16384, 3, shares=[1, 1, 1], seed=SEED_BASE + 2)
    assert np.array_equal(p, z["points"])


def test_edge_cases_no_model():
    # fewer than 3 points: getSamples fails -> no model (empty indices/values in PCL)
    for n in (0, 1, 2):
        r = O.sac_segment(np.zeros((n, 3), np.float32), 0.1)
        assert not r["ok"] and r["inliers"].size == 0 and not r["coeff"].any()
    # every triple collinear (equal ratios) -> 1000 failed getSamples tries -> no model
    t = np.arange(1, 11, dtype=np.float32)
    line = np.stack([t, 2 * t, 4 * t], 1)
    r = O.sac_segment(line, 0.1)
    assert not r["ok"] and r["draws"] == 1000
    # identical points: 0/0 = NaN ratios make the sample "good" (IEEE), the cross product is 0 and
    # Eigen 3.3's normalize() leaves it 0 -> degenerate plane (0,0,0,0) holding every point (w = 1
    # ends the loop after one iteration); the refit of a zero covariance divides 0/0 in eigen33 ->
    # NaN coefficients -> the re-selection keeps no inlier.  PCL returns exactly that.
    r = O.sac_segment(np.ones((10, 3), np.float32), 0.1)
    assert r["ok"] and r["n_unrefined"] == 10 and r["iterations"] == 1
    assert not r["coeff_unrefined"].any() and np.isnan(r["coeff"]).all() and r["inliers"].size == 0
    # threshold left at DBL_MAX -> "No threshold set!"
    r = O.sac_segment(np.random.default_rng(0).random((50, 3), np.float32), np.finfo(np.float64).max)
    assert not r["ok"]


def test_collinear_points_rejected_and_twin_agrees():
    t = np.linspace(0, 1, 40, dtype=np.float32)
    line = np.stack([t, 2 * t, 3 * t], 1).astype(np.float32)
    off = np.random.default_rng(3).random((10, 3)).astype(np.float32)
    pts = np.concatenate([line, off])
    r = O.sac_segment(pts, 0.01)
    tw = T.sac_segment(pts, 0.01)
    assert r["draws"] == tw["draws"] and r["iterations"] == tw["iterations"]
    assert np.array_equal(r["inliers"], tw["inliers"])


def test_thr_ceil_semantics():
    for thr in (0.1, 0.02, 0.005, 1.0, 1e-30, 3.0e38):
        c = O.thr_ceil(thr)
        assert float(c) >= thr
        below = np.nextafter(c, np.float32(0))
        assert float(below) < thr


def test_indices_subset_and_order():
    rng = np.random.default_rng(5)
    pts = rng.random((300, 3)).astype(np.float32)
    idx = rng.permutation(300)[:200].astype(np.int32)  # unsorted subset (pcl setIndices)
    r = O.sac_segment(pts, 0.05, indices=idx)
    tw = T.sac_segment(pts, 0.05, indices=idx)
    assert np.array_equal(r["inliers"], tw["inliers"])
    assert set(r["inliers"]).issubset(set(idx))
    pos = {v: i for i, v in enumerate(idx)}
    assert all(pos[a] < pos[b] for a, b in zip(r["inliers"][:-1], r["inliers"][1:]))


@settings(max_examples=25, deadline=None)
@given(n=st.integers(3, 400), seed=st.integers(0, 2**31 - 1),
       thr=st.sampled_from([0.005, 0.02, 0.1]), quant=st.booleans())
def test_oracle_matches_numpy_twin(n, seed, thr, quant):
    rng = np.random.default_rng(seed)
    p, _, _ = plane_cloud(n, 2, seed=seed, outlier_frac=0.3)
    if quant:  # quantised coordinates: duplicates, ties, collinear triples
        p = (np.round(p * 4) / 4).astype(np.float32)
    mi = int(rng.integers(1, 80))
    r = O.sac_segment(p, thr, max_iterations=mi)
    tw = T.sac_segment(p, thr, max_iterations=mi)
    assert r["ok"] == tw["ok"] and r["draws"] == tw["draws"]
    assert r["iterations"] == tw["iterations"]
    if r["ok"]:
        assert np.array_equal(r["best_sample"], tw["best_sample"])
        assert np.array_equal(r["coeff_unrefined"].view(np.uint32), tw["coeff_unrefined"].view(np.uint32))
        assert r["n_unrefined"] == tw["n_unrefined"]
        assert np.allclose(r["coeff"], tw["coeff"], atol=1e-5)


def test_normals_and_regulate_on_planes():
    p, lab, planes = plane_cloud(3000, 2, seed=11, sigma=0.0005, outlier_frac=0.0)
    nrm = O.estimate_normals(p, 0.5)
    ok = ~np.isnan(nrm[:, 0])
    assert ok.mean() > 0.95
    for k in range(2):
        m = ok & (lab == k)
        dots = np.abs(nrm[m, :3] @ planes[k, :3])
        assert np.median(dots) > 0.999
    # viewpoint flip: (vp - p) . n >= 0
    assert np.all(np.einsum("ij,ij->i", -p[ok], nrm[ok, :3]) >= -1e-6)
    seed_idx = int(np.flatnonzero(lab == 0)[0])
    reg, proc, cnt = O.regulate_normals(p, nrm, seed_idx, True, 0.3)
    assert cnt == proc.sum() and proc[seed_idx]
    m = proc & (lab == 0) & ok
    # after BFS every processed normal of the seed's plane agrees in sign with the seed
    assert np.all(reg[m, :3] @ reg[seed_idx, :3] > 0)


@pytest.mark.parametrize("kind", ["planes", "quantized", "lattice", "duplicates", "line"])
def test_knn_grid_equals_brute_force(kind):
    """The oracle's k-NN normals search a uniform grid in Chebyshev shells (what full-size clouds
    use); the O(n^2) brute-force form is the definition (k smallest (dist2, index) pairs).  Equal
    bits on clouds built for ties: quantised coordinates, a lattice, duplicated points, a line."""
    rng = np.random.default_rng(0)
    if kind == "planes":
        p, _, _ = plane_cloud(5000, 4, seed=3, patch=2.0)
    elif kind == "quantized":
        p = (np.round(rng.uniform(0, 1, (3000, 3)) * 20) / 20).astype(np.float32)
    elif kind == "lattice":
        p = (np.stack(np.meshgrid(*[np.arange(11)] * 3), -1).reshape(-1, 3) * 0.5).astype(np.float32)
    elif kind == "duplicates":
        p = np.repeat(rng.uniform(0, 1, (400, 3)), 5, axis=0).astype(np.float32)
    else:
        p = np.zeros((2000, 3), np.float32)
        p[:, 0] = np.arange(2000) * 0.01
    for k in (3, 8, 20):
        a = O.estimate_normals_knn(p, k)
        b = O.estimate_normals_knn(p, k, brute=True)
        assert np.array_equal(a.view(np.uint32), b.view(np.uint32)), k
