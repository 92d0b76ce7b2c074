"""GPU (gfx950): the HIP path through the C ABI against the oracle and the golden fixtures.

Bar: bit-exact indices / best sample / iteration counts / coefficients in PCL-refit mode and in
fast-refit mode (the exact-moment LS refit of exact_refit.hpp, restated by the oracle).
"""
import json
import os
import subprocess
import threading

import numpy as np
import pytest

import dialog_amd as D
from dialog_amd.pcd import read_pcd
from dialog_amd.synth import SEED_BASE, plane_cloud
from oracle import oracle as O

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def gpu_segment(ctx, pts, thr, indices=None, refit=D.DLG_REFIT_PCL, **kw):
    cloud = D.Cloud(ctx, pts, indices=indices)
    try:
        prm = D.make_params(thr, refit_mode=refit, **kw)
        return D.segment_cloud(cloud, prm)
    finally:
        cloud.close()


def assert_same_as_oracle(inl, coeff, st, r):
    assert st["has_model"] == r["ok"]
    assert st["iterations"] == r["iterations"], (st["iterations"], r["iterations"])
    assert st["draws"] == r["draws"]
    if not r["ok"]:
        assert inl.size == 0
        return
    assert list(st["best_sample"]) == list(r["best_sample"])
    assert np.array_equal(st["coeff_unrefined"].view(np.uint32), r["coeff_unrefined"].view(np.uint32))
    assert st["n_unrefined"] == r["n_unrefined"]
    assert np.array_equal(coeff.view(np.uint32), r["coeff"].view(np.uint32)), (coeff, r["coeff"])
    assert np.array_equal(inl, r["inliers"])


@pytest.mark.parametrize("name", ["pcl_defaults", "h4096", "pcl_defaults_t02"])
def test_double_shadow_bit_exact(gpu_ctx, golden_dir, name):
    pts = read_pcd(os.path.join(golden_dir, "double_shadow.pcd"))
    g = json.load(open(os.path.join(golden_dir, "double_shadow.json")))["configs"][name]
    kw = {k: g[k] for k in ("max_iterations", "probability") if k in g}
    inl, coeff, st = gpu_segment(gpu_ctx, pts, g["threshold"], **kw)
    assert st["iterations"] == g["iterations"] and st["draws"] == g["draws"]
    assert list(st["best_sample"]) == g["best_sample"]
    assert list(st["coeff_unrefined"].view(np.uint32)) == g["coeff_unrefined_bits"]
    assert list(coeff.view(np.uint32)) == g["coeff_bits"]
    assert list(inl) == g["inliers"]


@pytest.mark.parametrize("name", ["pcl_defaults", "h4096"])
def test_double_shadow_fast_refit(gpu_ctx, golden_dir, name):
    """DLG_REFIT_FAST: bit-exact against the oracle's restatement of the exact-moment refit
    (exact_refit.hpp), and within 1e-5 of the golden two-pass double LS plane."""
    pts = read_pcd(os.path.join(golden_dir, "double_shadow.pcd"))
    g = json.load(open(os.path.join(golden_dir, "double_shadow.json")))["configs"][name]
    kw = {k: g[k] for k in ("max_iterations", "probability") if k in g}
    inl, coeff, st = gpu_segment(gpu_ctx, pts, g["threshold"], refit=D.DLG_REFIT_FAST, **kw)
    r = O.sac_segment(pts, g["threshold"], refit="fast", **kw)
    assert_same_as_oracle(inl, coeff, st, r)
    ref = np.array(g["coeff_double"], np.float32)
    sgn = 1.0 if np.dot(coeff[:3], ref[:3]) >= 0 else -1.0
    assert np.abs(sgn * coeff - ref).max() < 1e-5


def test_synth_c2_small_golden(gpu_ctx, golden_dir):
    z = np.load(os.path.join(golden_dir, "synth_c2_small.npz"))
    inl, coeff, st = gpu_segment(gpu_ctx, z["points"], float(z["threshold"]),
                                 max_iterations=int(z["max_iterations"]),
                                 probability=float(z["probability"]))
    assert st["iterations"] == int(z["iterations"])
    assert np.array_equal(st["best_sample"], z["best_sample"])
    assert np.array_equal(coeff.view(np.uint32), z["coeff"].view(np.uint32))
    assert np.array_equal(inl, z["inliers"])
    assert st["launches"] == 1  # 4096 hypotheses scored in one launch


def test_synth_c3_small_extract_golden(gpu_ctx, golden_dir):
    z = np.load(os.path.join(golden_dir, "synth_c3_small.npz"))
    cloud = D.Cloud(gpu_ctx, z["points"])
    prm = D.make_params(float(z["threshold"]), max_iterations=int(z["max_iterations"]),
                        probability=float(z["probability"]))
    e = D.extract_planes(cloud, prm, max_planes=int(z["max_planes"]), min_inliers=int(z["min_inliers"]))
    assert e["n_planes"] == z["coeffs"].shape[0]
    assert np.array_equal(e["offsets"], z["offsets"])
    assert np.array_equal(e["inliers"], z["inliers"])
    assert np.array_equal(e["coeffs"].view(np.uint32), z["coeffs"].view(np.uint32))
    # the active list shrank by exactly the extracted inliers
    assert cloud.n_active == z["points"].shape[0] - z["offsets"][-1]
    cloud.reset()
    assert cloud.n_active == z["points"].shape[0]
    e2 = D.extract_planes(cloud, prm, max_planes=int(z["max_planes"]), min_inliers=int(z["min_inliers"]))
    assert np.array_equal(e2["inliers"], e["inliers"])  # idempotent after reset
    cloud.close()


@pytest.mark.parametrize("seed", range(12))
def test_random_clouds_vs_oracle(gpu_ctx, seed):
    rng = np.random.default_rng(1000 + seed)
    n = int(rng.choice([3, 4, 5, 17, 100, 1000, 5000, 20000]))
    p, _, _ = plane_cloud(n, int(rng.integers(1, 4)), seed=seed, outlier_frac=float(rng.uniform(0, 0.5)))
    if seed % 3 == 0:  # quantised: duplicates, ties, collinear draws
        p = (np.round(p * 2) / 2).astype(np.float32)
    thr = float(rng.choice([0.005, 0.02, 0.1, 0.25]))
    mi = int(rng.choice([1, 10, 50, 300, 1000, 5000]))
    pr = float(rng.choice([0.9, 0.99, 1.0]))
    r = O.sac_segment(p, thr, max_iterations=mi, probability=pr)
    inl, coeff, st = gpu_segment(gpu_ctx, p, thr, max_iterations=mi, probability=pr)
    assert_same_as_oracle(inl, coeff, st, r)


def test_edge_cases(gpu_ctx):
    for n in (0, 1, 2):
        inl, coeff, st = gpu_segment(gpu_ctx, np.zeros((n, 3), np.float32), 0.1)
        assert not st["has_model"] and inl.size == 0 and not coeff.any()
    t = np.arange(1, 11, dtype=np.float32)
    line = np.stack([t, 2 * t, 4 * t], 1)  # every triple collinear -> no sample in 1000 tries
    inl, coeff, st = gpu_segment(gpu_ctx, line, 0.1)
    r = O.sac_segment(line, 0.1)
    assert not st["has_model"] and st["draws"] == r["draws"] == 1000
    same = np.ones((10, 3), np.float32)  # NaN ratios -> "good" -> degenerate all-inlier plane
    inl, coeff, st = gpu_segment(gpu_ctx, same, 0.1)
    assert_same_as_oracle(inl, coeff, st, O.sac_segment(same, 0.1))
    p = np.random.default_rng(0).random((50, 3)).astype(np.float32)
    inl, coeff, st = gpu_segment(gpu_ctx, p, np.finfo(np.float64).max)
    assert not st["has_model"]
    # pcl::PointXYZ layout (16-byte stride)
    p4 = np.concatenate([p, np.ones((50, 1), np.float32)], 1)
    a = gpu_segment(gpu_ctx, p, 0.05)
    b = gpu_segment(gpu_ctx, p4, 0.05)
    assert np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1])


def test_indices_subset(gpu_ctx):
    rng = np.random.default_rng(5)
    pts = rng.random((3000, 3)).astype(np.float32)
    idx = rng.permutation(3000)[:2000].astype(np.int32)
    r = O.sac_segment(pts, 0.05, indices=idx, max_iterations=200)
    inl, coeff, st = gpu_segment(gpu_ctx, pts, 0.05, indices=idx, max_iterations=200)
    assert_same_as_oracle(inl, coeff, st, r)


def test_pcl_mirror_interface(gpu_ctx):
    p, _, _ = plane_cloud(5000, 2, seed=7)
    seg = D.SACSegmentation(gpu_ctx)
    seg.setOptimizeCoefficients(True)
    seg.setModelType(D.SACMODEL_PLANE)
    seg.setMethodType(D.SAC_RANSAC)
    seg.setDistanceThreshold(0.02)
    seg.setInputCloud(p)
    inl, coeff = seg.segment()
    r = O.sac_segment(p, 0.02)
    assert np.array_equal(inl, r["inliers"]) and np.array_equal(coeff, r["coeff"])


@pytest.mark.parametrize("world", [2, 3])
def test_loopback_sharded_equals_single(gpu_ctx, world):
    """Point-sharded over `world` in-process ranks (own buffers/streams, host-summed collectives):
    identical planes and inliers to the 1-rank run."""
    p, _, _ = plane_cloud(40000, 6, seed=99)
    prm = D.make_params(0.02, max_iterations=511, probability=1.0)
    cloud = D.Cloud(gpu_ctx, p)
    ref = D.extract_planes(cloud, prm, max_planes=6, min_inliers=200)
    cloud.close()
    ctxs = D.Context.loopback_group(world, 0)
    bounds = np.linspace(0, p.shape[0], world + 1).astype(np.int64)
    out = [None] * world
    errs = []

    def run(r):
        try:
            c = D.Cloud(ctxs[r], p[bounds[r]:bounds[r + 1]], id_base=int(bounds[r]))
            out[r] = D.extract_planes(c, prm, max_planes=6, min_inliers=200,
                                      capacity=p.shape[0])
            c.close()
        except Exception as e:  # pragma: no cover
            errs.append(e)

    th = [threading.Thread(target=run, args=(r,)) for r in range(world)]
    [t.start() for t in th]
    [t.join() for t in th]
    assert not errs, errs
    for r in range(world):
        assert out[r]["n_planes"] == ref["n_planes"]
        assert np.array_equal(out[r]["coeffs"].view(np.uint32), ref["coeffs"].view(np.uint32))
        assert np.array_equal(out[r]["offsets"], ref["offsets"])
        assert np.array_equal(out[r]["inliers"], ref["inliers"])
    for c in ctxs:
        c.close()


@pytest.mark.parametrize("world,n,refit,opt", [(2, 40000, "pcl", 1), (3, 300000, "fast", -1),
                                               (5, 200000, "pcl", None)])
def test_loopback_hyp_sharded_equals_oracle(gpu_ctx, world, n, refit, opt):
    """DLG_OPT_HYP_SHARD (SURVEY 8(e)'s small-N fallback): every in-process rank uploads the whole
    cloud and scores its slice of each batch's hypotheses (exhaustive kernels below the Morton
    copy's size, the pruned scorer above it), the counts are allreduced; every rank's segment()
    and extract-and-remove equal the oracle's bit for bit.  opt 1: set explicitly; -1 / None
    (the default): chosen by the library because every rank holds the same cloud (a point-
    sharded run would count each point once per rank and miss the oracle's counts)."""
    p, _, _ = plane_cloud(n, 6, seed=98 + world)
    mode = D.DLG_REFIT_PCL if refit == "pcl" else D.DLG_REFIT_FAST
    prm = D.make_params(0.02, max_iterations=511, probability=1.0, refit_mode=mode)
    ref = O.extract_planes(p, 0.02, max_planes=6, min_inliers=200, max_iterations=511,
                           probability=1.0, refit=refit)
    seg = O.sac_segment(p, 0.02, max_iterations=99, probability=0.99)
    prm_s = D.make_params(0.02, max_iterations=99, probability=0.99, refit_mode=D.DLG_REFIT_PCL)
    ctxs = D.Context.loopback_group(world, 0)
    out, sout, errs = [None] * world, [None] * world, []

    def run(r):
        try:
            if opt is not None:
                ctxs[r].set_option(D.DLG_OPT_HYP_SHARD, opt)
            c = D.Cloud(ctxs[r], p)
            out[r] = D.extract_planes(c, prm, max_planes=6, min_inliers=200, capacity=p.shape[0])
            c.reset()
            sout[r] = D.segment_cloud(c, prm_s, capacity=p.shape[0])
            c.close()
        except Exception as e:  # pragma: no cover
            errs.append(e)

    th = [threading.Thread(target=run, args=(r,)) for r in range(world)]
    [t.start() for t in th]
    [t.join() for t in th]
    for c in ctxs:
        c.close()
    assert not errs, errs
    for r in range(world):
        assert out[r]["n_planes"] == ref["n_planes"] >= 4
        assert np.array_equal(out[r]["coeffs"].view(np.uint32), ref["coeffs"].view(np.uint32))
        assert np.array_equal(out[r]["offsets"], ref["offsets"])
        assert np.array_equal(out[r]["inliers"], ref["inliers"])
        inl, coeff, st = sout[r]
        assert list(st["best_sample"]) == list(seg["best_sample"])
        assert np.array_equal(coeff.view(np.uint32), seg["coeff"].view(np.uint32))
        assert np.array_equal(inl, seg["inliers"])


@pytest.mark.slow
def test_large_cloud_properties(gpu_ctx):
    """1M-point C2 cloud: bit parity with the oracle on a bounded hypothesis budget, and
    size-independent properties of a full extract-and-remove run."""
    p, lab, planes = plane_cloud(1_000_000, 3, shares=[1, 1, 1], seed=SEED_BASE + 2)
    r = O.sac_segment(p, 0.02, max_iterations=63, probability=1.0)
    inl, coeff, st = gpu_segment(gpu_ctx, p, 0.02, max_iterations=63, probability=1.0)
    assert_same_as_oracle(inl, coeff, st, r)
    cloud = D.Cloud(gpu_ctx, p)
    prm = D.make_params(0.02, max_iterations=4095, probability=1.0, refit_mode=D.DLG_REFIT_FAST)
    e = D.extract_planes(cloud, prm, max_planes=5, min_inliers=500)
    assert e["n_planes"] >= 3  # later rounds may still find >= 500 outliers on some slab
    ids = e["inliers"]
    assert np.unique(ids).size == ids.size  # planes are disjoint
    for k in range(e["n_planes"]):
        s = ids[e["offsets"][k]:e["offsets"][k + 1]]
        assert np.all(np.diff(s) > 0)  # list order == ascending ids
        c = e["coeffs"][k]
        d = np.abs((c[0] * p[s, 0] + c[2] * p[s, 2]) + (c[1] * p[s, 1] + c[3]))
        assert np.all(d.astype(np.float64) < 0.02)
        if k < 3:  # the three generator planes come out first (they hold 30 % each)
            assert np.max(np.abs(planes[:, :3] @ c[:3])) > 0.999
    assert cloud.n_active == p.shape[0] - ids.size
    cloud.close()


def test_cpp_shim_runs_on_gpu(tmp_path):
    exe = tmp_path / "shim_smoke"
    lib = os.path.dirname(D.LIB_PATH)
    subprocess.run(["g++", "-std=c++17", "-O1", "-I", os.path.join(ROOT, "include"),
                    os.path.join(ROOT, "tests", "cpp", "shim_smoke.cpp"), "-o", str(exe), "-L", lib,
                    "-ldialog_amd", f"-Wl,-rpath,{lib}"], check=True)
    out = subprocess.run([str(exe)], capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stderr
    assert out.stdout.startswith("coeff ")
    lines = dict(ln.split(" ", 1) for ln in out.stdout.strip().splitlines())
    nrm = lines["normals"].split()
    assert int(nrm[0]) == 64 * 64 + 500 and int(nrm[2]) > 0 and int(nrm[4]) > 0
    pre = lines["preprocess"].split()
    assert 0 < int(pre[0]) == int(pre[1]) < 64 * 64 + 500
    post = [int(x) for x in lines["postprocess"].split()]
    assert post[0] > 64 * 32 and post[2] == 4 and post[3] == 1
    assert post[0] + post[1] <= 64 * 64 + 500


def test_cpp_plane_clouds_glue_runs_on_gpu(tmp_path):
    """INTEGRATION.md §3's segmentPlanesRansac() compiled against the shim with the reference's
    struct Plane (HeaderFile.h:81-88): six box faces -> six planes whose coeff.values are the
    3-component outward normals and whose border is left for polyPlanes (PlaneDetect.h:1364)."""
    exe = tmp_path / "plane_clouds_glue"
    lib = os.path.dirname(D.LIB_PATH)
    subprocess.run(["g++", "-std=c++17", "-O1", "-I", os.path.join(ROOT, "include"),
                    os.path.join(ROOT, "tests", "cpp", "plane_clouds_glue.cpp"), "-o", str(exe),
                    "-L", lib, "-ldialog_amd", f"-Wl,-rpath,{lib}"], check=True)
    out = subprocess.run([str(exe)], capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, (out.stdout, out.stderr)
    assert out.stdout.strip() == "planes 6 bad 0"


def test_rccl_one_rank_path(gpu_ctx):
    """The RCCL communicator code (dlopen, ncclCommInitRank, in-place allreduce, allgather,
    allreduce-max) on a real device with one rank (world 1 + a unique id): same planes as the
    plain context."""
    p, _, _ = plane_cloud(30000, 4, seed=5)
    prm = D.make_params(0.02, max_iterations=255, probability=1.0)
    c0 = D.Cloud(gpu_ctx, p)
    ref = D.extract_planes(c0, prm, max_planes=4, min_inliers=100)
    c0.close()
    uid = D.Context.unique_id()
    ctx = D.Context.distributed(0, 0, 1, uid)
    assert ctx.world == 1
    c1 = D.Cloud(ctx, p)
    out = D.extract_planes(c1, prm, max_planes=4, min_inliers=100)
    assert np.array_equal(out["inliers"], ref["inliers"])
    assert np.array_equal(out["coeffs"].view(np.uint32), ref["coeffs"].view(np.uint32))
    assert ctx.allreduce_max(3.5) == 3.5
    ctx.barrier()
    c1.close()
    ctx.close()


@pytest.mark.parametrize("mi", [0, 5, 50, 400])
def test_probability_one_bad_draws(gpu_ctx, mi):
    """probability = 1 rounds take the speculative device pick (k_pick_p1); with many bad
    (collinear) draws the batch of max_iterations + 1 draws cannot finish PCL's loop, so the
    host replay overturns the pick and the round continues on the exact path.  Both must equal
    the PCL restatement (iterations, draws, best sample, coefficients, inliers)."""
    rng = np.random.default_rng(77 + mi)
    t = rng.random(60).astype(np.float32)
    line = np.stack([t, 2 * t, 4 * t], 1)  # collinear triples: isSampleGood false
    off = rng.random((12, 3)).astype(np.float32)  # a few points off the line
    p = np.concatenate([line, off]).astype(np.float32)
    r = O.sac_segment(p, 0.05, max_iterations=mi, probability=1.0)
    inl, coeff, st = gpu_segment(gpu_ctx, p, 0.05, max_iterations=mi, probability=1.0)
    assert_same_as_oracle(inl, coeff, st, r)
    assert st["draws"] > mi + 1 or not r["ok"]  # bad draws were consumed beyond one batch


def test_probability_one_extract_rounds(gpu_ctx):
    """extract-and-remove with probability 1 (every round speculative) equals the oracle's
    sequential extraction, with the refined planes and inliers bit-identical."""
    p, _, _ = plane_cloud(6000, 4, seed=99, outlier_frac=0.2)
    prm = D.make_params(0.02, max_iterations=255, probability=1.0)
    cloud = D.Cloud(gpu_ctx, p)
    try:
        e = D.extract_planes(cloud, prm, max_planes=5, min_inliers=50)
    finally:
        cloud.close()
    r = O.extract_planes(p, 0.02, max_planes=5, min_inliers=50, max_iterations=255, probability=1.0)
    assert e["n_planes"] == r["n_planes"]
    assert np.array_equal(e["coeffs"].view(np.uint32), r["coeffs"].view(np.uint32))
    assert np.array_equal(e["offsets"], r["offsets"]) and np.array_equal(e["inliers"], r["inliers"])
