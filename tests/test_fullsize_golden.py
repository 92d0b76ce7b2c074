"""GPU at BASELINE.json's full sizes against the oracle's full-size results
(tests/golden/fullsize.json, made by tests/golden/make_fullsize.py in the build container):

  c2       1M points, 3 planes, one segment() of 4096 hypotheses (configs[1])   pcl, fast refit
  c3       10M points, 20 planes, extract-and-remove (configs[2], the bench)    fast, pcl, none
  c4shape  100M points, 20 planes, the same extraction on one GPU (configs[3]) fast, pcl
  c5       10M points, 20 planes: k = 20 normals -> RegulateNormal -> NORMAL_PLANE extraction,
           all on the cloud's device copy (configs[4])                          pcl, fast

Bit-exact: iterations, best sample, coefficient bit patterns, per-plane inlier counts and the
SHA-256 of every plane's inlier-id list.  The fast refit (the bench's mode) is also run with the
lean rounds off and sharded over an in-process group of ranks: the same bits.  The input cloud is
regenerated here from the seeded generator and its SHA-256 checked first.
"""
import hashlib
import json
import os
import threading

import numpy as np
import pytest

import dialog_amd as D
from dialog_amd.synth import plane_cloud

pytestmark = [pytest.mark.gpu, pytest.mark.slow]
GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "fullsize.json")
DB = json.load(open(GOLD)) if os.path.exists(GOLD) else {}
MODES = {"pcl": dict(refit_mode=D.DLG_REFIT_PCL), "fast": dict(refit_mode=D.DLG_REFIT_FAST),
         "none": dict(optimize=False)}


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


_CLOUDS = {}


def cloud(name):
    if name not in _CLOUDS:
        _CLOUDS.clear()  # (one full-size cloud in host memory at a time)
        w = DB[name]
        p, _, _ = plane_cloud(w["n_points"], w["planes"], seed=w["seed"], shares=w["shares"])
        assert sha(p) == w["cloud_sha256"], "the generator did not reproduce the golden cloud"
        _CLOUDS[name] = p
    return _CLOUDS[name]


def params(mode, **extra):
    return D.make_params(0.02, max_iterations=4095, probability=1.0, hypotheses_per_launch=4096,
                         **MODES[mode], **extra)


def check_extract(e, g):
    assert e["n_planes"] == g["n_planes"]
    assert [[int(v) for v in c.view(np.uint32)] for c in e["coeffs"]] == g["coeff_bits"]
    offs = e["offsets"]
    assert [int(offs[k + 1] - offs[k]) for k in range(e["n_planes"])] == g["counts"]
    assert [sha(e["inliers"][offs[k]:offs[k + 1]]) for k in range(e["n_planes"])] == g["inliers_sha256"]


def modes_of(name):
    return sorted(DB.get(name, {}).get("modes", {}))


@pytest.mark.skipif("c2" not in DB, reason="fullsize.json has no c2")
@pytest.mark.parametrize("mode", modes_of("c2"))
def test_c2_segment(gpu_ctx, mode):
    g = DB["c2"]["modes"][mode]
    p = cloud("c2")
    cl = D.Cloud(gpu_ctx, p)
    inl, coeff, st = D.segment_cloud(cl, params(mode))
    cl.close()
    assert st["iterations"] == g["iterations"] and st["draws"] == g["draws"]
    assert st["launches"] == 1
    assert [int(v) for v in st["best_sample"]] == g["best_sample"]
    assert [int(v) for v in st["coeff_unrefined"].view(np.uint32)] == g["coeff_unrefined_bits"]
    assert st["n_unrefined"] == g["n_unrefined"]
    assert [int(v) for v in coeff.view(np.uint32)] == g["coeff_bits"]
    assert inl.size == g["n_inliers"] and sha(inl) == g["inliers_sha256"]


@pytest.mark.skipif("c3" not in DB, reason="fullsize.json has no c3")
@pytest.mark.parametrize("mode", modes_of("c3"))
def test_c3_extract(gpu_ctx, mode):
    p = cloud("c3")
    cl = D.Cloud(gpu_ctx, p)
    e = D.extract_planes(cl, params(mode), max_planes=20, min_inliers=500, capacity=p.shape[0])
    cl.close()
    check_extract(e, DB["c3"]["modes"][mode])
    assert e["stats"]["lean_rounds"] == e["stats"]["rounds"]  # the bench's path


@pytest.mark.skipif("c3" not in DB or "fast" not in DB["c3"]["modes"], reason="no c3/fast")
def test_c3_fast_two_pass_and_sharded(gpu_ctx):
    """The bench mode through the two-pass selects, and sharded over 2 in-process ranks."""
    p = cloud("c3")
    g = DB["c3"]["modes"]["fast"]
    ctx = D.Context(0)
    ctx.set_option(D.DLG_OPT_LEAN_ROUNDS, 0)
    cl = D.Cloud(ctx, p)
    e = D.extract_planes(cl, params("fast"), max_planes=20, min_inliers=500, capacity=p.shape[0])
    cl.close()
    ctx.close()
    assert e["stats"]["lean_rounds"] == 0
    check_extract(e, g)
    ctxs = D.Context.loopback_group(2, 0)
    half = p.shape[0] // 2
    out, errs = [None, None], []

    def run(r):
        try:
            lo, hi = (0, half) if r == 0 else (half, p.shape[0])
            c = D.Cloud(ctxs[r], p[lo:hi], id_base=lo)
            out[r] = D.extract_planes(c, params("fast"), max_planes=20, min_inliers=500,
                                      capacity=p.shape[0])
            c.close()
        except Exception as ex:  # pragma: no cover
            errs.append(ex)

    th = [threading.Thread(target=run, args=(r,)) for r in range(2)]
    [t.start() for t in th]
    [t.join() for t in th]
    for c in ctxs:
        c.close()
    assert not errs, errs
    for r in range(2):
        check_extract(out[r], g)
        assert out[r]["stats"]["lean_rounds"] > 0  # (both shards hold a Morton copy)


def run_sharded(p, bounds, mode, profile=False, options=()):
    """extract_planes over in-process loopback ranks, rank r holding p[bounds[r]:bounds[r+1]]
    (options: (option, value) pairs set on every rank's context)."""
    W = len(bounds) - 1
    ctxs = D.Context.loopback_group(W, 0)
    out, errs = [None] * W, []

    def run(r):
        try:
            if profile:
                ctxs[r].set_profiling(True)
            for o, v in options:
                ctxs[r].set_option(o, v)
            lo, hi = bounds[r], bounds[r + 1]
            c = D.Cloud(ctxs[r], p[lo:hi], id_base=lo)
            out[r] = D.extract_planes(c, params(mode), max_planes=20, min_inliers=500,
                                      capacity=p.shape[0])
            c.close()
        except Exception as ex:  # pragma: no cover
            print(f"rank {r}: {ex!r}", flush=True)  # (the other ranks may now wait forever)
            errs.append(ex)

    th = [threading.Thread(target=run, args=(r,)) for r in range(W)]
    [t.start() for t in th]
    [t.join() for t in th]
    for c in ctxs:
        c.close()
    assert not errs, errs
    return out


@pytest.mark.skipif("c3" not in DB, reason="fullsize.json has no c3")
@pytest.mark.parametrize("bounds", ["halves", "uneven3"])
def test_c3_pcl_sharded(gpu_ctx, bounds):
    """DLG_REFIT_PCL over in-process ranks (halves: lean rounds on both; uneven3: one shard below
    the Morton-copy size, so the list path): the nine float chains are walked rank after rank in
    list order, and the planes equal the one-rank oracle's PCL refit bit for bit."""
    p = cloud("c3")
    b = [0, p.shape[0] // 2, p.shape[0]] if bounds == "halves" else [0, 100_000, 4_000_000, p.shape[0]]
    out = run_sharded(p, b, "pcl")
    for r in range(len(b) - 1):
        check_extract(out[r], DB["c3"]["modes"]["pcl"])
        assert (out[r]["stats"]["lean_rounds"] > 0) == (bounds == "halves")


@pytest.mark.skipif("c3" not in DB, reason="fullsize.json has no c3")
def test_c3_fast_uneven_shards_agree_on_lean(gpu_ctx):
    """One shard below the Morton-copy size (131072 points), one above: the ranks agree once per
    extraction that lean rounds need every rank's spatial copy, so both take the list path, and
    the planes still equal the one-rank oracle's bit for bit."""
    p = cloud("c3")
    out = run_sharded(p, [0, 100_000, p.shape[0]], "fast")
    for r in range(2):
        check_extract(out[r], DB["c3"]["modes"]["fast"])
        assert out[r]["stats"]["lean_rounds"] == 0


@pytest.mark.skipif("c4shape" not in DB, reason="fullsize.json has no c4shape")
@pytest.mark.parametrize("mode", modes_of("c4shape"))
def test_c4shape_extract_one_gpu(gpu_ctx, mode):
    """configs[3]'s 100M-point cloud on one GPU (the 8-GPU run shards it)."""
    p = cloud("c4shape")
    cl = D.Cloud(gpu_ctx, p)
    e = D.extract_planes(cl, params(mode), max_planes=20, min_inliers=500, capacity=p.shape[0])
    cl.close()
    check_extract(e, DB["c4shape"]["modes"][mode])


C4_PROTOCOLS = [(m, 0) for m in modes_of("c4shape")] + \
    ([("pcl", 1), ("pcl", 2)] if "pcl" in modes_of("c4shape") else [])


@pytest.mark.skipif("c4shape" not in DB, reason="fullsize.json has no c4shape")
@pytest.mark.parametrize("mode,proto", C4_PROTOCOLS)
def test_c4shape_sharded_loopback(gpu_ctx, mode, proto):
    """configs[3] as BASELINE states it: the 100M-point cloud sharded over 8 ranks (12.5M points
    each: every shard is far above the 131072-point Morton-copy cut-off, so every rank scores
    with the pruned kernel and every round is a lean round).  An in-process loopback group on one
    GPU stands in for the 8 RCCL ranks (the same driver code; host-relayed collectives).  PCL
    mode (DLG_OPT_FS_ONE_WALK = proto): every rank walks its shard's nine float chains from its
    refined guesses at once; 0: rebases on the guess the first walks propagate, walks again, and
    the exact chain values travel rank to rank through k_fs_repair (7 hops per round, each
    repair a few windows); 1 (round 4): no rebase, the repairs start ~1000 quanta off; 2: as 0
    with parallel repair iterations and host checks instead of the hand-over.  Every rank's planes and inlier lists equal the one-rank oracle's bit for
    bit.  The per-rank walk and repair device times are printed (and written to $DLG_REPORT if
    set)."""
    p = cloud("c4shape")
    n, W = p.shape[0], 8
    b = [n * r // W for r in range(W + 1)]
    out = run_sharded(p, b, mode, profile=True,
                      options=[(D.DLG_OPT_FS_ONE_WALK, proto)])
    g = DB["c4shape"]["modes"][mode]
    rows = []
    for r in range(W):
        check_extract(out[r], g)
        st = out[r]["stats"]
        assert st["lean_rounds"] == st["rounds"], (r, st)
        rows.append(dict(rank=r, points=b[r + 1] - b[r], rounds=st["rounds"],
                         walk_ms=round(st["refit_walk_ms"], 4),
                         repair_ms=round(st["refit_repair_ms"], 4),
                         rebase_ms=round(st["refit_rebase_ms"], 4),
                         repairs=st["refit_repairs"],
                         score_ms=round(st["score_ms"], 4), select_ms=round(st["select_ms"], 4),
                         wall_ms=round(st["wall_ms"], 2)))
    if mode == "pcl":
        assert all(rw["walk_ms"] > 0 for rw in rows)
        assert rows[0]["repair_ms"] == 0 and all(rw["repair_ms"] >= 0 for rw in rows[1:])
        # (every rank takes the same branches: the exactness checks read allgathered values)
        assert len({rw["repairs"] for rw in rows}) == 1
        assert rows[0]["repairs"] == (W - 1) * rows[0]["rounds"] if proto != 2 else \
            rows[0]["repairs"] <= (W - 1) * rows[0]["rounds"]
    rep = dict(mode=mode, proto=proto, ranks=W, rows=rows)
    print("\n" + json.dumps(rep))
    if os.environ.get("DLG_REPORT"):
        with open(os.environ["DLG_REPORT"], "a") as f:
            f.write(json.dumps(rep) + "\n")


@pytest.mark.skipif("c2" not in DB, reason="fullsize.json has no c2")
@pytest.mark.parametrize("mode", modes_of("c2"))
def test_c2_hyp_sharded_loopback(gpu_ctx, mode):
    """configs[1]'s 1M-point cloud on 8 ranks the way SURVEY 8(e) falls back for small N, with
    default options: point shards would leave 125k points per rank, under the 131072-point
    Morton-copy cut-off, so dlg_shard_range hands every rank the whole cloud (its own pruned
    scorer), and DLG_OPT_HYP_SHARD's default sees the replicated cloud and splits the 4096
    hypotheses 512 per rank; the allreduced counts give the golden iterations, best sample and
    bits."""
    g = DB["c2"]["modes"][mode]
    p = cloud("c2")
    W = 8
    ctxs = D.Context.loopback_group(W, 0)
    out, errs = [None] * W, []

    def run(r):
        try:
            lo, hi, rep = D.shard_range(p.shape[0], r, W)
            assert rep and (lo, hi) == (0, p.shape[0])
            assert ctxs[r].get_option(D.DLG_OPT_HYP_SHARD) == -1
            c = D.Cloud(ctxs[r], p[lo:hi], id_base=lo)
            out[r] = D.segment_cloud(c, params(mode), capacity=p.shape[0])
            c.close()
        except Exception as ex:  # pragma: no cover
            errs.append(ex)

    th = [threading.Thread(target=run, args=(r,)) for r in range(W)]
    [t.start() for t in th]
    [t.join() for t in th]
    for c in ctxs:
        c.close()
    assert not errs, errs
    for r in range(W):
        inl, coeff, st = out[r]
        assert st["iterations"] == g["iterations"] and st["draws"] == g["draws"]
        assert [int(v) for v in st["best_sample"]] == g["best_sample"]
        assert [int(v) for v in coeff.view(np.uint32)] == g["coeff_bits"]
        assert inl.size == g["n_inliers"] and sha(inl) == g["inliers_sha256"]


@pytest.mark.skipif("c5" not in DB, reason="fullsize.json has no c5")
@pytest.mark.parametrize("mode", modes_of("c5"))
def test_c5_fullsize(gpu_ctx, mode):
    """configs[4] at its quoted size, the reference's order (estimateNormal PlaneDetect.h:515-545,
    regulateNormal :547-665, then the plane stage) on the cloud's device copy, as the bench's
    chain_regulate times it: k = 20 normals (dlg_cloud_estimate_normals; the float32 bits of all
    10M (normal, curvature) records against the oracle's SHA-256), RegulateNormal (BFS r 0.1 from
    point 0, outward; reached count and the regulated records' SHA-256), then SACMODEL_NORMAL_PLANE
    (w 0.1) extract-and-remove over the regulated normals: coefficient bits, counts and inlier
    SHA-256s.  The extraction's rounds run lean (the Morton copy's NORMAL_PLANE rounds)."""
    w = DB["c5"]
    ch = w["chain"]
    p = cloud("c5")
    cl = D.Cloud(gpu_ctx, p)
    try:
        nrm = cl.estimate_normals(k=ch["k"], copy_out=True)
        assert sha(nrm) == ch["normals_sha256"]
        del nrm
        _, reached, reg = cl.regulate_normals(ch["reg_seed"], ch["reg_outward"], ch["reg_radius"],
                                              copy_out=True)
        assert reached == ch["reached"]
        assert sha(reg) == ch["regulated_sha256"]
        del reg
        prm = params(mode, model=D.SACMODEL_NORMAL_PLANE, normal_distance_weight=ch["weight"])
        e = D.extract_planes(cl, prm, max_planes=20, min_inliers=500, capacity=p.shape[0])
    finally:
        cl.close()
    check_extract(e, w["modes"][mode])
    assert e["stats"]["lean_rounds"] > 0, e["stats"]
