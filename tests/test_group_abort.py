"""Failure propagation across the ranks of a group (errors come back as status codes,
on every rank -- the reference prints and returns, PlaneDetect.h:371-375, 592-596).

A rank whose dlg_extract_planes fails aborts its group: every peer blocked in (or entering) a
collective returns DLG_ERR_COMM naming that rank and its error, within seconds, instead of waiting
forever (round 5's 8-rank hang: one rank's select gave up, seven waited).  Also here: the
per-round divergence check (DLG_OPT_SYNC_CHECK), the select tile-numbering A/B
(DLG_OPT_SEL1_TICKET) and the survivors' sphere bounds on a side stream (DLG_OPT_BOUNDS_STREAM),
each against the one-rank run, and dlg_shard_range's host arithmetic (CPU).
"""
import threading
import time

import numpy as np
import pytest

import dialog_amd as D
from dialog_amd.synth import plane_cloud

N, PLANES, W = 2_000_000, 8, 4  # 500k points per rank: every shard has a Morton copy (lean rounds)
_CACHE = {}


def cloud():
    if "p" not in _CACHE:
        _CACHE["p"], _, _ = plane_cloud(N, PLANES, seed=0xD1A106 + 60)
    return _CACHE["p"]


def params(mode):
    refit = D.DLG_REFIT_PCL if mode == "pcl" else D.DLG_REFIT_FAST
    return D.make_params(0.02, max_iterations=4095, probability=1.0, refit_mode=refit)


def one_rank(gpu_ctx, mode):
    key = ("ref", mode)
    if key not in _CACHE:
        c = D.Cloud(gpu_ctx, cloud())
        _CACHE[key] = D.extract_planes(c, params(mode), max_planes=PLANES, min_inliers=500)
        c.close()
    return _CACHE[key]


def same(a, b):
    assert a["n_planes"] == b["n_planes"]
    assert np.array_equal(a["coeffs"].view(np.uint32), b["coeffs"].view(np.uint32))
    assert np.array_equal(a["offsets"], b["offsets"])
    assert np.array_equal(a["inliers"], b["inliers"])


def run_group(mode, options=(), per_rank=None, join_s=120.0):
    """extract_planes over a W-rank loopback group, rank r on its shard; -> per-rank
    (result dict | DialogError, seconds from the start to the return)."""
    p = cloud()
    b = [p.shape[0] * r // W for r in range(W + 1)]
    ctxs = D.Context.loopback_group(W, 0)
    res = [None] * W
    t0 = time.monotonic()

    def run(r):
        c = None
        try:
            for o, v in options:
                ctxs[r].set_option(o, v)
            for o, v in (per_rank or {}).get(r, ()):
                ctxs[r].set_option(o, v)
            c = D.Cloud(ctxs[r], p[b[r]:b[r + 1]], id_base=b[r])
            out = D.extract_planes(c, params(mode), max_planes=PLANES, min_inliers=500,
                                   capacity=p.shape[0])
            res[r] = (out, time.monotonic() - t0)
        except D.DialogError as e:
            res[r] = (e, time.monotonic() - t0)
        except Exception as e:  # pragma: no cover
            res[r] = (e, time.monotonic() - t0)
        finally:
            if c is not None:
                c.close()

    th = [threading.Thread(target=run, args=(r,), daemon=True) for r in range(W)]
    [t.start() for t in th]
    for t in th:
        t.join(max(0.1, join_s - (time.monotonic() - t0)))
    hung = [r for r in range(W) if th[r].is_alive()]
    if not hung:
        for c in ctxs:
            c.close()
    assert not hung, f"ranks {hung} never returned"
    return res


@pytest.mark.gpu
@pytest.mark.parametrize("mode,victim,round_", [("fast", 2, 3), ("pcl", 0, 2), ("pcl", 3, 5)])
def test_fault_in_one_rank_fails_every_rank(gpu_ctx, mode, victim, round_):
    """One rank of a 4-rank group fails in the middle of extract round `round_` (after the
    round's scoring, DLG_OPT_FAULT_INJECT): it returns its own error, every peer returns
    DLG_ERR_COMM naming it, all within seconds of each other; the aborted group's contexts close,
    and a new group on the same device runs the extraction to the one-rank bits."""
    res = run_group(mode, per_rank={victim: [(D.DLG_OPT_FAULT_INJECT, round_ + 1)]})
    errs = [r[0] for r in res]
    assert all(isinstance(e, D.DialogError) for e in errs), errs
    assert errs[victim].status == D.DLG_ERR_INTERNAL and "injected fault" in str(errs[victim])
    for r in range(W):
        if r != victim:
            assert errs[r].status == D.DLG_ERR_COMM, (r, errs[r])
            assert f"rank {victim} failed" in str(errs[r]) and "injected fault" in str(errs[r])
    t = [r[1] for r in res]
    assert max(t) - t[victim] < 5.0, t
    ok = run_group(mode)
    for r in range(W):
        same(ok[r][0], one_rank(gpu_ctx, mode))


@pytest.mark.gpu
def test_sync_check_and_side_stream_match_one_rank(gpu_ctx):
    """DLG_OPT_SYNC_CHECK (per-round allgather of round, inliers, coefficient bits and collectives
    issued) passes on a healthy group, with the survivors' sphere bounds on a side stream
    (DLG_OPT_BOUNDS_STREAM) on every rank: the one-rank planes and inliers bit for bit."""
    res = run_group("pcl", options=[(D.DLG_OPT_SYNC_CHECK, 1), (D.DLG_OPT_BOUNDS_STREAM, 1)])
    for r in range(W):
        assert not isinstance(res[r][0], Exception), res[r][0]
        same(res[r][0], one_rank(gpu_ctx, "pcl"))
        assert res[r][0]["stats"]["lean_rounds"] == res[r][0]["stats"]["rounds"]


@pytest.mark.gpu
@pytest.mark.parametrize("ticket,side", [(0, 0), (1, 1), (0, 1)])
def test_select_tile_numbering_and_side_stream_one_rank(gpu_ctx, ticket, side):
    """The single-pass selects' tile numbering (DLG_OPT_SEL1_TICKET: 1 tickets, 0 workgroup index;
    the default -1 takes tickets while another context shares the device) and the side-stream
    bounds give the default path's bits on one rank."""
    ctx = D.Context(0)
    ctx.set_option(D.DLG_OPT_SEL1_TICKET, ticket)
    ctx.set_option(D.DLG_OPT_BOUNDS_STREAM, side)
    c = D.Cloud(ctx, cloud())
    e = D.extract_planes(c, params("fast"), max_planes=PLANES, min_inliers=500)
    c.close()
    ctx.close()
    same(e, one_rank(gpu_ctx, "fast"))
    assert e["stats"]["lean_rounds"] == e["stats"]["rounds"]


@pytest.mark.gpu
def test_options_reported(gpu_ctx):
    ctx = D.Context(0)
    assert ctx.get_option(D.DLG_OPT_SEL1_TICKET) == -1
    assert ctx.get_option(D.DLG_OPT_BOUNDS_STREAM) == 0
    assert ctx.get_option(D.DLG_OPT_SPATIAL_CURVE) == 1
    assert ctx.get_option(D.DLG_OPT_HYP_SHARD) == -1
    assert ctx.get_option(D.DLG_OPT_COMM_TIMEOUT_MS) == 600000
    ctx.set_option(D.DLG_OPT_COMM_TIMEOUT_MS, 1234)
    assert ctx.get_option(D.DLG_OPT_COMM_TIMEOUT_MS) == 1234
    with pytest.raises(D.DialogError):
        ctx.set_option(D.DLG_OPT_HYP_SHARD, 2)
    ctx.close()


@pytest.mark.parametrize("n,world", [(1_000_000, 8), (10_000_000, 8), (100_000_000, 8),
                                     (2_000_000, 4), (1_000, 1), (0, 3)])
def test_shard_range_cpu(n, world):
    """dlg_shard_range (host arithmetic, no device): contiguous shards covering [0, n) in rank
    order, or the whole cloud on every rank when a shard would hold fewer than 131072 points."""
    rng = [D.shard_range(n, r, world) for r in range(world)]
    rep = world > 1 and n // world < 131072
    assert all(x[2] == rep for x in rng)
    if rep:
        assert all((x[0], x[1]) == (0, n) for x in rng)
    else:
        assert rng[0][0] == 0 and rng[-1][1] == n
        assert all(rng[r][1] == rng[r + 1][0] for r in range(world - 1))

