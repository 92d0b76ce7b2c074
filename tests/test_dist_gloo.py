"""N > 1 on the CPU: the point-sharded RANSAC protocol over torch.distributed
`gloo` with world_size 2 and 3, driven by the product's host controller (dlg_sac_control_*, the
replay dlg_sac_segment runs between its kernels) -- see tests/dist_protocol.py.  Sharded extract-
and-remove must reproduce the single-process PCL restatement bit for bit, and every rank must
take the same decisions.  The GPU-side counterpart (same protocol through the library's own
collectives, loopback ranks on one device) is tests/test_gpu_parity.py::test_sharded_*.
"""
import os
import socket
import sys

import numpy as np
import pytest
import torch.multiprocessing as mp

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.dirname(HERE))

from oracle import oracle as O  # noqa: E402


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _entry(rank, world, port, out_dir, kw):
    import dist_protocol
    dist_protocol.run(rank, world, port, out_dir, **kw)


@pytest.mark.parametrize("world,sizes,refit", [(2, None, "pcl"), (3, [1500, 4000, 500], "pcl"),
                                               (2, None, "fast"), (4, [0, 2500, 2000, 1500], "fast")],
                         ids=["ws2-even-pcl", "ws3-ragged-pcl", "ws2-even-fast", "ws4-empty-rank-fast"])
def test_sharded_extract_gloo(tmp_path, world, sizes, refit):
    n = 6000
    if sizes is None:
        sizes = [n // world] * world
        sizes[-1] += n - sum(sizes)
    kw = dict(n_points=n, n_planes=3, threshold=0.02, max_planes=4, min_inliers=50,
              max_iterations=120, probability=0.99, batch=64, sizes=sizes, refit=refit)
    mp.start_processes(_entry, args=(world, _port(), str(tmp_path), kw), nprocs=world,
                       join=True, start_method="spawn")
    outs = [np.load(tmp_path / f"rank{r}.npz") for r in range(world)]
    for o in outs[1:]:   # identical decisions, results and collective sequence on every rank
        for k in ("coeffs", "inliers", "offsets", "decisions", "log"):
            assert np.array_equal(o[k], outs[0][k]), k
    # the driver's sequence: one active-count allgather, [the quantum], then per
    # round samples + counts per batch, the refit exchange, the (in, out) allgather, the ids
    log = [tuple(e.split(":")) for e in outs[0]["log"]]
    assert log[0] == ("allgather", "int64", "1")
    i = 1
    if refit == "fast":
        assert log[1] == ("allreduce_max", "float64", "1")
        i = 2
    rounds = 0
    while i < len(log):
        assert log[i][0] == "allreduce_sum" and log[i][1] == "int32"
        d = int(log[i][2]) // 12
        while log[i][:2] == ("allreduce_sum", "int32") and int(log[i][2]) % 12 == 0 and \
                log[i + 1] == ("allreduce_sum", "int32", str(int(log[i][2]) // 12)):
            i += 2  # one batch: samples (12 D int32), counts (D int32)
        assert d > 0
        if refit == "fast":
            assert log[i] == ("allreduce_sum", "int64", "25")
            i += 1
        else:
            assert log[i] == ("allgather", "int64", "1") and log[i + 1][:2] == ("allgather", "int32")
            i += 2
        assert log[i] == ("allgather", "int32", "2")
        i += 1
        if i < len(log) and log[i] == ("allgather", "int64", "1"):  # accepted plane: its ids
            i += 2 if i + 1 < len(log) and log[i + 1][:2] == ("allgather", "int32") else 1
        rounds += 1
    assert rounds >= 3
    from dialog_amd.synth import plane_cloud
    pts, _, _ = plane_cloud(n, 3, seed=913)
    ref = O.extract_planes(pts, 0.02, max_planes=4, min_inliers=50, max_iterations=120,
                           probability=0.99, refit=refit)
    got = outs[0]
    assert ref["n_planes"] >= 3 and got["coeffs"].shape[0] == ref["n_planes"]
    assert np.array_equal(got["coeffs"].view(np.uint32), ref["coeffs"].view(np.uint32))
    assert np.array_equal(got["offsets"], ref["offsets"])
    assert np.array_equal(got["inliers"], ref["inliers"])


def test_control_matches_oracle_single_rank():
    """dlg_sac_control_* alone (no ranks): iterations, draws, best sample of PCL's loop."""
    import dialog_amd as D
    from dialog_amd.synth import plane_cloud
    pts, _, _ = plane_cloud(4000, 3, seed=77)
    for mi, p, batch in [(200, 0.99, 64), (50, 0.99, 4096), (300, 1.0, 100), (5, 0.5, 1)]:
        prm = D.make_params(0.02, max_iterations=mi, probability=p)
        ctl = D.RansacControl(prm, pts.shape[0], batch)
        best = None
        while True:
            pos = ctl.next()
            if pos.shape[0] == 0:
                break
            good = np.zeros(len(pos), np.int32)
            cnt = np.zeros(len(pos), np.int32)
            for i, (a, b, c) in enumerate(pos):
                ok, co = O.plane_coefficients(pts[a], pts[b], pts[c])
                good[i] = ok
                cnt[i] = O.count_within(pts, co, 0.02) if ok else 0
            bi, fin = ctl.consume(cnt, good)
            if bi >= 0:
                best = pos[bi].copy()
            if fin:
                break
        r = ctl.result()
        ref = O.sac_segment(pts, 0.02, max_iterations=mi, probability=p)
        assert (r["iterations"], r["draws"], r["n_unrefined"]) == \
            (ref["iterations"], ref["draws"], ref["n_unrefined"])
        assert list(best) == list(ref["best_sample"])
    ctl = D.RansacControl(D.make_params(0.02), 2)   # < 3 points: no draw, no model
    assert ctl.next().shape[0] == 0 and not ctl.result()["has_model"]
    # max_iterations = 0: PCL's max_skip = 10 * max_iterations = 0, the loop never runs
    ctl = D.RansacControl(D.make_params(0.02, max_iterations=0, probability=1.0), 100)
    ref = O.sac_segment(np.random.default_rng(1).random((100, 3)).astype(np.float32), 0.02,
                        max_iterations=0, probability=1.0)
    assert ctl.next().shape[0] == 0 and not ctl.result()["has_model"] and not ref["ok"]
    assert ref["draws"] == 0


@pytest.mark.parametrize("world,refit,batch", [(2, "pcl", 64), (3, "fast", 200), (4, "pcl", 100)],
                         ids=["ws2-pcl", "ws3-fast", "ws4-pcl-few-groups"])
def test_hyp_sharded_extract_gloo(tmp_path, world, refit, batch):
    """DLG_OPT_HYP_SHARD (SURVEY 8(e)'s small-N fallback) over gloo: every rank holds the whole
    cloud, scores its slice of each batch's hypotheses (whole 64-hypothesis groups; with fewer
    groups than ranks some ranks score none) and the counts are allreduced -- the only
    collective, once per batch.  Every rank's planes equal the single-process oracle's."""
    n = 6000
    kw = dict(n_points=n, n_planes=3, threshold=0.02, max_planes=4, min_inliers=50,
              max_iterations=120, probability=0.99, batch=batch, sizes=[n] * world, refit=refit,
              hyp_shard=True)
    mp.start_processes(_entry, args=(world, _port(), str(tmp_path), kw), nprocs=world,
                       join=True, start_method="spawn")
    outs = [np.load(tmp_path / f"rank{r}.npz") for r in range(world)]
    for o in outs[1:]:
        for k in ("coeffs", "inliers", "offsets", "decisions", "log"):
            assert np.array_equal(o[k], outs[0][k]), k
    log = [tuple(e.split(":")) for e in outs[0]["log"]]
    assert log and all(e[:2] == ("allreduce_sum", "int32") and 0 < int(e[2]) <= batch for e in log)
    from dialog_amd.synth import plane_cloud
    pts, _, _ = plane_cloud(n, 3, seed=913)
    ref = O.extract_planes(pts, 0.02, max_planes=4, min_inliers=50, max_iterations=120,
                           probability=0.99, refit=refit)
    got = outs[0]
    assert ref["n_planes"] >= 3 and got["coeffs"].shape[0] == ref["n_planes"]
    assert np.array_equal(got["coeffs"].view(np.uint32), ref["coeffs"].view(np.uint32))
    assert np.array_equal(got["offsets"], ref["offsets"])
    assert np.array_equal(got["inliers"], ref["inliers"])


def test_hyp_slices_partition():
    """The slices of driver.cpp one_batch / dist_protocol.hyp_slice partition [0, D) into whole
    64-hypothesis groups (an exhaustive kernel's padded group stays inside its rank's slice)."""
    from dist_protocol import hyp_slice
    for D in (1, 63, 64, 65, 100, 511, 4096, 4000):
        for R in (1, 2, 3, 5, 8, 16):
            sl = [hyp_slice(D, r, R) for r in range(R)]
            assert sl[0][0] == 0 and sl[-1][1] == D
            for (a, b), (c, d) in zip(sl, sl[1:]):
                assert b == c and a <= b
            for a, b in sl:
                assert a % 64 == 0 and (b % 64 == 0 or b == D)
