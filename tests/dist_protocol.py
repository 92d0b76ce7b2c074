"""Worker of tests/test_dist_gloo.py: the point-sharded multi-rank RANSAC protocol of
SURVEY.md §8(e) run by world_size CPU processes over torch.distributed `gloo`.

Every rank drives the product's host controller (dialog_amd.RansacControl = dlg_sac_control_*,
the replay dlg_extract_planes runs between its kernels) on the global active count, and issues
exactly the collectives the library issues per GPU (driver.cpp), in the same order
and with the same types and sizes, with the oracle standing in for the device kernels (test
infrastructure):

  once per extraction:
    allgather int64[1]            every rank's active count (allgather_i64)
    allreduce-max f64[1]          fast refit: the cloud's largest finite |coordinate| (its quantum;
                                  once per cloud)
  per round, per batch of D draws:
    allreduce-sum int32[12 D]     the draws' SampleRecs {gid, x, y, z} as int32 bit patterns: the
                                  owning rank contributes, the others zeros (k_gather_samples)
    allreduce-sum int32[D]        inlier counts of the rank's shard (k_score)
  per round, refit:
    pcl : allgather int64[1] + padded allgather int32[3 m]   the unrefined inliers' xyz in rank
          order (= PCL's list order), summed sequentially in float on every rank
    fast: allreduce-sum int64[25] the exact moment digits (exact_refit.hpp)
  per round, select:
    allgather int32[2]            every rank's (inliers, survivors): the next round's counts
  per accepted plane (gather_inliers):
    allgather int64[1] + padded allgather int32[m]           the inlier ids in rank order

Each rank logs (op, dtype, count) of every collective; the test checks the logs are identical
across ranks and that the result equals the single-process restatement bit for bit.

hyp_shard (DLG_OPT_HYP_SHARD, SURVEY 8(e)'s small-N fallback): every rank holds the whole cloud
and runs the whole round; per batch of D draws rank r scores only its slice of the hypotheses
(whole 64-hypothesis groups: groups [U r / R, U (r + 1) / R) of U = ceil(D / 64)) and the counts
are allreduced -- the only collective:
    allreduce-sum int32[D]        per batch
"""
from __future__ import annotations

import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)


class Coll:
    """the collectives of comm.cpp over gloo, logged"""

    def __init__(self, dist, torch):
        self.dist, self.torch, self.log = dist, torch, []

    def allreduce_sum(self, arr):
        self.log.append(("allreduce_sum", str(arr.dtype), int(arr.size)))
        t = self.torch.from_numpy(np.ascontiguousarray(arr).copy())
        self.dist.all_reduce(t)
        return t.numpy()

    def allreduce_max_f64(self, v):
        self.log.append(("allreduce_max", "float64", 1))
        t = self.torch.tensor([float(v)], dtype=self.torch.float64)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX)
        return float(t.item())

    def allgather(self, arr):
        self.log.append(("allgather", str(arr.dtype), int(arr.size)))
        t = self.torch.from_numpy(np.ascontiguousarray(arr).copy())
        outs = [self.torch.zeros_like(t) for _ in range(self.dist.get_world_size())]
        self.dist.all_gather(outs, t)
        return np.stack([o.numpy() for o in outs])

    def gather_lists(self, arr, width):
        """driver.cpp gather_lists: counts by allgather_i64, then one padded allgather"""
        cnt = self.allgather(np.array([arr.size // width], np.int64))[:, 0]
        m = int(cnt.max())
        if m == 0:
            return arr[:0]
        buf = np.zeros(m * width, arr.dtype)
        buf[:arr.size] = arr
        g = self.allgather(buf)
        return np.concatenate([g[r, :cnt[r] * width] for r in range(len(cnt))])


def _pcl_refit(O, xyz, coeff):
    """optimizeModelCoefficients over inlier xyz in list order (PCL float, oracle arithmetic)."""
    if xyz.shape[0] < 4:
        return coeff.copy()
    cov, cen = O.mean_cov(xyz, np.arange(xyz.shape[0], dtype=np.int32))
    _, v = O.eigen33(cov)
    f = np.float32
    dot = f(f(v[0] * cen[0]) + f(v[2] * cen[2])) + f(f(v[1] * cen[1]) + f(f(0) * cen[3]))
    return np.array([v[0], v[1], v[2], f(-1.0) * dot], np.float32)


def hyp_slice(D, rank, world):
    """driver.cpp one_batch: this rank's hypotheses [lo, hi) under DLG_OPT_HYP_SHARD"""
    U = (D + 63) // 64
    return min(D, 64 * (U * rank // world)), min(D, 64 * (U * (rank + 1) // world))


def run(rank, world, port, out_dir, n_points, n_planes, threshold, max_planes, min_inliers,
        max_iterations, probability, batch, sizes, refit="pcl", gather=True, hyp_shard=False):
    sys.path.insert(0, ROOT)
    import torch
    import torch.distributed as dist

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import dialog_amd as D
    from dialog_amd.synth import plane_cloud
    from oracle import numpy_twin as T
    from oracle import oracle as O

    cc = Coll(dist, torch)
    pts, _, _ = plane_cloud(n_points, n_planes, seed=913)   # the global cloud (host copy)
    bounds = np.concatenate([[0], np.cumsum(sizes)])
    mine_ids = (np.arange(n_points, dtype=np.int32) if hyp_shard else
                np.arange(bounds[rank], bounds[rank + 1], dtype=np.int32))
    local = mine_ids.copy()                                  # active global ids, list order
    prm = D.make_params(threshold, max_iterations=max_iterations, probability=probability,
                        hypotheses_per_launch=batch,
                        refit_mode=D.DLG_REFIT_FAST if refit == "fast" else D.DLG_REFIT_PCL)
    coeffs, inliers, offsets, decisions = [], [], [0], []
    floor_n = max(3, min_inliers)
    active = (np.array([local.shape[0]], np.int64) if hyp_shard else
              cc.allgather(np.array([local.shape[0]], np.int64))[:, 0])
    qexp = None
    while len(coeffs) < max_planes:
        N = int(active.sum())
        offset = 0 if hyp_shard else int(active[:rank].sum())
        if N < floor_n:
            break
        if refit == "fast" and qexp is None and world > 1 and not hyp_shard:
            # the cloud's global quantum, before the first round's draws (driver.cpp segment_impl)
            fin_pts = pts[mine_ids][np.isfinite(pts[mine_ids]).all(axis=1)]
            f = float(np.abs(fin_pts).max()) if fin_pts.size else 0.0
            qexp = int(np.frexp(cc.allreduce_max_f64(f))[1])
        ctl = D.RansacControl(prm, N, batch)
        best_coeff = None
        shard = np.ascontiguousarray(pts[local])
        while True:
            pos = ctl.next()
            if pos.shape[0] == 0:
                break
            Dn = pos.shape[0]
            # k_gather_samples: SampleRec {gid, x, y, z}, owner contributes, int32 bit patterns
            rec = np.zeros((Dn, 3, 4), np.int32)
            mine = (pos >= offset) & (pos < offset + local.shape[0])
            g = local[pos[mine] - offset]
            rec[mine, 0] = g
            rec[mine, 1:] = pts[g].view(np.int32)
            if not hyp_shard:
                rec = cc.allreduce_sum(rec.reshape(-1)).reshape(Dn, 3, 4)
            smp = np.ascontiguousarray(rec[:, :, 1:]).view(np.float32)
            # k_build_hyps + k_score on the local shard, allreduce of the counts
            good = np.zeros(Dn, np.int32)
            cnt = np.zeros(Dn, np.int32)
            hyp = np.zeros((Dn, 4), np.float32)
            lo, hi = hyp_slice(Dn, rank, world) if hyp_shard else (0, Dn)
            for d in range(Dn):
                ok, c = O.plane_coefficients(smp[d, 0], smp[d, 1], smp[d, 2])
                good[d] = int(ok)
                hyp[d] = c
                if ok and lo <= d < hi:
                    cnt[d] = O.count_within(shard, c, threshold) if shard.shape[0] else 0
            cnt = cc.allreduce_sum(cnt)
            b, fin = ctl.consume(cnt, good)
            if b >= 0:
                best_coeff = hyp[b].copy()
            if fin:
                break
        res = ctl.result()
        ctl.close()
        if best_coeff is None:
            break
        decisions.append((res["iterations"], res["draws"], res["n_unrefined"], res["best_draw"]))
        sel = T.within(best_coeff, shard, threshold) if shard.shape[0] else np.zeros(0, bool)
        if hyp_shard and refit == "pcl":
            refined = _pcl_refit(O, shard[sel], best_coeff)
        elif hyp_shard:
            if qexp is None:
                fin_pts = pts[np.isfinite(pts).all(axis=1)]
                qexp = int(np.frexp(float(np.abs(fin_pts).max()) if fin_pts.size else 0.0)[1])
            dig = O.mom_digits(pts, local[sel], qexp) if sel.any() else np.zeros(25, np.int64)
            refined = O.refit_digits(dig, best_coeff, qexp)
        elif refit == "pcl":
            xyz = cc.gather_lists(shard[sel].reshape(-1).view(np.int32).copy(), 3)
            refined = _pcl_refit(O, xyz.view(np.float32).reshape(-1, 3), best_coeff)
        else:
            dig = O.mom_digits(pts, local[sel], qexp) if sel.any() else np.zeros(25, np.int64)
            dig = cc.allreduce_sum(dig)
            refined = O.refit_digits(dig, best_coeff, qexp)
        sel = T.within(refined, shard, threshold) if shard.shape[0] else np.zeros(0, bool)
        rk = (np.array([[int(sel.sum()), int((~sel).sum())]], np.int32) if hyp_shard else
              cc.allgather(np.array([int(sel.sum()), int((~sel).sum())], np.int32)))
        n_in = int(rk[:, 0].sum())
        if n_in == 0 or n_in < min_inliers:
            break
        ids = (local[sel].copy() if (hyp_shard or not gather) else
               cc.gather_lists(local[sel].copy(), 1))
        coeffs.append(refined)
        inliers.append(ids)
        offsets.append(offsets[-1] + n_in)
        local = local[~sel]                     # local compaction, order kept
        active = rk[:, 1].astype(np.int64)
    np.savez(os.path.join(out_dir, f"rank{rank}.npz"),
             coeffs=np.array(coeffs, np.float32).reshape(-1, 4),
             inliers=np.concatenate(inliers).astype(np.int32) if inliers else np.zeros(0, np.int32),
             offsets=np.array(offsets, np.int64), decisions=np.array(decisions, np.int64),
             log=np.array([f"{o}:{t}:{n}" for o, t, n in cc.log]))
    dist.barrier()
    dist.destroy_process_group()
