"""Worker of tests/test_dist_gloo.py: the point-sharded multi-rank RANSAC protocol of
SURVEY.md §8(e) run by world_size CPU processes over torch.distributed `gloo`.

Every rank drives the product's host controller (dialog_amd.RansacControl = dlg_sac_control_*,
the same replay dlg_sac_segment runs between its kernels) on the global active count, and does
per rank what the library does per GPU, with the oracle standing in for the device kernels
(test infrastructure):

  * rank r holds a contiguous block of the global list (ascending global ids);
  * draws: the controller's global list positions -> the owning rank contributes the point, the
    others zeros, summed as int32 bit patterns (allreduce; exact, keeps -0.0) -- k_gather_samples;
  * isSampleGood + coefficients (oracle; k_build_hyps), inlier counts on the local shard
    (oracle; k_score) -> allreduce(sum) of int32[D] -> RansacControl.consume;
  * PCL refit: the unrefined inliers' xyz gathered in rank order (= PCL's list order) and summed
    sequentially in float; final select on each shard, gathered in rank order; compaction local.

The result must equal the single-process PCL restatement (oracle.extract_planes) bit for bit.
"""
from __future__ import annotations

import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)


def _allgather_var(dist, torch, arr, dtype):
    """rank-ordered concatenation of variable-length 1-D arrays (padded all_gather)."""
    n = torch.tensor([arr.shape[0]], dtype=torch.int64)
    world = dist.get_world_size()
    ns = [torch.zeros(1, dtype=torch.int64) for _ in range(world)]
    dist.all_gather(ns, n)
    ns = [int(v.item()) for v in ns]
    m = max(max(ns), 1)
    buf = torch.zeros(m, dtype=dtype)
    buf[:arr.shape[0]] = torch.from_numpy(arr)
    outs = [torch.zeros(m, dtype=dtype) for _ in range(world)]
    dist.all_gather(outs, buf)
    return np.concatenate([o[:k].numpy() for o, k in zip(outs, ns)]), ns


def _pcl_refit(O, xyz, coeff):
    """optimizeModelCoefficients over inlier xyz in list order (PCL float, oracle arithmetic)."""
    if xyz.shape[0] < 4:
        return coeff.copy()
    cov, cen = O.mean_cov(xyz, np.arange(xyz.shape[0], dtype=np.int32))
    _, v = O.eigen33(cov)
    f = np.float32
    dot = f(f(v[0] * cen[0]) + f(v[2] * cen[2])) + f(f(v[1] * cen[1]) + f(f(0) * cen[3]))
    return np.array([v[0], v[1], v[2], f(-1.0) * dot], np.float32)


def run(rank, world, port, out_dir, n_points, n_planes, threshold, max_planes, min_inliers,
        max_iterations, probability, batch, sizes):
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

    pts, _, _ = plane_cloud(n_points, n_planes, seed=913)   # the global cloud (host copy)
    bounds = np.concatenate([[0], np.cumsum(sizes)])
    local = np.arange(bounds[rank], bounds[rank + 1], dtype=np.int32)  # active global ids
    prm = D.make_params(threshold, max_iterations=max_iterations, probability=probability,
                        hypotheses_per_launch=batch)
    coeffs, inliers, offsets, decisions = [], [], [0], []
    floor_n = max(3, min_inliers)
    while len(coeffs) < max_planes:
        # allgather of n_active -> global N and this rank's offset in the global list
        na, ns = _allgather_var(dist, torch, np.array([local.shape[0]], np.int64), torch.int64)
        N = int(na.sum())
        offset = int(na[:rank].sum())
        if N < floor_n:
            break
        ctl = D.RansacControl(prm, N, batch)
        best_coeff = None
        while True:
            pos = ctl.next()
            if pos.shape[0] == 0:
                break
            Dn = pos.shape[0]
            # k_gather_samples: owner contributes, int32 bit-pattern sum across ranks
            smp = np.zeros((Dn, 3, 3), np.float32)
            mine = (pos >= offset) & (pos < offset + local.shape[0])
            smp[mine] = pts[local[pos[mine] - offset]]
            t = torch.from_numpy(smp.view(np.int32).copy())
            dist.all_reduce(t)
            smp = t.numpy().view(np.float32)
            # k_build_hyps + k_score on the local shard, allreduce of the counts
            good = np.zeros(Dn, np.int32)
            cnt = np.zeros(Dn, np.int32)
            hyp = np.zeros((Dn, 4), np.float32)
            shard = np.ascontiguousarray(pts[local])
            for d in range(Dn):
                ok, c = O.plane_coefficients(smp[d, 0], smp[d, 1], smp[d, 2])
                good[d] = int(ok)
                hyp[d] = c
                if ok:
                    cnt[d] = O.count_within(shard, c, threshold) if shard.shape[0] else 0
            t = torch.from_numpy(cnt.copy())
            dist.all_reduce(t)
            b, fin = ctl.consume(t.numpy(), good)
            if b >= 0:
                best_coeff = hyp[b].copy()
            if fin:
                break
        res = ctl.result()
        ctl.close()
        if best_coeff is None:
            break
        decisions.append((res["iterations"], res["draws"], res["n_unrefined"], res["best_draw"]))
        shard = np.ascontiguousarray(pts[local])
        sel = T.within(best_coeff, shard, threshold) if shard.shape[0] else np.zeros(0, bool)
        xyz, _ = _allgather_var(dist, torch, shard[sel].reshape(-1).copy(), torch.float32)
        refined = _pcl_refit(O, xyz.reshape(-1, 3), best_coeff)
        sel = T.within(refined, shard, threshold) if shard.shape[0] else np.zeros(0, bool)
        ids, _ = _allgather_var(dist, torch, local[sel].copy(), torch.int32)
        if ids.shape[0] == 0 or ids.shape[0] < min_inliers:
            break
        coeffs.append(refined)
        inliers.append(ids)
        offsets.append(offsets[-1] + ids.shape[0])
        local = local[~sel]                     # local compaction, order kept
    np.savez(os.path.join(out_dir, f"rank{rank}.npz"),
             coeffs=np.array(coeffs, np.float32).reshape(-1, 4),
             inliers=np.concatenate(inliers).astype(np.int32) if inliers else np.zeros(0, np.int32),
             offsets=np.array(offsets, np.int64), decisions=np.array(decisions, np.int64))
    dist.barrier()
    dist.destroy_process_group()
