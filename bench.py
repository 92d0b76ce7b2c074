"""bench.py -- headline benchmark: point-plane inlier tests/s of the MI355X RANSAC plane path.

Workload (BASELINE.json configs[2], the 10M-point cloud the metric is quoted on): per GPU a 10M-
point synthetic cloud with 20 planes (+10 % outliers, BASELINE.md §3 generator), sequential
extract-and-remove RANSAC: each round scores 4096 hypotheses (max_iterations 4095, probability 1.0
-> k = inf, exactly 4096 PCL iterations) over the remaining points, refits (fast double mode),
selects and compacts the inliers; stop after 20 planes or when a plane has < 500 inliers.
One step = one full extraction from the pristine cloud (inputs resident in HBM).

Multi-GPU (weak scaling, torchrun one process per GPU): rank r holds its own 10M-point shard of
one global cloud (same 20 planes); every round all ranks score the same hypotheses on their
shards with one RCCL allreduce of the int32[4096] counts.

value = useful point-plane tests (PCL iterations x global active points, summed over rounds) / s,
whole job.  Roofline: the scoring kernel (k_score_bf16 by default), against the f32 VALU peak with
SURVEY 8(d)'s algorithmic 7 ops per test, timed with HIP events on the library's stream.  cpu_baseline: the PCL-1.8 restatement (oracle, 1 thread) on
a bounded sample of the same workload, rank 0 at N = 1 only.
"""
from __future__ import annotations

import argparse
import json
import os
import platform
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "G point–plane inlier tests/sec + %HBM-roofline, 10M-pt cloud, 1/2/4/8 GPU"
VALU_PEAK_TOPS = 256 * 4 * 32 * 2.4e9 / 1e12   # f32 VALU lane-ops/s (no FMA): 78.6 T
HBM_PEAK_GBS = 8000.0


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--points", type=int, default=10_000_000, help="points per GPU")
    ap.add_argument("--planes", type=int, default=20)
    ap.add_argument("--hyps", type=int, default=4096)
    ap.add_argument("--threshold", type=float, default=0.02)
    ap.add_argument("--min-inliers", type=int, default=500)
    ap.add_argument("--refit", choices=["fast", "pcl"], default="fast")
    ap.add_argument("--cpu-hyps", type=int, default=1024, help="hypotheses in the CPU-baseline sample")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--torch-dist", action="store_true",
                    help="rendezvous through torch.distributed even at N=1 (runtime check)")
    ap.add_argument("--no-events", action="store_true",
                    help="no HIP timing events in the timed steps (A/B of their host cost)")
    ap.add_argument("--no-secondary", action="store_true",
                    help="skip the C5 (normals + NORMAL_PLANE + post-process) secondary measurement")
    return ap.parse_args()


def c5_secondary(D, ctx, a):
    """BASELINE.json configs[4] (C5), reported beside the headline (not `value`): 10M points,
    k = 20 normals and radius normals on the GPU, then SACMODEL_NORMAL_PLANE extract-and-remove
    (weight 0.1) with the C3 RANSAC settings; plus RegulateNormal over the same cloud."""
    from dialog_amd.synth import SEED_BASE, plane_cloud
    pts, _, _ = plane_cloud(a.points, a.planes, seed=SEED_BASE + 5)
    out = {"workload": "C5: 10M-pt 20-plane cloud, k=20 normals, NORMAL_PLANE (w=0.1) extract; "
                       "postProcessPlanes on a 10M-pt 20-plane scene (1000-vertex borders)",
           "points": a.points}

    def timed(f, reps=2):
        f()
        ctx.synchronize()
        t0 = time.perf_counter()
        for _ in range(reps):
            r = f()
        ctx.synchronize()
        return r, (time.perf_counter() - t0) / reps * 1e3

    nrm, out["normals_knn20_ms"] = timed(lambda: D.estimate_normals(pts, k=20, ctx=ctx))
    rn, out["normals_radius0.1_ms"] = timed(lambda: D.estimate_normals(pts, radius=0.1, ctx=ctx))
    reg, out["regulate_r0.1_ms"] = timed(lambda: D.regulate_normals(pts, rn, 0, True, 0.1, ctx=ctx), 1)
    out["regulate_reached"] = reg[2]
    # preProcess with the reference's default min_dist_between_points (Dialog/config.txt:3)
    pp, out["preprocess_0.001_ms"] = timed(lambda: D.preprocess(pts, 0.001, ctx=ctx), 1)
    out["preprocess_kept"] = int(len(pp[1]))
    cloud = D.Cloud(ctx, pts)
    cloud.set_normals(nrm)
    prm = D.make_params(a.threshold, max_iterations=a.hyps - 1, probability=1.0,
                        refit_mode=D.DLG_REFIT_FAST, hypotheses_per_launch=a.hyps,
                        gather_inliers=False, model=D.SACMODEL_NORMAL_PLANE,
                        normal_distance_weight=0.1)

    def step():
        cloud.reset()
        return D.extract_planes(cloud, prm, max_planes=a.planes, min_inliers=a.min_inliers,
                                capacity=a.points)

    e, ms = timed(step)
    st = e["stats"]
    out.update({"np_extract_ms": round(ms, 2), "np_planes": e["n_planes"],
                "np_value": round(st["tests"] / (ms / 1e3) / 1e9, 3),
                "np_unit": "G point-plane tests/s",
                "np_kernel_tests_per_s": round(st["tests_scored"] / (st["score_ms"] / 1e3) / 1e9, 3)
                if st["score_ms"] else None})
    for k in ("normals_knn20_ms", "normals_radius0.1_ms", "regulate_r0.1_ms", "preprocess_0.001_ms"):
        out[k] = round(out[k], 2)
    cloud.close()
    # postProcessPlanes on the same cloud size: 70% of each plane's points in its points_set,
    # 1000-vertex concave borders, config.ini [PlaneDetect] T_dist 0.1 / radius_local 0.1 /
    # T_cluster_num 500
    from dialog_amd.synth import postprocess_scene
    pc, planes = postprocess_scene(a.points, a.planes, n_border=1000, seed=SEED_BASE + 5)
    pprm = D.PostProcessParams(0.1, 0.1, 500, 0, 12345)
    po, out["post_process_ms"] = timed(lambda: D.post_process_planes(pc, planes, pprm, ctx=ctx))
    out["post_process_ms"] = round(out["post_process_ms"], 2)
    out["post_absorbed"] = int(sum(x.size for x in po[1]))
    out["post_remaining"] = int(po[2].size)
    return out


def main():
    a = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    use_torch = world > 1 or a.torch_dist
    dist = None
    if use_torch:
        # torch first (its HIP runtime then serves libdialog_amd.so too: one runtime per process);
        # gloo on the CPU only carries the RCCL unique id.  The data path is RCCL inside the lib.
        import torch.distributed as dist  # noqa: F811
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29533")
        dist.init_process_group("gloo", rank=rank, world_size=world)
    import dialog_amd as D
    from dialog_amd.synth import SEED_BASE, plane_cloud

    if world > 1:
        uid = D.Context.unique_id() if rank == 0 else None
        box = [uid]
        dist.broadcast_object_list(box, src=0)
        ctx = D.Context.distributed(local, rank, world, box[0])
    else:
        ctx = D.Context(local)
    ctx.set_profiling(not a.no_events)

    seed = SEED_BASE + 3
    t0 = time.time()
    pts, _, _ = plane_cloud(a.points, a.planes, seed=seed, shard=rank)
    gen_s = time.time() - t0
    t0 = time.perf_counter()
    cloud = D.Cloud(ctx, pts, id_base=rank * a.points)
    ctx.synchronize()
    upload_s = time.perf_counter() - t0
    prm = D.make_params(a.threshold, max_iterations=a.hyps - 1, probability=1.0,
                        refit_mode=D.DLG_REFIT_FAST if a.refit == "fast" else D.DLG_REFIT_PCL,
                        hypotheses_per_launch=a.hyps, gather_inliers=False)

    # the caller's inlier-id buffer, kept across steps (a C++ caller's std::vector)
    inl_buf = np.empty(a.points * world if prm.gather_inliers else a.points, np.int32)

    def step():
        cloud.reset()
        return D.extract_planes(cloud, prm, max_planes=a.planes, min_inliers=a.min_inliers,
                                out=inl_buf)

    for _ in range(a.warmup):
        step()
    ctx.barrier()
    ctx.synchronize()
    tests = scored = launches = 0
    score_ms = select_ms = 0.0
    planes = []
    inliers_local = 0  # this rank's inliers over the timed steps
    t0 = time.perf_counter()
    step_ms = []
    for _ in range(a.steps):
        ts = time.perf_counter()
        e = step()
        step_ms.append((time.perf_counter() - ts) * 1e3)
        s = e["stats"]
        tests += s["tests"]
        scored += s["tests_scored"]
        launches += s["score_launches"]
        score_ms += s["score_ms"]
        select_ms += s["select_ms"]
        planes.append(e["n_planes"])
        inliers_local += int(e["offsets"][-1])
    ctx.synchronize()
    ctx.barrier()
    elapsed = time.perf_counter() - t0
    elapsed = ctx.allreduce_max(elapsed)
    score_ms_max = ctx.allreduce_max(score_ms)

    value = tests / elapsed / 1e9  # G tests/s, whole job (tests counted over the global cloud)
    ms_per_step = elapsed / a.steps * 1e3
    # dominant kernel: k_score (this rank's launches; tests per rank = scored / world)
    per_rank_tests = scored / world
    avg_launch_ms = score_ms / max(launches, 1)
    ktests_per_s = per_rank_tests / (score_ms / 1e3) if score_ms > 0 else 0.0
    variant = int(os.environ.get("DLG_SCORE_VARIANT", "19"))
    pruned = variant == 19 and os.environ.get("DLG_PRUNE", "") != "0" and a.points >= 131072
    if pruned:
        kname = ("k_score_pruned (countWithinDistance over the Morton-ordered copy: super-tile and "
                 "tile bounding spheres rule out (tile, plane) pairs with no possible PCL inlier; "
                 "the rest as k_score_bf16's 32x32 bf16 matrix-core blocks + exact band "
                 "re-decision; 4096 hypotheses/launch)")
    else:
        kname = {19: "k_score_bf16<8> (countWithinDistance: plane distances on the bf16 matrix "
                     "cores, exact 3-way split operands; VALU sign count + rounding-band "
                     "re-decision in PCL op order; 4096 hypotheses/launch)",
                 5: "k_score<exact,4> (countWithinDistance in PCL op order on the VALU, 4096 "
                    "hypotheses/launch)"}.get(variant, f"score variant {variant}")
    # SURVEY 8(d) algorithmic bytes of a scoring launch: the active points once (12 B each) +
    # the hypotheses (32 B plane record + 4 B count); sum over launches / kernel time
    alg_bytes = 12.0 * per_rank_tests / max(a.hyps, 1) + 36.0 * a.hyps * launches
    achieved = alg_bytes / (score_ms / 1e3) / 1e9 if score_ms else 0.0
    roofline = {
        "kernel": kname,
        "bound": "hbm",
        "achieved": round(achieved, 2),
        "peak": HBM_PEAK_GBS,
        "unit": "GB/s",
        "frac": round(achieved / HBM_PEAK_GBS, 4),
        "traffic": None,
        "avg_launch_ms": round(avg_launch_ms, 4),
        "launches": launches,
        "tests_per_s_in_kernel": ktests_per_s,
        "hbm_roofline_tests_per_s": HBM_PEAK_GBS * 1e9 / 12.0 * a.hyps,
        "valu_view": {"ops_per_test": 7, "pcl_equivalent_TFLOPs": round(7.0 * ktests_per_s / 1e12, 2),
                      "valu_peak_TFLOPs": round(VALU_PEAK_TOPS, 2)},
        "note": "north-star definition: tests/s against the HBM roofline of streaming each "
                "active point (12 B) once per 4096-hypothesis launch, i.e. achieved = algorithmic "
                "bytes (12 B x active points + 36 B x hypotheses per launch) / kernel time vs "
                "8 TB/s; frac = tests/s / hbm_roofline_tests_per_s.  At 4096 hypotheses per "
                "pass the launch is not memory-bound (2.7e15 tests/s HBM roof); it is issue/"
                "latency-bound on the (tile, plane) pairs the bounding spheres cannot rule out "
                "(DESIGN.md sec. 5).  Kernel time from HIP events on the library's stream.  "
                "valu_view restates the same tests as PCL's 7 f32 ops each (exceeds the VALU "
                "peak because the pruned kernel skips the pairs it rules out).  "
                "memory_bound_passes: the H_pass = 1 passes of each round against HBM",
    }
    # the memory-bound passes of a round (H_pass = 1): fast refit moments (12 B/pt), then
    # selectWithinDistance + compaction of the list-ordered SoA and of the Morton copy (each: a
    # 12 B/pt count pass, a 16 B/pt read + 16 B/survivor write scatter; 4 B per inlier id);
    # timed with HIP events around the phase (incl. the small reduce/refit kernels between)
    sum_active = per_rank_tests / max(a.hyps, 1)  # sum over rounds of this rank's active points
    n_copies = 2 if pruned else 1
    lean = pruned and world == 1 and os.environ.get("DLG_LEAN", "") != "0" and a.refit == "fast"
    if lean:
        # lean-list rounds: moments (12 B/pt) and the single-pass select of the Morton copy (16 B
        # read, 16 B per survivor, a 1 B stamp per inlier), then the list from the stamps (4 B
        # index + 1 B stamp read, 4 B per survivor index, 4 + 4 B per inlier id)
        sel_bytes = (12.0 * sum_active + 16.0 * sum_active + 16.0 * (sum_active - inliers_local)
                     + 1.0 * inliers_local + 5.0 * sum_active
                     + 4.0 * (sum_active - inliers_local) + 8.0 * inliers_local)
    else:
        sel_bytes = (12.0 * sum_active + n_copies * (28.0 * sum_active + 16.0 * (sum_active - inliers_local))
                     + 4.0 * inliers_local)
    sel_gbs = sel_bytes / (select_ms / 1e3) / 1e9 if select_ms > 0 else 0.0
    roofline["memory_bound_passes"] = {
        "phase": "refit moments + selectWithinDistance + compaction (%s)"
                 % ("lean rounds: single-pass select of the Morton copy + the index list from "
                    "the inlier stamps" if lean else
                    "list-ordered SoA and Morton copy" if pruned else "list-ordered SoA"),
        "bound": "hbm", "achieved": round(sel_gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
        "frac": round(sel_gbs / HBM_PEAK_GBS, 4), "bytes_per_step": round(sel_bytes / a.steps),
        "ms_per_step": round(select_ms / a.steps, 3)}
    traffic_file = os.path.join(ROOT, "profiles", "score_traffic.json")
    if os.path.exists(traffic_file):
        try:
            tj = json.load(open(traffic_file))
            roofline["traffic"] = tj.get("hbm_bytes_per_launch")
            roofline["traffic_source"] = tj.get("source")
        except Exception:
            pass

    secondary = None
    if world == 1 and not a.no_secondary:
        secondary = c5_secondary(D, ctx, a)

    cpu = None
    if rank == 0 and world == 1 and not a.no_cpu_baseline:
        from oracle import oracle as O
        t0 = time.perf_counter()
        r = O.sac_segment(pts, a.threshold, max_iterations=a.cpu_hyps - 1, probability=1.0)
        cdt = time.perf_counter() - t0
        cpu = {"value": round(r["iterations"] * pts.shape[0] / cdt / 1e9, 4),
               "unit": "G point-plane tests/s", "cores": 1, "kind": "port",
               "sample": f"one PCL SACSegmentation::segment (first extraction round) on the same "
                         f"{pts.shape[0]}-pt cloud with {a.cpu_hyps} hypotheses + refit + select, "
                         f"oracle/pcl_oracle.c single thread, {cdt:.1f} s",
               "host_cpu": platform.processor() or platform.machine(),
               "host_nproc": os.cpu_count()}

    if rank == 0:
        out = {
            "metric": METRIC, "value": round(value, 3), "unit": "G point-plane tests/s",
            "n_gpus": world, "steps": a.steps, "warmup": a.warmup,
            "ms_per_step": round(ms_per_step, 3), "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "f32", "data": "synthetic",
            "config": {"workload": "C3: sequential extract-and-remove RANSAC, 10M-pt 20-plane "
                                   "synthetic cloud per GPU (BASELINE.json configs[2]; C4 shape "
                                   "when N>1: shards of one cloud, RCCL allreduce of counts)",
                       "points_per_gpu": a.points, "global_points": a.points * world,
                       "planes": a.planes, "hypotheses_per_round": a.hyps,
                       "threshold": a.threshold, "min_inliers": a.min_inliers,
                       "refit": a.refit, "planes_extracted": planes[-1] if planes else 0,
                       "parallelism": f"point-sharded x{world}"},
            "roofline": roofline,
            "cpu_baseline": cpu,
            "secondary": secondary,
            "step_ms": [round(x, 2) for x in step_ms],  # this rank's host time per step
            "tests_per_step": tests // max(a.steps, 1),
            "tests_scored_per_step": scored // max(a.steps, 1),
            "score_ms_per_step_max_rank": round(score_ms_max / a.steps, 3),
            "select_ms_per_step": round(select_ms / a.steps, 3),
            "gen_s": round(gen_s, 2),
            # PCIe-inclusive view (never `value`): host xyz -> SoA upload of this rank's shard
            "upload_ms": round(upload_s * 1e3, 2),
            "value_incl_upload": round(tests / (elapsed + a.steps * upload_s) / 1e9, 3),
        }
        print(json.dumps(out), flush=True)
    cloud.close()
    ctx.close()
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
