"""bench.py -- headline benchmark: point-plane inlier tests/s of the MI355X RANSAC plane path.

Workload (BASELINE.json configs[2], the 10M-point cloud the metric is quoted on): per GPU a 10M-
point synthetic cloud with 20 planes (+10 % outliers, BASELINE.md §3 generator), sequential
extract-and-remove RANSAC: each round scores 4096 hypotheses (max_iterations 4095, probability 1.0
-> k = inf, exactly 4096 PCL iterations) over the remaining points, refits with PCL's float
arithmetic (DLG_REFIT_PCL: computeMeanAndCovarianceMatrix's nine sequential float sums, evaluated
bit-exactly on the device, then PCL's float eigen33), selects and compacts the inliers; stop after
20 planes or when a plane has < 500 inliers.  One step = one full extraction from the pristine
cloud (inputs resident in HBM).  The planes and inlier lists equal the oracle's restatement of
PCL 1.8 bit for bit (tests/test_fullsize_golden.py).

Multi-GPU (one process per GPU: torchrun, or `--gpus N`, which starts the N ranks itself): weak
scaling by default -- rank r holds its own 10M-point shard of one global cloud (same 20 planes);
--global-points 100000000 runs configs[3] (C4) strong-sharded.  Every round all ranks score the
same hypotheses on their shards with one RCCL allreduce of the int32[4096] counts; the refit's
float sums run over the ranks' inlier segments in global order.

value = useful point-plane tests (PCL iterations x global active points, summed over rounds) / s,
whole job.  Roofline: the pruned scoring launch against HBM with SURVEY 8(d)'s algorithmic bytes,
with its PMC traffic, issue view and the work the pruning leaves (pruned_work).  Extra lines in
the same JSON object: refit_fast (DLG_REFIT_FAST, an exact least-squares refit -- NOT PCL's
arithmetic: its planes differ from PCL's), incl_index_build (the Morton copy + spheres rebuilt
every step), secondary (C5).  cpu_baseline: the PCL-1.8 restatement (oracle) on the box's host
cores (every CPU the process can use for countWithinDistance: its affinity mask capped by the
cgroup CPU quota; the box's 16-CPU share and a single-thread sample beside it), rank 0 at N = 1.
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
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--points", type=int, default=10_000_000, help="points per GPU (weak scaling)")
    ap.add_argument("--global-points", type=int, default=0,
                    help="strong scaling: this many points in all, sharded over the GPUs "
                         "(BASELINE configs[3], C4: 100M)")
    ap.add_argument("--planes", type=int, default=20)
    ap.add_argument("--hyps", type=int, default=4096)
    ap.add_argument("--threshold", type=float, default=0.02)
    ap.add_argument("--min-inliers", type=int, default=500)
    ap.add_argument("--refit", choices=["pcl", "fast"], default="pcl",
                    help="pcl (default): PCL's float refit, bit-exact; fast: exact LS refit (not PCL)")
    ap.add_argument("--cpu-hyps", type=int, default=1024,
                    help="hypotheses in the single-thread CPU-baseline sample")
    ap.add_argument("--cpu-threads", type=int, default=16,
                    help="threads of the all-core CPU leg (the GPU box's CPU share: 16)")
    ap.add_argument("--alt-steps", type=int, default=3,
                    help="steps of the other refit mode's line (refit_fast / refit_pcl; 0: skip)")
    ap.add_argument("--no-extras", action="store_true",
                    help="skip the other-refit, index-build and pruning-work measurements")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--torch-dist", action="store_true",
                    help="rendezvous through torch.distributed even at N=1 (runtime check)")
    ap.add_argument("--select-tile", type=int, default=0,
                    help="points per single-pass select tile (DLG_OPT_SELECT_TILE; 0: library default)")
    ap.add_argument("--opt", action="append", default=[], metavar="NAME=VALUE",
                    help="A/B only: a context option, e.g. FS_SEGMENTS=1 (DLG_OPT_FS_SEGMENTS)")
    ap.add_argument("--no-events", action="store_true",
                    help="no HIP timing events in the timed steps (A/B of their host cost)")
    ap.add_argument("--events", type=int, default=2, choices=(1, 2),
                    help="timing-event level of the timed steps (dlg_set_profiling; 2: the scoring "
                         "and select phases only, the PCL walk timed in extra untimed steps)")
    ap.add_argument("--no-secondary", action="store_true",
                    help="skip the C5 (normals + NORMAL_PLANE + post-process) secondary measurement")
    ap.add_argument("--dry-ranks", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--dry-fail-rank", type=int, default=-1, help=argparse.SUPPRESS)
    return ap.parse_args()


def c5_secondary(D, ctx, a):
    """BASELINE.json configs[4] (C5), reported beside the headline (not `value`): 10M points,
    k = 20 normals and radius normals on the GPU, then SACMODEL_NORMAL_PLANE extract-and-remove
    (weight 0.1) with the C3 RANSAC settings; plus RegulateNormal over the same cloud."""
    from dialog_amd.synth import SEED_BASE, plane_cloud
    pts, _, _ = plane_cloud(a.points, a.planes, seed=SEED_BASE + 5)
    out = {"workload": "C5: 10M-pt 20-plane cloud, k=20 normals, NORMAL_PLANE (w=0.1) extract; "
                       "postProcessPlanes on a 10M-pt 20-plane scene (1000-vertex borders); "
                       "chain_ms = device-resident normals (dlg_cloud_estimate_normals) + extract; "
                       "chain_regulate_ms = normals + RegulateNormal + extract, all on the "
                       "cloud's device copy (dlg_cloud_regulate_normals)",
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
    # the device-resident chain: k = 20 normals computed from the cloud's device copy and
    # attached to it (dlg_cloud_estimate_normals), then the NORMAL_PLANE extraction
    _, out["cloud_normals_knn20_ms"] = timed(lambda: cloud.estimate_normals(k=20))
    _, out["cloud_normals_radius0.1_ms"] = timed(lambda: cloud.estimate_normals(radius=0.1))
    prm = D.make_params(a.threshold, max_iterations=a.hyps - 1, probability=1.0,
                        refit_mode=D.DLG_REFIT_PCL if a.refit == "pcl" else D.DLG_REFIT_FAST,
                        hypotheses_per_launch=a.hyps,
                        gather_inliers=False, model=D.SACMODEL_NORMAL_PLANE,
                        normal_distance_weight=0.1)

    def step():
        cloud.reset()
        return D.extract_planes(cloud, prm, max_planes=a.planes, min_inliers=a.min_inliers,
                                capacity=a.points)

    def chain():
        cloud.estimate_normals(k=20)
        return D.extract_planes(cloud, prm, max_planes=a.planes, min_inliers=a.min_inliers,
                                capacity=a.points)

    _, out["chain_ms"] = timed(chain)
    out["chain_ms"] = round(out["chain_ms"], 2)

    def chain_regulate():
        # the reference's order: estimateNormal (k = 20) -> regulateNormal (BFS, r 0.1, seed 0)
        # -> the NORMAL_PLANE extraction on the regulated normals, all on the cloud's device copy
        # (dlg_cloud_estimate_normals, dlg_cloud_regulate_normals: no host round trip)
        cloud.estimate_normals(k=20)
        cloud.regulate_normals(0, True, 0.1)
        return D.extract_planes(cloud, prm, max_planes=a.planes, min_inliers=a.min_inliers,
                                capacity=a.points)

    cloud.estimate_normals(k=20)
    _, out["cloud_regulate_r0.1_ms"] = timed(lambda: cloud.regulate_normals(0, True, 0.1), 2)
    out["cloud_regulate_r0.1_ms"] = round(out["cloud_regulate_r0.1_ms"], 2)
    _, out["chain_regulate_ms"] = timed(chain_regulate, 1)
    out["chain_regulate_ms"] = round(out["chain_regulate_ms"], 2)
    out["cloud_normals_knn20_ms"] = round(out["cloud_normals_knn20_ms"], 2)
    out["cloud_normals_radius0.1_ms"] = round(out["cloud_normals_radius0.1_ms"], 2)
    # HBM views of the device-resident stages (SURVEY 8(d) per-point bytes: the point read once,
    # the (normal, curvature) record written once; RegulateNormal: points + normals read, normals
    # + processed flag written).  None of them is HBM-bound -- the neighbour search (cell scans,
    # candidate distances, the k-selection or the BFS frontier) bounds them -- so frac states how
    # far each stage is from streaming its data once.
    n = a.points
    views = {"normals_knn20": (28.0, out["cloud_normals_knn20_ms"]),
             "normals_radius0.1": (28.0, out["cloud_normals_radius0.1_ms"]),
             "regulate_r0.1 (host records in and out, PCIe incl.)": (37.0, out["regulate_r0.1_ms"])}
    out["rooflines"] = {
        k: {"bound": "latency (neighbour search); hbm view", "alg_bytes_per_point": b,
            "achieved": round(b * n / (ms / 1e3) / 1e9, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(b * n / (ms / 1e3) / 1e9 / HBM_PEAK_GBS, 5)}
        for k, (b, ms) in views.items() if ms}
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


def launch_ranks(n: int, argv: list[str]) -> int:
    """`bench.py --gpus N` without a launcher (no WORLD_SIZE in the environment): start N fresh
    worker processes of this script, one per GPU, with RANK / LOCAL_RANK / WORLD_SIZE / MASTER_*
    set as torch.distributed.run sets them, and wait for them.  The parent never imports torch or
    dialog_amd and makes no HIP call, so nothing is initialised on a GPU before the workers start;
    rank 0 prints the JSON line, the parent exits with the first non-zero worker status."""
    import socket
    import subprocess
    with socket.socket() as s:  # a free rendezvous port on the loopback interface
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n),
                   LOCAL_WORLD_SIZE=str(n), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__), *argv], env=env))
    rc = 0
    alive = list(procs)
    while alive:  # a failed rank ends the others (they would wait in a collective forever)
        for p in list(alive):
            c = p.poll()
            if c is None:
                continue
            alive.remove(p)
            if c != 0 and rc == 0:
                rc = c
                for q in alive:
                    q.terminate()
        time.sleep(0.05)
    return rc


def main():
    a = parse()
    if "WORLD_SIZE" not in os.environ and a.gpus > 1:
        sys.exit(launch_ranks(a.gpus, sys.argv[1:]))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if a.gpus > 1 and a.gpus != world:
        raise SystemExit(f"--gpus {a.gpus} but WORLD_SIZE={world}")
    if a.dry_ranks:  # (test of the launcher: the rank's environment, no GPU)
        env = {k: os.environ.get(k) for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_ADDR",
                                              "MASTER_PORT")}
        print(json.dumps(env), file=sys.stderr, flush=True)
        if a.dry_fail_rank >= 0:  # one rank fails, the others would wait (as in a collective)
            if int(os.environ.get("RANK", "0")) == a.dry_fail_rank:
                sys.exit(3)
            time.sleep(60)
        if int(os.environ.get("RANK", "0")) == 0:
            print(json.dumps({"n_gpus": world, "rank": 0}), flush=True)
        return
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
    ctx.set_profiling(0 if a.no_events else a.events)
    if a.select_tile:
        ctx.set_option(D.DLG_OPT_SELECT_TILE, a.select_tile)
    for o in a.opt:
        name, val = o.split("=", 1)
        ctx.set_option(getattr(D, "DLG_OPT_" + name), int(val))

    strong = a.global_points > 0
    if strong:  # C4: one global cloud sharded over the ranks (last rank takes the remainder)
        per = a.global_points // world
        a.points = per + (a.global_points - per * world if rank == world - 1 else 0)
        id_base = rank * per
    else:
        id_base = rank * a.points
    seed = SEED_BASE + (4 if strong else 3)
    t0 = time.time()
    pts, _, _ = plane_cloud(a.points, a.planes, seed=seed, shard=rank)
    gen_s = time.time() - t0
    t0 = time.perf_counter()
    cloud = D.Cloud(ctx, pts, id_base=id_base)
    ctx.synchronize()
    upload_s = time.perf_counter() - t0
    prm = D.make_params(a.threshold, max_iterations=a.hyps - 1, probability=1.0,
                        refit_mode=D.DLG_REFIT_FAST if a.refit == "fast" else D.DLG_REFIT_PCL,
                        hypotheses_per_launch=a.hyps, gather_inliers=False)

    # the caller's inlier-id buffer, kept across steps (a C++ caller's std::vector)
    inl_buf = np.empty(a.points * world if prm.gather_inliers else a.points, np.int32)
    global_points = a.global_points if strong else a.points * world

    def step():
        cloud.reset()
        return D.extract_planes(cloud, prm, max_planes=a.planes, min_inliers=a.min_inliers,
                                out=inl_buf)

    for _ in range(a.warmup):
        step()
    ctx.barrier()
    ctx.synchronize()
    tests = scored = launches = 0
    spec_misses = host_checks = 0
    score_ms = select_ms = walk_ms = 0.0
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
        walk_ms += s["refit_walk_ms"]
        spec_misses += s["spec_misses"]
        host_checks += s["pcl_host_checks"]
        planes.append(e["n_planes"])
        inliers_local += int(e["offsets"][-1])
    ctx.synchronize()
    ctx.barrier()
    elapsed = time.perf_counter() - t0
    elapsed = ctx.allreduce_max(elapsed)
    score_ms_max = ctx.allreduce_max(score_ms)
    walk_note = "timed with events on its dispatch in the timed steps"
    if not a.no_events and a.events == 2 and a.refit == "pcl":
        # the walk's own events cost the stream ~0.1 ms/step (C3): it is timed in a few extra
        # steps after the timed region instead, scaled to the timed steps' count
        ctx.set_profiling(1)
        k_ph = 3
        w_ph = 0.0
        for _ in range(k_ph):
            w_ph += step()["stats"]["refit_walk_ms"]
        ctx.synchronize()
        ctx.set_profiling(2)
        walk_ms = w_ph / k_ph * a.steps
        walk_note = (f"timed with events on its dispatch in {k_ph} extra steps after the timed "
                     "region (the timed steps carry only the scoring and select events)")

    value = tests / elapsed / 1e9  # G tests/s, whole job (tests counted over the global cloud)
    lean_rounds = int(e["stats"]["lean_rounds"])
    rounds_per_step = int(e["stats"]["rounds"])

    extras = {}
    if not a.no_extras:
        def timed_steps(fn, k):
            ctx.barrier()
            ctx.synchronize()
            t = time.perf_counter()
            out = [fn() for _ in range(k)]
            ctx.synchronize()
            ctx.barrier()
            return out, ctx.allreduce_max(time.perf_counter() - t) / k

        # (1) the other refit mode's line: DLG_REFIT_FAST beside the PCL headline (or PCL's
        # beside a --refit fast run)
        if a.alt_steps > 0:
            alt = "fast" if a.refit == "pcl" else "pcl"
            prm_alt = D.make_params(a.threshold, max_iterations=a.hyps - 1, probability=1.0,
                                    refit_mode=D.DLG_REFIT_FAST if alt == "fast" else D.DLG_REFIT_PCL,
                                    hypotheses_per_launch=a.hyps, gather_inliers=False)

            def step_alt():
                cloud.reset()
                return D.extract_planes(cloud, prm_alt, max_planes=a.planes,
                                        min_inliers=a.min_inliers, out=inl_buf)
            step_alt()
            outs, sec = timed_steps(step_alt, a.alt_steps)
            t_alt = sum(o["stats"]["tests"] for o in outs) / len(outs)
            extras["refit_" + alt] = {
                "mode": ("DLG_REFIT_FAST: exact least-squares refit (integer moments + Jacobi) -- "
                         "NOT PCL's arithmetic: its planes and inliers differ from PCL's"
                         if alt == "fast" else
                         "DLG_REFIT_PCL: PCL's float refit, bit-exact with the oracle"),
                "value": round(t_alt / sec / 1e9, 3), "unit": "G point-plane tests/s",
                "ms_per_step": round(sec * 1e3, 3), "steps": a.alt_steps,
                "planes_extracted": int(outs[-1]["n_planes"])}

        # (2) device-side, including the spatial index (Morton sort + sphere bounds) per step
        def step_index():
            cloud.drop_spatial()
            cloud.build_spatial()
            return step()
        step_index()
        outs, sec = timed_steps(step_index, max(2, min(a.steps, 5)))
        extras["incl_index_build"] = {
            "value": round(sum(o["stats"]["tests"] for o in outs) / len(outs) / sec / 1e9, 3),
            "unit": "G point-plane tests/s", "ms_per_step": round(sec * 1e3, 3),
            "note": "each step rebuilds the Hilbert-ordered copy and its bounding spheres from "
                    "the device-resident cloud (dlg_cloud_drop_spatial + dlg_cloud_build_spatial), "
                    "then extracts; inputs resident in HBM"}

        # (3) the pruned kernel's actual work (one untimed extraction with its counters on)
        ctx.set_option(D.DLG_OPT_PRUNE_STATS, 1)
        ctx.set_profiling(False)
        ep = step()
        st = ctx.prune_stats(reset=True)
        ctx.set_option(D.DLG_OPT_PRUNE_STATS, 0)
        ctx.set_profiling(0 if a.no_events else a.events)
        nl = max(int(ep["stats"]["score_launches"]), 1)
        full_pairs = ep["stats"]["tests_scored"] / world / 32.0  # (tile, plane) pairs if unpruned
        extras["pruned_work"] = {
            "pairs_evaluated_per_launch": round(st["pairs"] / nl),
            "pair_fraction": round(st["pairs"] / max(full_pairs, 1.0), 5),
            "passes_per_launch": round(st["blocks"] / nl),
            "pass_fill": round(st["pairs"] / max(128.0 * st["blocks"], 1.0), 4),
            "tile_list_entries_per_launch": round(st["list_entries"] / nl),
            # load balance: the workgroups' mean span against the longest one (100 MHz ticks)
            "workgroup_span_us_mean": round(st["wg_ticks_sum"] / max(st["workgroups"], 1) / 100.0, 2),
            "workgroup_span_us_max": round(st["wg_ticks_max"] / 100.0, 2),
            "evaluated_tests_per_step": int(32 * st["pairs"] * world),
            "note": "(tile, plane) pairs the bounding spheres could not rule out, each evaluated "
                    "as 32 exact PCL-order point tests (k_score_tiles_ex: lanes as planes, two "
                    "planes of one tile per lane, 64 lanes per pass); `value` counts PCL's tests "
                    "(iterations x active points), the kernel evaluates pair_fraction of them"}
    ms_per_step = elapsed / a.steps * 1e3
    # dominant kernel: the scoring launch (this rank's launches; tests per rank = scored / world)
    per_rank_tests = scored / world
    avg_launch_ms = score_ms / max(launches, 1)
    ktests_per_s = per_rank_tests / (score_ms / 1e3) if score_ms > 0 else 0.0
    pruned = a.points >= 131072  # (the library builds the Morton copy for such clouds)
    kname = ("k_prune_supers + k_score_tiles_ex (countWithinDistance over the Hilbert-ordered copy: "
             "super-tile and tile bounding spheres rule out (tile, plane) pairs with no possible "
             "PCL inlier; the rest evaluated exactly in PCL's f32 op order, lanes as planes; "
             f"{a.hyps} hypotheses/launch)" if pruned else
             "k_score_bf16<8> (countWithinDistance on the bf16 matrix cores + exact band "
             f"re-decision; {a.hyps} hypotheses/launch)")
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
        "algorithmic_bytes_per_launch": round(alg_bytes / max(launches, 1)),
        "avg_launch_ms": round(avg_launch_ms, 4),
        "launches": launches,
        "tests_per_s_in_kernel": ktests_per_s,
        "hbm_roofline_tests_per_s": HBM_PEAK_GBS * 1e9 / 12.0 * a.hyps,
        "valu_view": {"ops_per_test": 7, "pcl_equivalent_TFLOPs": round(7.0 * ktests_per_s / 1e12, 2),
                      "valu_peak_TFLOPs": round(VALU_PEAK_TOPS, 2)},
        "note": "north-star definition: tests/s against the HBM roofline of streaming each "
                "active point (12 B) once per 4096-hypothesis launch, i.e. achieved = algorithmic "
                "bytes (12 B x active points + 36 B x hypotheses per launch) / kernel time vs "
                "8 TB/s.  At 4096 hypotheses per pass the launch is not memory-bound (2.7e15 "
                "tests/s HBM roof): it is issue/latency-bound on the (tile, plane) pairs the "
                "bounding spheres cannot rule out -- see issue_view (PMC) and pruned_work.  "
                "Kernel time from HIP events on the library's stream.  traffic: PMC FETCH_SIZE "
                "(calibrated) + WRITE_SIZE per launch.  memory_bound_passes: the H_pass = 1 "
                "passes of each round against HBM",
    }
    if "pruned_work" in extras:
        roofline["pruned_work"] = extras.pop("pruned_work")
    # the memory-bound passes of a round (H_pass = 1), timed with HIP events around the phase
    # (incl. the small reduce/refit kernels between)
    sum_active = per_rank_tests / max(a.hyps, 1)  # sum over rounds of this rank's active points
    per_rank_points_total = a.points
    lean = pruned and lean_rounds == rounds_per_step
    if lean:
        # lean-list rounds, the phase from the scoring's end to the round's end: the speculative
        # pick, the moments over the Morton copy's near tiles (counted as 12 B per inlier: the
        # tiles whose sphere can hold one), the single-pass select of the Morton copy (16 B read,
        # 16 B per survivor, a 1 B stamp per inlier), the list from the stamps (4 B index + 1 B
        # stamp read, 4 B per survivor index, 4 + 4 B per inlier id) and the survivors' tile
        # bounding spheres (12 B per survivor read, 16 B per 32-point tile written)
        surv = sum_active - inliers_local
        sel_bytes = (12.0 * inliers_local
                     + 16.0 * sum_active + 16.0 * surv + 1.0 * inliers_local
                     + 5.0 * sum_active + 4.0 * surv + 8.0 * inliers_local
                     + 12.0 * surv + 0.5 * surv)
        if a.refit == "pcl" and "UNREFINED_LIST=0" in a.opt:
            # PCL refit instead of the moments, round 5's form: the stamp pass visits the same
            # near tiles (the 12 B per inlier above), the inlier bitmap over pristine indices is
            # written and read once per round, and the float-sum passes leave nine 64-byte chunk
            # records (9 B per inlier).  The float-sum passes' re-reads of the compacted list
            # (k_fs_prep, k_fs_inc, k_fs_l1) are implementation traffic not counted here; the
            # chains' walk (k_fs_walk: sequential, latency-bound) is timed on its own and left out
            # of this phase.
            sel_bytes += (2.0 * per_rank_points_total / 8.0 * rounds_per_step * a.steps
                          + 9.0 * inliers_local)
        elif a.refit == "pcl":
            # PCL refit, round 6 (k_ulist): the unrefined inliers from one pass over the list
            # (4 B index + 12 B coordinates per active point, 12 B per inlier written) instead of
            # the near-tile moments' 12 B per inlier above; the chunk records as before
            sel_bytes += 16.0 * sum_active + 9.0 * inliers_local
    else:
        n_copies = 2 if pruned else 1
        sel_bytes = (12.0 * sum_active + n_copies * (28.0 * sum_active + 16.0 * (sum_active - inliers_local))
                     + 4.0 * inliers_local)
    mb_ms = select_ms - walk_ms  # (the PCL refit's walk: not a memory-bound pass)
    # SURVEY 8(d)'s algorithmic bytes of the select / compaction pass: each active point read
    # once (12 B), the N-bit active mask, 4 B per emitted inlier -- per round, summed.  `frac` is
    # against these; sel_bytes above (what the implementation's passes move: the Morton copy's
    # 16-byte reads and survivor writes, the index list, stamps, bitmap, sphere bounds, ...) is the
    # implementation view, reported beside it
    alg_mb = (12.0 * sum_active + per_rank_points_total / 8.0 * rounds_per_step * a.steps
              + 4.0 * inliers_local)
    sel_gbs = alg_mb / (mb_ms / 1e3) / 1e9 if mb_ms > 0 else 0.0
    impl_gbs = sel_bytes / (mb_ms / 1e3) / 1e9 if mb_ms > 0 else 0.0
    roofline["memory_bound_passes"] = {
        "phase": "%s + selectWithinDistance + compaction (%s)"
                 % ("PCL float refit (the unrefined inliers in list order, exact float sums, "
                    "eigen33)"
                    if a.refit == "pcl" else "refit moments",
                    "lean rounds: single-pass select of the Morton copy + the index list from "
                    "the inlier stamps" if lean else
                    "list-ordered SoA and Morton copy" if pruned else "list-ordered SoA"),
        "bound": "hbm", "achieved": round(sel_gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
        "frac": round(sel_gbs / HBM_PEAK_GBS, 4),
        "algorithmic_bytes_per_step": round(alg_mb / a.steps),
        "algorithmic_bytes": "SURVEY 8(d): 12 B per active point + N/8 (active mask) + 4 B per "
                             "emitted inlier, per round",
        "traffic": {"bytes_per_step": round(sel_bytes / a.steps), "achieved": round(impl_gbs, 1),
                    "frac": round(impl_gbs / HBM_PEAK_GBS, 4),
                    "over_algorithmic": round(sel_bytes / alg_mb, 2) if alg_mb else None,
                    "note": "the bytes the implementation's passes move (counted per pass, "
                            "bench.py), not PMC"},
        "ms_per_step": round(mb_ms / a.steps, 3)}
    if walk_ms > 0:
        roofline["memory_bound_passes"]["excluded"] = {
            "refit_walk_ms_per_step": round(walk_ms / a.steps, 3),
            "note": "k_fs_walk, PCL's nine float chains walked in list order (one wave per chain, "
                    "latency-bound: DESIGN.md 5d), " + walk_note}
    # PMC-derived numbers of the same binary and workload (tools/traffic.py, tools/pmc_issue.py
    # over separate rocprofv3 --pmc passes of `bench.py --steps 1`), when present
    for fname, key in (("score_traffic.json", "traffic"), ("score_issue.json", "issue_view")):
        f = os.path.join(ROOT, "profiles", fname)
        if os.path.exists(f) and a.points == 10_000_000 and not strong:
            try:
                tj = json.load(open(f))
                if key == "traffic":
                    roofline["traffic"] = tj.get("hbm_bytes_per_launch")
                    roofline["traffic_source"] = tj.get("source")
                    if roofline["traffic"]:
                        roofline["traffic_over_algorithmic"] = round(
                            roofline["traffic"] / roofline["algorithmic_bytes_per_launch"], 3)
                else:
                    roofline["issue_view"] = tj
                    pw = roofline.get("pruned_work")
                    vi = tj.get("per_launch", {}).get("SQ_INSTS_VALU")
                    if pw and vi and pw.get("evaluated_tests_per_step") and launches:
                        # (wave instructions; evaluated tests from the stats run of the same
                        # workload: VALU lane-instructions per evaluated test)
                        ev = pw["evaluated_tests_per_step"] / world / (launches / a.steps)
                        tj["valu_lane_insts_per_evaluated_test"] = round(64.0 * vi / ev, 2)
            except Exception:
                pass

    secondary = None
    if world == 1 and not a.no_secondary:
        secondary = c5_secondary(D, ctx, a)

    cpu = None
    if rank == 0 and world == 1 and not a.no_cpu_baseline:
        from oracle import oracle as O
        model = platform.processor() or platform.machine()
        try:
            for ln in open("/proc/cpuinfo"):
                if ln.startswith("model name"):
                    model = ln.split(":", 1)[1].strip()
                    break
        except OSError:
            pass
        # three legs of the oracle's segment() (countWithinDistance over OpenMP threads; integer
        # sums: the same counts): every host CPU the process can use (the headline cpu leg: the
        # affinity mask, capped by the cgroup's CPU quota -- on the GPU box 256 CPUs in the mask
        # but a 16-CPU quota, where 256 threads ran 525 s, throttled), the box's CPU share
        # (--cpu-threads, 16 on the GPU box; the same leg when the quota already is 16), and one
        # thread (PCL 1.8's RANSAC is serial)
        try:
            affinity = len(os.sched_getaffinity(0))
        except AttributeError:
            affinity = os.cpu_count() or 1
        quota = None  # the cgroup's CPU limit (cpu.max "quota period"), in CPUs
        try:
            q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
            quota = None if q == "max" else round(int(q) / int(per), 2)
        except (OSError, ValueError):
            pass
        try:
            numa = len([d for d in os.listdir("/sys/devices/system/node") if d.startswith("node")])
        except OSError:
            numa = None

        def seg_leg(threads, hyps):
            O.set_threads(threads)
            t0 = time.perf_counter()
            r = O.sac_segment(pts, a.threshold, max_iterations=hyps - 1, probability=1.0)
            dt = time.perf_counter() - t0
            return r["iterations"] * pts.shape[0] / dt / 1e9, dt

        usable = affinity if quota is None else max(1, min(affinity, int(quota)))
        v_all, dt_all = seg_leg(usable, a.hyps)
        thr = max(1, min(a.cpu_threads, usable))
        v_share, dt_share = (v_all, dt_all) if thr == usable else seg_leg(thr, a.hyps)
        v_one, dt_one = seg_leg(1, a.cpu_hyps)
        O.set_threads(1)
        cpu = {"value": round(v_all, 4),
               "unit": "G point-plane tests/s", "cores": usable, "kind": "port",
               "sample": f"one PCL SACSegmentation::segment (the first extraction round) on the "
                         f"same {pts.shape[0]}-pt cloud with {a.hyps} hypotheses + refit + select, "
                         f"oracle/pcl_oracle.c with countWithinDistance over {usable} OpenMP "
                         f"threads (every CPU the process can use: {affinity} in its affinity "
                         f"mask, cgroup CPU quota {quota if quota is not None else 'none'}; OpenMP "
                         f"static schedule, threads placed by the OS over {numa} NUMA node(s)), "
                         f"{dt_all:.1f} s",
               "share": {"value": round(v_share, 4), "cores": thr,
                         "sample": f"the same segment() over {thr} threads (the GPU box's CPU "
                                   f"share per GPU), {dt_share:.1f} s"},
               "single_thread": {
                   "value": round(v_one, 4), "cores": 1,
                   "sample": f"the same segment() with {a.cpu_hyps} hypotheses, one thread (PCL "
                             f"1.8's RANSAC is serial), {dt_one:.1f} s"},
               "host_cpu": model, "host_nproc": os.cpu_count(), "affinity_cpus": affinity,
               "cgroup_cpu_quota": quota, "numa_nodes": numa}

    if rank == 0:
        xchg = ("RCCL allreduce of the hypotheses' counts; the PCL refit's nine float chains "
                "walked over the ranks' inlier segments in global order (each rank from its "
                "guess, repaired from the previous rank's 9-float end state)"
                if a.refit == "pcl" else
                "RCCL allreduce of the hypotheses' counts and of exact refit moments")
        out = {
            "metric": METRIC, "value": round(value, 3), "unit": "G point-plane tests/s",
            "n_gpus": world, "steps": a.steps, "warmup": a.warmup,
            "ms_per_step": round(ms_per_step, 3), "higher_is_better": True,
            "scaling": "strong" if strong else "weak",
            "vs_baseline": None, "dtype": "f32", "data": "synthetic",
            "config": {"workload": (
                           "C4: 100M-pt 20-plane synthetic cloud sharded over the GPUs "
                           "(BASELINE.json configs[3]), sequential extract-and-remove RANSAC, "
                           + xchg if strong else
                           ("C3: sequential extract-and-remove RANSAC, 10M-pt 20-plane synthetic "
                            "cloud per GPU (BASELINE.json configs[2]; N>1: shards of one cloud, "
                            + xchg + ")"
                            if a.points == 10_000_000 and a.planes == 20 else
                            f"sequential extract-and-remove RANSAC, {a.points / 1e6:g}M-pt "
                            f"{a.planes}-plane synthetic cloud per GPU (not the C3 size: "
                            f"{'C4 shape on one GPU' if a.points == 100_000_000 else 'custom'})")),
                       "points_per_gpu": a.points, "global_points": global_points,
                       "planes": a.planes, "hypotheses_per_round": a.hyps,
                       "threshold": a.threshold, "min_inliers": a.min_inliers,
                       "refit": a.refit, "planes_extracted": planes[-1] if planes else 0,
                       "lean_rounds": lean_rounds, "rounds": rounds_per_step,
                       "parallelism": f"point-sharded x{world}"},
            "roofline": roofline,
            "cpu_baseline": cpu,
            **extras,
            "secondary": secondary,
            "step_ms": [round(x, 2) for x in step_ms],  # this rank's host time per step
            "tests_per_step": tests // max(a.steps, 1),
            # hypotheses launched x active points (= tests_per_step for p = 1 workloads); the
            # tests the pruned kernel actually evaluates: roofline.pruned_work
            "tests_launched_per_step": scored // max(a.steps, 1),
            "score_ms_per_step_max_rank": round(score_ms_max / a.steps, 3),
            "select_ms_per_step": round(select_ms / a.steps, 3),
            "refit_walk_ms_per_step": round(walk_ms / a.steps, 3),
            # speculative computeModel decisions the host replay overturned (each redoes its
            # round's refit + select), and PCL-refit tails the host had to confirm
            "spec_misses_per_step": round(spec_misses / a.steps, 3),
            "pcl_host_checks_per_step": round(host_checks / a.steps, 3),
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
