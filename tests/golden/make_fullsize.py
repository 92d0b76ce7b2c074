"""Full-size golden summaries (BASELINE.json configs at their quoted sizes) from the oracle.

Run in the build container (the oracle's countWithinDistance on all host cores; integer counts, so
the thread count does not change a result).  Writes tests/golden/fullsize.json: per workload the
SHA-256 of the generated float32 cloud (the GPU test checks it reproduced the same input), and per
refit mode the RANSAC result: iterations / best sample / coefficient bit patterns / inlier counts
and the SHA-256 of every plane's inlier-id list (int32 little-endian, list order).

  c2        1M points, 3 planes (+10 % outliers), 4096 hypotheses, one segment()  [configs[1]]
  c3        10M points, 20 planes, extract-and-remove, 4096 hypotheses per round [configs[2]]
  c4shape   100M points, 20 planes, the same extraction (C4 on one GPU)          [configs[3]]
  c5        10M points, 20 planes: k = 20 normals -> RegulateNormal (seed point 0, outward,
            r 0.1) -> SACMODEL_NORMAL_PLANE (w 0.1) extract-and-remove               [configs[4]]
            (the SHA-256 of the normals' and the regulated normals' float32 bits, the number
            of points the BFS reached, then the extraction as above)

Modes: "pcl" (PCL's float refit, DLG_REFIT_PCL), "fast" (the product's exact-moment refit,
DLG_REFIT_FAST -- the bench's mode), "none" (optimize off: lean rounds without a refit).
Usage: python tests/golden/make_fullsize.py [c2[:mode,...]] [c3[:...]] [c4shape] [--threads N]
(a workload without modes runs all of its modes; existing entries of other modes are kept)
"""
from __future__ import annotations

import hashlib
import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from dialog_amd.synth import SEED_BASE, plane_cloud  # noqa: E402
from oracle import oracle as O  # noqa: E402

OUT = os.path.join(HERE, "fullsize.json")
THR = 0.02

WORKLOADS = {
    "c2": dict(n=1_000_000, planes=3, seed=SEED_BASE + 2, shares=[1, 1, 1], kind="segment",
               modes=["pcl", "fast"]),
    "c3": dict(n=10_000_000, planes=20, seed=SEED_BASE + 3, kind="extract",
               modes=["fast", "pcl", "none"]),
    "c4shape": dict(n=100_000_000, planes=20, seed=SEED_BASE + 4, kind="extract",
                    modes=["fast", "pcl"]),
    "c5": dict(n=10_000_000, planes=20, seed=SEED_BASE + 5, kind="np_chain",
               modes=["pcl", "fast"], k=20, reg_seed=0, reg_outward=True, reg_radius=0.1,
               weight=0.1),
}


def sha(a) -> str:
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def cloud(w):
    p, _, _ = plane_cloud(w["n"], w["planes"], seed=w["seed"], shares=w.get("shares"))
    return p


_NORMALS = {}


def np_chain_normals(w, p):
    """k-NN normals -> RegulateNormal (oracle), cached per workload; -> (normals, regulated,
    reached, summary)"""
    if "c5" not in _NORMALS:
        t0 = time.time()
        nrm = O.estimate_normals_knn(p, w["k"])
        t1 = time.time()
        reg, _, reached = O.regulate_normals(p, nrm, w["reg_seed"], w["reg_outward"], w["reg_radius"])
        t2 = time.time()
        print(f"c5 normals {t1 - t0:.1f} s, regulate {t2 - t1:.1f} s", flush=True)
        _NORMALS["c5"] = (reg, dict(k=w["k"], normals_sha256=sha(nrm), reg_seed=w["reg_seed"],
                                    reg_outward=w["reg_outward"], reg_radius=w["reg_radius"],
                                    reached=int(reached), regulated_sha256=sha(reg),
                                    weight=w["weight"], oracle_normals_s=round(t1 - t0, 1),
                                    oracle_regulate_s=round(t2 - t1, 1)))
    return _NORMALS["c5"]


def run(name, w, p, mode):
    kw = dict(max_iterations=4095, probability=1.0)
    if w["kind"] == "np_chain":
        kw["normals"] = np_chain_normals(w, p)[0]
        kw["normal_distance_weight"] = w["weight"]
    if mode == "none":
        kw["optimize"] = False
    else:
        kw["refit"] = mode
    t0 = time.time()
    if w["kind"] == "segment":
        r = O.sac_segment(p, THR, **kw)
        rec = dict(iterations=r["iterations"], draws=int(r["draws"]),
                   best_sample=[int(v) for v in r["best_sample"]],
                   coeff_unrefined_bits=[int(v) for v in r["coeff_unrefined"].view(np.uint32)],
                   n_unrefined=int(r["n_unrefined"]),
                   coeff_bits=[int(v) for v in r["coeff"].view(np.uint32)],
                   n_inliers=int(r["inliers"].size), inliers_sha256=sha(r["inliers"]))
    else:
        e = O.extract_planes(p, THR, max_planes=20, min_inliers=500, **kw)
        offs = e["offsets"]
        rec = dict(n_planes=int(e["n_planes"]),
                   coeff_bits=[[int(v) for v in c.view(np.uint32)] for c in e["coeffs"]],
                   counts=[int(offs[k + 1] - offs[k]) for k in range(e["n_planes"])],
                   inliers_sha256=[sha(e["inliers"][offs[k]:offs[k + 1]])
                                   for k in range(e["n_planes"])])
    rec["oracle_s"] = round(time.time() - t0, 1)
    print(f"{name}/{mode}: {rec['oracle_s']} s", flush=True)
    return rec


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    threads = os.cpu_count() or 1
    if "--threads" in sys.argv:
        threads = int(sys.argv[sys.argv.index("--threads") + 1])
        args = [a for a in args if a != str(threads)]
    O.set_threads(threads)
    todo = args or ["c2", "c3"]
    db = json.load(open(OUT)) if os.path.exists(OUT) else {}
    db["_about"] = ("oracle (oracle/pcl_oracle.c) results at BASELINE.json's full sizes; "
                    "generated by tests/golden/make_fullsize.py; threshold 0.02, 4095 max "
                    "iterations, probability 1 (4096 hypotheses per round), min_inliers 500")
    for item in todo:
        name, _, ms = item.partition(":")
        w = WORKLOADS[name]
        p = cloud(w)
        ent = dict(n_points=w["n"], planes=w["planes"], seed=w["seed"], kind=w["kind"],
                   shares=w.get("shares"), threshold=THR, cloud_sha256=sha(p),
                   modes=db.get(name, {}).get("modes", {}))
        if w["kind"] == "np_chain":
            ent["chain"] = np_chain_normals(w, p)[1]
        if db.get(name, {}).get("cloud_sha256", ent["cloud_sha256"]) != ent["cloud_sha256"]:
            ent["modes"] = {}
        for mode in (ms.split(",") if ms else w["modes"]):
            ent["modes"][mode] = run(name, w, p, mode)
            db[name] = ent
            json.dump(db, open(OUT, "w"), indent=1)
        del p
    print("written", OUT)


if __name__ == "__main__":
    main()
