"""Generate the committed golden fixtures (run in the build container; outputs are data).

  rng_kat.json           mt19937(12345u) raw stream and PCL rnd() = raw >> 1, produced by
                         libstdc++ std::mt19937 (compiled here) and by numpy's MT19937 -- two
                         implementations independent of the oracle
  double_shadow.json     oracle results on the reference's bundled Dialog/double_shadow.pcd
                         (tests/golden/double_shadow.pcd, a byte copy of that data file):
                         PCL defaults and the 4096-hypothesis configuration
  synth_c2_small.npz     3-plane cloud (C2 shape, 16384 pts) + single-plane RANSAC results
  synth_c3_small.npz     20-plane cloud (C3 shape, 32768 pts) + extract-and-remove results

Every oracle result is cross-checked against the independent numpy twin before it is written.
No reference code is executed (the reference is an MSVC/Qt application with no Python).
"""
from __future__ import annotations

import json
import os
import subprocess
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from dialog_amd.pcd import read_pcd  # noqa: E402
from dialog_amd.synth import SEED_BASE, plane_cloud  # noqa: E402
from oracle import numpy_twin as T  # noqa: E402
from oracle import oracle as O  # noqa: E402


def f32bits(a):
    return [int(v) for v in np.asarray(a, np.float32).view(np.uint32)]


def rng_kat(n=16):
    src = r"""
#include <random>
#include <cstdio>
int main(){ std::mt19937 g(12345u); for(int i=0;i<%d;i++) printf("%%u\n", (unsigned)g()); }
""" % n
    with tempfile.TemporaryDirectory() as d:
        cpp = os.path.join(d, "mt.cpp")
        exe = os.path.join(d, "mt")
        open(cpp, "w").write(src)
        subprocess.run(["g++", "-O2", cpp, "-o", exe], check=True)
        out = subprocess.run([exe], check=True, capture_output=True, text=True).stdout.split()
    std_raw = [int(v) for v in out]
    np_raw = [int(v) for v in np.random.RandomState(12345)._bit_generator.random_raw(n)]
    assert std_raw == np_raw
    assert [int(v) for v in O.mt_stream(n)] == std_raw
    return dict(seed=12345, mt19937_raw=std_raw, rnd=[v >> 1 for v in std_raw],
                sources=["libstdc++ std::mt19937", "numpy MT19937 legacy seeding"])


def seg_record(pts, thr, **kw):
    r = O.sac_segment(pts, thr, **kw)
    t = T.sac_segment(pts, thr, max_iterations=kw.get("max_iterations", 50),
                      probability=kw.get("probability", 0.99))
    assert r["ok"] == t["ok"]
    assert np.array_equal(r["best_sample"], t["best_sample"])
    assert np.array_equal(r["coeff_unrefined"].view(np.uint32), t["coeff_unrefined"].view(np.uint32))
    assert r["iterations"] == t["iterations"] and r["draws"] == t["draws"]
    assert r["n_unrefined"] == t["n_unrefined"]
    assert np.abs(r["coeff"] - t["coeff"]).max() < 1e-5
    return r


def main():
    os.makedirs(HERE, exist_ok=True)
    with open(os.path.join(HERE, "rng_kat.json"), "w") as f:
        json.dump(rng_kat(), f, indent=1)

    pts = read_pcd(os.path.join(HERE, "double_shadow.pcd"))
    recs = {}
    for name, thr, kw in [("pcl_defaults", 0.005, dict()),
                          ("h4096", 0.005, dict(max_iterations=4095, probability=1.0)),
                          ("pcl_defaults_t02", 0.02, dict())]:
        r = seg_record(pts, thr, **kw)
        rd = O.sac_segment(pts, thr, refit_double=True, **kw)
        recs[name] = dict(threshold=thr, **{k: v for k, v in kw.items()},
                          iterations=r["iterations"], draws=r["draws"],
                          best_sample=[int(v) for v in r["best_sample"]],
                          coeff_unrefined_bits=f32bits(r["coeff_unrefined"]),
                          n_unrefined=int(r["n_unrefined"]), coeff_bits=f32bits(r["coeff"]),
                          inliers=[int(v) for v in r["inliers"]],
                          coeff_double=[float(v) for v in rd["coeff"]],
                          inliers_double=[int(v) for v in rd["inliers"]])
    with open(os.path.join(HERE, "double_shadow.json"), "w") as f:
        json.dump(dict(n_points=int(pts.shape[0]), configs=recs), f, indent=0)

    # C2-shaped small cloud: 3 planes + 10 % outliers, 4096 hypotheses in one launch
    p2, lab2, planes2 = plane_cloud(16384, 3, shares=[1, 1, 1], seed=SEED_BASE + 2)
    r = seg_record(p2, 0.02, max_iterations=4095, probability=1.0)
    np.savez_compressed(os.path.join(HERE, "synth_c2_small.npz"), points=p2, threshold=0.02,
                        max_iterations=4095, probability=1.0, best_sample=r["best_sample"],
                        coeff_unrefined=r["coeff_unrefined"], n_unrefined=r["n_unrefined"],
                        coeff=r["coeff"], inliers=r["inliers"], iterations=r["iterations"])

    # C3-shaped small cloud: 20 planes, sequential extract-and-remove
    p3, lab3, planes3 = plane_cloud(32768, 20, seed=SEED_BASE + 3)
    e = O.extract_planes(p3, 0.02, max_planes=20, min_inliers=200, max_iterations=1023,
                         probability=1.0)
    et = T.extract_planes(p3, 0.02, max_planes=20, min_inliers=200, max_iterations=1023,
                          probability=1.0)
    assert e["n_planes"] == et["n_planes"]
    assert np.array_equal(e["offsets"], et["offsets"])
    assert np.abs(e["coeffs"] - et["coeffs"]).max() < 1e-5
    np.savez_compressed(os.path.join(HERE, "synth_c3_small.npz"), points=p3, threshold=0.02,
                        max_iterations=1023, probability=1.0, min_inliers=200, max_planes=20,
                        coeffs=e["coeffs"], offsets=e["offsets"], inliers=e["inliers"])
    # normals (SURVEY.md §8(c) fixture 4): radius + k = 20 on a small 3-plane cloud, and the
    # RegulateNormal BFS from seed 0 with the seed flipped (is_norm_direction_valid = 0)
    pn, _, _ = plane_cloud(2048, 3, outlier_frac=0.05, seed=SEED_BASE + 5, patch=1.0)
    rn = O.estimate_normals(pn, 0.1)
    kn = O.estimate_normals_knn(pn, 20)
    reg, proc, _ = O.regulate_normals(pn, rn, 0, False, 0.08)
    np.savez_compressed(os.path.join(HERE, "normals_small.npz"), points=pn, radius=0.1, k=20,
                        radius_normals=rn, knn_normals=kn, seed_idx=0, r_regulate=0.08,
                        regulated=reg, processed=proc)
    # SACMODEL_NORMAL_PLANE (config C5 shape, small): radius normals from the oracle, one segment
    # and one extract-and-remove run, PCL float refit
    pp, _, _ = plane_cloud(8192, 3, outlier_frac=0.1, seed=SEED_BASE + 6, patch=2.0)
    pnrm = O.estimate_normals(pp, 0.1)
    sg = O.sac_segment(pp, 0.05, max_iterations=200, probability=0.99, normals=pnrm,
                       normal_distance_weight=0.1)
    ex = O.extract_planes(pp, 0.05, max_planes=6, min_inliers=200, max_iterations=255,
                          probability=1.0, normals=pnrm, normal_distance_weight=0.3)
    np.savez_compressed(os.path.join(HERE, "normal_plane_small.npz"), points=pp, normals=pnrm,
                        seg_threshold=0.05, seg_lambda=0.1, seg_max_iterations=200,
                        seg_probability=0.99, seg_coeff=sg["coeff"], seg_inliers=sg["inliers"],
                        seg_iterations=sg["iterations"], seg_best_sample=sg["best_sample"],
                        ex_threshold=0.05, ex_lambda=0.3, ex_max_iterations=255, ex_min_inliers=200,
                        ex_max_planes=6, ex_coeffs=ex["coeffs"], ex_offsets=ex["offsets"],
                        ex_inliers=ex["inliers"])
    print("golden fixtures written to", HERE)


if __name__ == "__main__":
    main()
