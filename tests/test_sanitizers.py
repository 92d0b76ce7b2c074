"""Host-side sanitizer runs (ASan + UBSan) of the product's host C++ and of the oracle.

* tests/cpp/sac_control_san.cpp + dialog_amd/csrc/sac_control.cpp: the product's RANSAC controller
  (drawIndexSample replay, computeModel's loop, through its C ABI) and host_math.hpp (mt19937
  rnd(), refit_pcl_float, eigen33<float>) built with g++ -fsanitize=address,undefined, driven by a
  brute-force host scorer; its result must equal the oracle's segment() bit for bit.
* tests/cpp/oracle_san.c + oracle/pcl_oracle.c: every oracle entry point under the sanitizers.

A sanitizer finding aborts the program (-fno-sanitize-recover=all), which fails the test.  The
device code is not covered here (GPU sanitizers are not available on the pool).
"""
import os
import subprocess

import numpy as np
import pytest

from oracle import oracle as O

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SAN = ["-O1", "-g", "-ffp-contract=off", "-fsanitize=address,undefined",
       "-fno-sanitize-recover=all", "-fno-omit-frame-pointer"]
ENV = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1",
           UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")


@pytest.fixture(scope="module")
def control_exe(tmp_path_factory):
    exe = str(tmp_path_factory.mktemp("san") / "sac_control_san")
    subprocess.run(["g++", "-std=c++17", *SAN, os.path.join(ROOT, "tests/cpp/sac_control_san.cpp"),
                    os.path.join(ROOT, "dialog_amd/csrc/sac_control.cpp"), "-o", exe], check=True)
    return exe


def run_control(exe, p, thr, mi, prob, batch):
    lines = [f"{p.shape[0]} {thr!r} {mi} {prob!r} {batch}"]
    lines += [" ".join(float(v).hex() for v in row) for row in p]
    r = subprocess.run([exe], input="\n".join(lines) + "\n", capture_output=True, text=True,
                       env=ENV, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    return r.stdout.split()


@pytest.mark.parametrize("case", range(8))
def test_controller_under_sanitizers_equals_oracle(control_exe, case):
    from dialog_amd.synth import plane_cloud
    rng = np.random.default_rng(300 + case)
    n = int(rng.choice([3, 7, 200, 1500]))
    p, _, _ = plane_cloud(n, int(rng.integers(1, 4)), seed=case, outlier_frac=0.3)
    if case % 3 == 0:
        p = (np.round(p * 2) / 2).astype(np.float32)  # duplicates and collinear draws
    thr = float(rng.choice([0.01, 0.05, 0.2]))
    mi = int(rng.choice([0, 5, 50, 400]))
    prob = float(rng.choice([0.9, 0.99, 1.0]))
    batch = int(rng.choice([1, 7, 64, 0]))
    out = run_control(control_exe, p, thr, mi, prob, batch)
    r = O.sac_segment(p, thr, max_iterations=mi, probability=prob)
    assert int(out[0]) == r["iterations"] and int(out[1]) == r["draws"]
    assert bool(int(out[2])) == r["ok"]
    if r["ok"]:
        assert [int(v) for v in out[3:6]] == list(r["best_sample"])
        assert int(out[6]) == r["n_unrefined"]
        assert [int(w, 16) for w in out[7:11]] == [int(v) for v in r["coeff"].view(np.uint32)]


def test_oracle_under_sanitizers(tmp_path):
    exe = str(tmp_path / "oracle_san")
    subprocess.run(["gcc", "-std=gnu11", "-fopenmp", *SAN, os.path.join(ROOT, "tests/cpp/oracle_san.c"),
                    os.path.join(ROOT, "oracle/pcl_oracle.c"), "-lm", "-o", exe], check=True)
    r = subprocess.run([exe], capture_output=True, text=True, env=ENV, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    assert r.stdout.startswith("checksum ")


def test_alpha_shape_under_sanitizers(tmp_path):
    """The border's host module (dialog_amd/csrc/alpha_shape.hpp: Delaunay sweep-hull, alpha
    filter, PCL's polygon walk, ConcaveHull's transform chain) under ASan + UBSan, on random,
    quantised (duplicates, cocircular), collinear and tiny inputs."""
    exe = str(tmp_path / "alpha_san")
    src = tmp_path / "alpha_san.cpp"
    src.write_text(r'''
#include <cstdio>
#include <random>
#include <vector>
#include "alpha_shape.hpp"
int main() {
  std::mt19937 g(7);
  std::uniform_real_distribution<double> u(0.0, 10.0);
  long total = 0;
  for (int c = 0; c < 6; ++c) {
    const int n = c == 5 ? 3 : 2000;
    std::vector<double> xy(2 * n);
    for (int i = 0; i < n; ++i) {
      double x = u(g), y = u(g);
      if (c == 1) { x = (int)x; y = (int)y; }          // duplicates, cocircular grid points
      if (c == 2) { y = 2 * (int)x + 1; x = (int)x; }  // exactly collinear
      if (c == 3) { x *= 1e-7; y *= 1e-7; }
      xy[2 * i] = x; xy[2 * i + 1] = y;
    }
    const dlg::alpha::Tri2 T = dlg::alpha::Delaunay(xy.data(), n).run();
    const dlg::alpha::AlphaShape S = dlg::alpha::alpha_shape(xy.data(), T, c == 3 ? 1e-7 : 0.5);
    std::vector<float> p3(3 * (size_t)n);
    for (int i = 0; i < n; ++i) { p3[3 * i] = (float)xy[2 * i]; p3[3 * i + 1] = (float)xy[2 * i + 1]; p3[3 * i + 2] = 0.25f * (float)xy[2 * i]; }
    const dlg::alpha::Hull2 H = dlg::alpha::concave_hull_2d(p3.data(), n, 0.5);
    total += (long)T.tri.size() + (long)S.av.size() + (long)H.pts.size();
  }
  std::printf("%ld\n", total);
  return 0;
}
''')
    subprocess.run(["g++", "-std=c++17", *SAN, "-I", os.path.join(ROOT, "dialog_amd/csrc"), str(src),
                    "-o", exe], check=True)
    r = subprocess.run([exe], capture_output=True, text=True, env=ENV, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    assert int(r.stdout.split()[0]) > 0
