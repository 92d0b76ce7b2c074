"""The fast refit (DLG_REFIT_FAST, dialog_amd/csrc/exact_refit.hpp) on the CPU: the product's header
compiled for the host equals the oracle's independent restatement (orc_refit_exact) bit for bit,
whatever the order of the inliers, and lies within float rounding of the float64 LS plane.

The device runs the same header (tests/test_gpu_parity.py: GPU fast-mode segment / extract ==
the oracle with refit="fast", bit-exact).  Cases: planes at several scales and offsets, inliers
in forward / reversed / shuffled order, mixed magnitudes (tiny coordinates next to large ones),
n = 4, collinear and coincident inliers.
"""
import os
import subprocess

import numpy as np
import pytest

from oracle import oracle as O

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def harness(tmp_path_factory):
    exe = tmp_path_factory.mktemp("er") / "exact_refit_host"
    subprocess.run(["g++", "-std=c++17", "-O2", "-ffp-contract=off",
                    os.path.join(ROOT, "tests", "cpp", "exact_refit_host.cpp"), "-o", str(exe)],
                   check=True)
    return str(exe)


def host_refit(exe, pts, qexp, cin):
    lines = [f"{pts.shape[0]} {qexp} " + " ".join(float(c).hex() for c in cin)]
    lines += [" ".join(float(v).hex() for v in row) for row in pts]
    out = subprocess.run([exe], input="\n".join(lines) + "\n", capture_output=True, text=True,
                         check=True).stdout.split()
    return np.array([int(w, 16) for w in out], np.uint32).view(np.float32)


def ls_plane(pts):
    p = pts.astype(np.float64)
    c = p.mean(0)
    w, v = np.linalg.eigh(np.cov((p - c).T, bias=True))
    n = v[:, 0]
    return n, -n @ c


def make(case, rng):
    if case == "unit":
        n = rng.normal(size=3)
        n /= np.linalg.norm(n)
        u = np.cross(n, [1.0, 0, 0]); u /= np.linalg.norm(u)
        v = np.cross(n, u)
        st = rng.uniform(-5, 5, (5000, 2))
        p = 1.5 * n + st[:, :1] * u + st[:, 1:] * v + rng.normal(0, 0.005, (5000, 1)) * n
        return p.astype(np.float32), 5.0
    if case == "far":
        p, _ = make("unit", rng)
        return (p + np.float32(3000.0)).astype(np.float32), 3010.0
    if case == "tiny":
        p, _ = make("unit", rng)
        return (p * np.float32(1e-6)).astype(np.float32), 1e-5
    if case == "mixed":  # coordinates spanning many binades
        p, _ = make("unit", rng)
        p[::3, 0] *= np.float32(1e-9)
        return p.astype(np.float32), 20.0
    if case == "four":
        return rng.uniform(-1, 1, (4, 3)).astype(np.float32), 1.0
    if case == "collinear":
        t = rng.uniform(-1, 1, 300).astype(np.float32)
        return np.stack([t, 2 * t, -t], 1).astype(np.float32), 2.0
    if case == "coincident":
        return np.tile(np.float32([[0.25, -0.5, 2.0]]), (50, 1)), 2.0
    raise ValueError(case)


CASES = ["unit", "far", "tiny", "mixed", "four", "collinear", "coincident"]


@pytest.mark.parametrize("case", CASES)
def test_host_header_equals_oracle(harness, case):
    rng = np.random.default_rng(CASES.index(case) + 11)
    pts, fmax = make(case, rng)
    qexp = O.fast_qexp(np.vstack([pts, [[fmax, 0, 0]]]).astype(np.float32))
    cin = np.float32([0.0, 0.0, 1.0, 0.0])
    idx = np.arange(pts.shape[0], dtype=np.int32)
    ref = O.refit_exact(pts, idx, cin, qexp)
    for order in (idx, idx[::-1].copy(), rng.permutation(idx).astype(np.int32)):
        got = host_refit(harness, pts[order], qexp, cin)
        assert np.array_equal(got.view(np.uint32), ref.view(np.uint32)), (case, got, ref)
        o2 = O.refit_exact(pts, order, cin, qexp)  # the oracle is order-independent too
        assert np.array_equal(o2.view(np.uint32), ref.view(np.uint32))
    if case in ("unit", "far", "tiny", "mixed"):
        n, d = ls_plane(pts)
        if n @ ref[:3] < 0:
            n, d = -n, -d
        assert np.abs(ref[:3] - n).max() < 2e-6
        assert abs(ref[3] - d) < 2e-6 * max(1.0, abs(d))


def test_oracle_fast_segment_close_to_double(tmp_path):
    from dialog_amd.synth import plane_cloud
    p, _, _ = plane_cloud(30000, 3, seed=77)
    kw = dict(max_iterations=300, probability=1.0)
    a = O.sac_segment(p, 0.02, refit="fast", **kw)
    b = O.sac_segment(p, 0.02, refit="double", **kw)
    sg = 1.0 if a["coeff"][:3] @ b["coeff"][:3] > 0 else -1.0  # (the double twin has no orientation)
    assert np.abs(a["coeff"] - sg * b["coeff"]).max() < 1e-6
    assert a["coeff"][:3] @ a["coeff_unrefined"][:3] > 0  # fast refit keeps the unrefined side


def test_big_to_double_correctly_rounded(harness):
    """big_to_double (192-bit two's complement -> double) against Python's correctly rounded
    int -> float: random magnitudes of every bit length, exact ties, ties +- 1, all-ones runs."""
    rng = np.random.default_rng(7)
    vals = [0, 1, -1, 2**53, 2**53 + 1, 2**54 + 2, 2**54 + 6, -(2**190), 2**190 - 1]
    for L in range(1, 191):
        for _ in range(6):
            vals.append(int(rng.integers(0, 2**62)) << max(0, L - 62) | int(rng.integers(0, 2**62)))
            vals[-1] &= (1 << L) - 1
            vals[-1] |= 1 << (L - 1)
        if L > 54:
            m = (int(rng.integers(0, 2**52)) | 2**52) << (L - 53)
            half = 1 << (L - 54)
            vals += [m + half, m + half - 1, m + half + 1, m + 3 * half, (1 << L) - 1]
    vals += [-v for v in list(vals)]
    vals = [v for v in vals if -(2**191) <= v < 2**191]
    lines = []
    for v in vals:
        u = v & ((1 << 192) - 1)
        lines.append(" ".join(f"{(u >> (32 * k)) & 0xFFFFFFFF:x}" for k in range(6)))
    out = subprocess.run([harness, "B"], input="\n".join(lines) + "\n", capture_output=True,
                         text=True, check=True).stdout.split()
    got = np.array([int(w, 16) for w in out], np.uint64).view(np.float64)
    want = np.array([float(v) for v in vals], np.float64)
    bad = np.nonzero(got.view(np.uint64) != want.view(np.uint64))[0]
    assert bad.size == 0, [(vals[i], got[i], want[i]) for i in bad[:5]]
