"""CPU: PCL's sequential float sums evaluated in parallel (dialog_amd/csrc/fsum.hpp).

The device's DLG_REFIT_PCL refit (fsum.hip) evaluates computeMeanAndCovarianceMatrix's nine
sequential float accumulators by fan runs around guessed starts, translated where the lemma of
fsum.hpp proves the shift exact, descended into otherwise.  tests/cpp/fsum_host.cpp builds the same
records with the same header on the host; here they must equal the literal loop (PCL's
`accu[k] += ...` in list order) bit for bit on inputs chosen to break a sloppy version: sums that
hover around zero and change binade every few steps, drifting sums, quantised values (rounding
ties everywhere), mixed magnitudes 1e-20..1e20, subnormals, exact zeros, values whose squares
overflow, constant and alternating sequences, and guesses perturbed by up to 200 quanta (so the
failed lanes and the reruns run).  Sizes straddle the chunk (64) and unit (4096) boundaries, with
walk windows of 64 records (the device's), 7 and 1.

Also: the device form of the refit's tail (transcendentals checked against float rounding
boundaries) equals the host refit_pcl_float on the same sums; the "uncertain" flag is rare.
"""
import ctypes
import os
import subprocess

import numpy as np
import pytest

from dialog_amd.synth import plane_cloud

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
P = ctypes.c_void_p


@pytest.fixture(scope="module")
def fs(tmp_path_factory):
    so = tmp_path_factory.mktemp("fsum") / "libfsum_host.so"
    subprocess.run(["g++", "-std=c++17", "-O2", "-ffp-contract=off", "-shared", "-fPIC",
                    os.path.join(ROOT, "tests", "cpp", "fsum_host.cpp"), "-o", str(so)], check=True)
    return ctypes.CDLL(str(so))


def run(fs, x, y, z, width=64, noise=0):
    x, y, z = (np.ascontiguousarray(v, np.float32) for v in (x, y, z))
    n = x.size
    out = np.zeros(9, np.float32)
    st = np.zeros(3, np.int64)
    fs.fs_host(P(x.ctypes.data), P(y.ctypes.data), P(z.ctypes.data), ctypes.c_int64(n),
               ctypes.c_int(width), ctypes.c_int(noise), P(out.ctypes.data), P(st.ctypes.data))
    ref = np.zeros(9, np.float32)
    fs.fs_literal(P(x.ctypes.data), P(y.ctypes.data), P(z.ctypes.data), ctypes.c_int64(n),
                  P(ref.ctypes.data))
    return out, ref, st


def same_bits(a, b):
    return np.array_equal(a.view(np.uint32), b.view(np.uint32))


def gen(kind, n, rng):
    if kind == "hover":
        a = rng.normal(size=(3, n))
    elif kind == "quant":
        a = np.round(rng.normal(size=(3, n)) * 8) / 8
    elif kind == "mags":
        a = rng.normal(size=(3, n)) * 10.0 ** rng.integers(-20, 20, size=(3, n))
    elif kind == "drift":
        a = rng.normal(loc=0.001, size=(3, n))
    elif kind == "zeros":
        a = rng.normal(size=(3, n)) * (rng.random((3, n)) < 0.3)
    elif kind == "subnormal":
        a = rng.normal(size=(3, n)) * 1e-20
    elif kind == "const":
        a = np.full((3, n), 0.1)
    elif kind == "alternating":
        a = np.tile([1e6, -1e6 + 0.5, 3.0], (3, n // 3 + 1))[:, :n]
    elif kind == "far":
        a = rng.normal(size=(3, n)) + 1000
    elif kind == "ints":
        a = rng.integers(-3, 4, size=(3, n)).astype(float)
    elif kind == "overflow":
        a = rng.normal(size=(3, n)) * 1e18
    else:
        raise ValueError(kind)
    return a.astype(np.float32)


KINDS = ["hover", "quant", "mags", "drift", "zeros", "subnormal", "const", "alternating", "far",
         "ints", "overflow"]
SIZES = [1, 2, 3, 63, 64, 65, 4095, 4096, 4097, 70000]


@pytest.mark.parametrize("kind", KINDS)
def test_parallel_sums_equal_literal_loop(fs, kind):
    rng = np.random.default_rng(KINDS.index(kind) + 11)
    for n in SIZES:
        for width, noise in ((64, 0), (7, 0), (64, 3), (1, 200)):
            x, y, z = gen(kind, n, rng)
            out, ref, _ = run(fs, x, y, z, width, noise)
            nan = np.isnan(ref)
            assert np.array_equal(np.isnan(out), nan), (kind, n, width, noise)
            assert same_bits(out[~nan], ref[~nan]), (kind, n, width, noise, out, ref)


def test_parallel_sums_on_plane_inliers(fs):
    """The refit's real input: inliers of a C3-like cloud's planes (10 x 10 patches, offsets in
    [-5, 5], list order), several hundred thousand points, three window widths."""
    p, _, planes = plane_cloud(3_000_000, 12, seed=0xD1A106 + 3)
    for k in range(0, 12, 3):
        d = np.abs(p.astype(np.float64) @ planes[k, :3] + planes[k, 3])
        sel = np.nonzero(d < 0.02)[0]
        x, y, z = p[sel, 0], p[sel, 1], p[sel, 2]
        for width in (1, 8, 64):
            out, ref, st = run(fs, x, y, z, width)
            assert same_bits(out, ref), (k, width)
        # the walk (64 wide, as on the device) mostly translates: lanes handled alone and reruns
        # are a small share of the nine chains' chunk records
        assert st[1] + st[2] < 0.05 * 9 * (sel.size / 64 + 1), st


def test_refit_tail_device_form_equals_host(fs):
    """fs_refit_tail (device arithmetic, transcendentals checked) == refit_pcl_float on the same
    inliers whenever it reports certainty; the flag itself is rare."""
    rng = np.random.default_rng(5)
    unc = 0
    for t in range(300):
        n = int(rng.integers(4, 2000))
        nrm = rng.normal(size=3)
        nrm /= np.linalg.norm(nrm)
        u = np.cross(nrm, [1.0, 0, 0])
        u /= np.linalg.norm(u)
        v = np.cross(nrm, u)
        st = rng.uniform(-5, 5, (n, 2))
        off = rng.uniform(-50, 50, 3) if t % 3 else np.zeros(3)
        pts = (off + st[:, :1] * u + st[:, 1:] * v + rng.normal(0, 0.01, (n, 1)) * nrm)
        pts = np.ascontiguousarray(pts.astype(np.float32))
        sums = np.zeros(9, np.float32)
        cx, cy, cz = (np.ascontiguousarray(pts[:, k]) for k in range(3))
        fs.fs_literal(P(cx.ctypes.data), P(cy.ctypes.data), P(cz.ctypes.data), ctypes.c_int64(n),
                      P(sums.ctypes.data))
        cin = np.array([0.0, 0.0, 1.0, 0.0], np.float32)
        dev = np.zeros(4, np.float32)
        flag = ctypes.c_int(0)
        fs.fs_refit_host(P(sums.ctypes.data), ctypes.c_int64(n), P(cin.ctypes.data),
                         P(dev.ctypes.data), ctypes.byref(flag))
        host = np.zeros(4, np.float32)
        fs.fs_refit_pcl_host(P(pts.ctypes.data), ctypes.c_int64(n), P(cin.ctypes.data),
                             P(host.ctypes.data))
        unc += flag.value
        if not flag.value:
            assert same_bits(dev, host), (t, dev, host)
    assert unc <= 3
