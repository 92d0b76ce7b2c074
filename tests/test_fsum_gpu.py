"""GPU: DLG_REFIT_PCL's device sums (fsum.hip) on caller data against the literal loop, bit for bit.

dlg_float_sums runs the product kernels (k_fs_prep, k_fs_inc, k_fs_l1, k_fs_walk) on the given
points; the reference is PCL's single-pass float loop of computeMeanAndCovarianceMatrix's dense
branch (tests/cpp/fsum_host.cpp fs_literal, accu[k] += term in list order) and the host refit
refit_pcl_float (the oracle's arithmetic).  Inputs: the adversarial kinds of tests/test_fsum.py
(sums hovering around zero, quantised values, mixed magnitudes 1e-20..1e20, subnormals, zeros,
overflowing squares, constant and alternating sequences, far offsets) at sizes straddling the
chunk (64), unit (4096) and 64-unit scan boundaries, and the real input: the inliers of C3-like
planes (several hundred thousand points, some with sums that hover near zero).
"""
import ctypes
import os
import subprocess

import numpy as np
import pytest

import dialog_amd as D
from dialog_amd.synth import plane_cloud

from test_fsum import KINDS, gen

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
P = ctypes.c_void_p


@pytest.fixture(scope="module")
def fs(tmp_path_factory):
    so = tmp_path_factory.mktemp("fsum") / "libfsum_host.so"
    subprocess.run(["g++", "-std=c++17", "-O2", "-ffp-contract=off", "-shared", "-fPIC",
                    os.path.join(ROOT, "tests", "cpp", "fsum_host.cpp"), "-o", str(so)], check=True)
    return ctypes.CDLL(str(so))


def literal(fs, xyz):
    x, y, z = (np.ascontiguousarray(xyz[:, k], np.float32) for k in range(3))
    ref = np.zeros(9, np.float32)
    fs.fs_literal(P(x.ctypes.data), P(y.ctypes.data), P(z.ctypes.data), ctypes.c_int64(x.size),
                  P(ref.ctypes.data))
    return ref


def host_refit(fs, xyz, cin):
    a = np.ascontiguousarray(xyz, np.float32)
    c = np.ascontiguousarray(cin, np.float32)
    out = np.zeros(4, np.float32)
    fs.fs_refit_pcl_host(P(a.ctypes.data), ctypes.c_int64(a.shape[0]), P(c.ctypes.data),
                         P(out.ctypes.data))
    return out


def same(a, b):
    a, b = np.asarray(a, np.float32), np.asarray(b, np.float32)
    nan = np.isnan(b)
    return np.array_equal(np.isnan(a), nan) and np.array_equal(a[~nan].view(np.uint32),
                                                               b[~nan].view(np.uint32))


@pytest.mark.parametrize("kind", KINDS)
def test_device_sums_equal_literal_loop(gpu_ctx, fs, kind):
    rng = np.random.default_rng(KINDS.index(kind) + 101)
    for n in (1, 2, 63, 64, 65, 4095, 4096, 4097, 70000, 270000):
        xyz = np.ascontiguousarray(np.stack(gen(kind, n, rng), axis=1))
        sums, _, _, _ = gpu_ctx.float_sums(xyz)
        assert same(sums, literal(fs, xyz)), (kind, n, sums, literal(fs, xyz))


def test_device_sums_empty(gpu_ctx):
    sums, co, unc, _ = gpu_ctx.float_sums(np.zeros((0, 3), np.float32), cin=(1, 2, 3, 4))
    assert not sums.any() and not unc
    assert np.array_equal(co, np.float32([1, 2, 3, 4]))  # (< 4 inliers: coefficients kept)


def test_device_refit_on_plane_inliers(gpu_ctx, fs):
    """C3's real input (10M points, 20 planes: each plane's ~450k inliers in list order, among
    them sums that hover near zero) and a 4M-point list (more than 64 units: the scans' windows);
    sums and refined plane equal the literal loop and the host refit."""
    p, lab, planes = plane_cloud(10_000_000, 20, seed=0xD1A106 + 3)
    ms = []
    for k in range(8):
        xyz = np.ascontiguousarray(p[lab == k])
        cin = np.float32([planes[k, 0], planes[k, 1], planes[k, 2], planes[k, 3]])
        sums, co, unc, t = gpu_ctx.float_sums(xyz, cin=cin, reps=3)
        assert same(sums, literal(fs, xyz)), k
        if not unc:
            assert same(co, host_refit(fs, xyz, cin)), k
        ms.append(t)
    xyz = np.ascontiguousarray(p[:4_000_000])
    sums, _, _, t4 = gpu_ctx.float_sums(xyz, reps=2)
    assert same(sums, literal(fs, xyz))
    print(f"\nfloat sums + refit: {np.round(ms, 4).tolist()} ms per ~450k-point plane; "
          f"{t4:.4f} ms at 4M points")


def test_device_sums_poisoned_tables(fs):
    """Window tables are valid only with the current launch's stamp; reused scratch could hold
    words carrying that stamp (another layout's records, recycled device memory).  With
    DLG_OPT_FS_POISON every table entry is filled with a garbage value stamped for the next launch
    before fs_reset clears the tables: the sums must still equal the literal loop.  Hovering sums
    (planes through the origin) make the walk consult the tables."""
    ctx = D.Context(0)
    try:
        ctx.set_option(D.DLG_OPT_FS_POISON, 1)
        assert ctx.get_option(D.DLG_OPT_FS_POISON) == 1
        rng = np.random.default_rng(77)
        for kind in ("hover", "quant", "alternating"):
            for n in (4097, 270000, 900000):
                xyz = np.ascontiguousarray(np.stack(gen(kind, n, rng), axis=1))
                sums, _, _, _ = ctx.float_sums(xyz)
                assert same(sums, literal(fs, xyz)), (kind, n)
        p, lab, planes = plane_cloud(3_000_000, 6, seed=0xD1A106 + 3)
        for k in range(6):
            xyz = np.ascontiguousarray(p[lab == k])
            sums, _, _, _ = ctx.float_sums(xyz)
            assert same(sums, literal(fs, xyz)), k
    finally:
        ctx.close()


@pytest.mark.parametrize("segments,join", [(1, 1), (2, 1), (4, 1), (5, 1), (8, 1), (16, 1),
                                           (4, 0), (8, 0)])
def test_device_sums_segments(fs, segments, join):
    """DLG_OPT_FS_SEGMENTS (one rank): each chain's windows in that many segments, walked at once
    from the refined guesses and joined in order (a segment whose guess missed its exact start is
    walked again until it meets its recorded walk) -- by each chain's last segment walker in the
    walk's launch (DLG_OPT_FS_JOIN 1, the default) or by k_fs_segfix (0).  Every segmentation
    gives the literal loop's sums: hovering and quantised sequences (the guesses miss) and C3's
    planes."""
    ctx = D.Context(0)
    try:
        assert ctx.get_option(D.DLG_OPT_FS_JOIN) == 1
        ctx.set_option(D.DLG_OPT_FS_SEGMENTS, segments)
        ctx.set_option(D.DLG_OPT_FS_JOIN, join)
        assert ctx.get_option(D.DLG_OPT_FS_SEGMENTS) == segments
        rng = np.random.default_rng(500 + segments + 100 * join)
        for kind in ("hover", "quant", "alternating", "mags", "drift"):
            for n in (4097, 70000, 600000):
                xyz = np.ascontiguousarray(np.stack(gen(kind, n, rng), axis=1))
                sums, _, _, _ = ctx.float_sums(xyz)
                assert same(sums, literal(fs, xyz)), (kind, n)
        p, lab, planes = plane_cloud(4_000_000, 8, seed=0xD1A106 + 3)
        for k in range(8):
            xyz = np.ascontiguousarray(p[lab == k])
            cin = np.float32([planes[k, 0], planes[k, 1], planes[k, 2], planes[k, 3]])
            sums, co, unc, _ = ctx.float_sums(xyz, cin=cin)
            assert same(sums, literal(fs, xyz)), k
            if not unc:
                assert same(co, host_refit(fs, xyz, cin)), k
    finally:
        ctx.close()
