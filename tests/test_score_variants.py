"""Scoring-kernel variants must give bit-identical counts (countWithinDistance semantics).

The bf16 matrix-core variant decides most (point, plane) pairs from D = a x + b y + c z + d
computed with exactly split bf16 operands and re-decides, in PCL's op order, every pair whose
|D| lies within the rounding band of the threshold.  These cases load the band on purpose:
noise comparable to the threshold (many points near it), a cloud far from the origin (a wide
band: e grows with |coordinates|), NaN and infinite coordinates, point counts that leave partial
tiles, and hypothesis counts that leave partial plane groups.
"""
import ctypes as C

import numpy as np
import pytest

VARIANTS = (0, 1, 2)  # DLG_SCORE_EXACT (PCL op order), DLG_SCORE_BF16 (matrix cores), DLG_SCORE_PRUNED
# DLG_OPT_PRUNE_TILE_SCORER values besides the default DLG_TILE_EXACT: DLG_TILE_BF16 and the
# A/B-only variants 11, 14 (1 / 4 planes per lane), 12 (packed f32 tests) and the claim variants
# 15 (round 4's round-robin), 16 (list-length classes, no tail), 17 (tail, no classes), and
# DLG_TILE_MFMA (2: f32 matrix-core groups of 16 planes + band re-decision; 18: the same with
# every result re-decided, 19: a 64 u S band -- A/B checks of the band); the "wide" case's
# threshold puts most planes on every super-tile's list (lists past the 1024-entry register chunk)
TILE_SCORERS = (2, 18, 19, 1, 11, 12, 14, 15, 16, 17)


def counts(ctx, cloud, D, v, thr):
    import dialog_amd as DD
    from dialog_amd import _lib
    ms = C.c_double()
    out = np.zeros(D, np.int32)
    ctx.check(_lib.load().dlg_score_benchmark(ctx.h, cloud.h, D, v, 1, thr, C.byref(ms),
                                              out.ctypes.data_as(C.POINTER(C.c_int32))))
    return out


def make(case):
    from dialog_amd.synth import plane_cloud
    if case == "noisy":
        p, _, _ = plane_cloud(200_003, 5, sigma=0.015, seed=11)
        return p, 0.02
    if case == "far":
        p, _, _ = plane_cloud(150_001, 4, sigma=0.01, seed=12)
        return (p + np.float32(1000.0)).astype(np.float32), 0.02
    if case == "nonfinite":
        p, _, _ = plane_cloud(100_037, 4, sigma=0.01, seed=13)
        p[::97, 1] = np.nan
        p[5::1013, 2] = np.inf
        return p, 0.02
    if case == "wide":
        p, _, _ = plane_cloud(300_007, 6, sigma=0.01, seed=15)
        return p, 0.3
    if case == "tiny":
        p, _, _ = plane_cloud(1_000, 3, sigma=0.01, seed=14)
        return (p * np.float32(1e-3)).astype(np.float32), 2e-5
    raise ValueError(case)


@pytest.mark.gpu
@pytest.mark.parametrize("case", ["noisy", "far", "nonfinite", "wide", "tiny"])
def test_score_variants_bit_identical(gpu_ctx, case):
    import dialog_amd as D
    p, thr = make(case)
    cloud = D.Cloud(gpu_ctx, p)
    cloud.build_spatial()
    bad = []
    try:
        for nh in (1, 100, 257, 4096):
            ref = counts(gpu_ctx, cloud, nh, VARIANTS[0], thr)
            assert ref.sum() > 0
            for v in VARIANTS[1:]:
                got = counts(gpu_ctx, cloud, nh, v, thr)
                assert np.array_equal(got, ref), (case, nh, v, int((got != ref).sum()))
            # the pruned path's other tile scorers: bf16 blocks + band re-decision, the exact
            # scorer's 1- and 4-plane-per-lane A/B variants
            for ts in TILE_SCORERS:
                gpu_ctx.set_option(D.DLG_OPT_PRUNE_TILE_SCORER, ts)
                try:
                    assert gpu_ctx.get_option(D.DLG_OPT_PRUNE_TILE_SCORER) == ts
                    got = counts(gpu_ctx, cloud, nh, 2, thr)
                finally:
                    gpu_ctx.set_option(D.DLG_OPT_PRUNE_TILE_SCORER, D.DLG_TILE_EXACT)
                if not np.array_equal(got, ref):
                    bad.append((case, nh, ts, int((got != ref).sum()),
                                [(int(i), int(got[i]), int(ref[i])) for i in np.flatnonzero(got != ref)[:4]]))
        assert not bad, bad
    finally:
        cloud.close()
