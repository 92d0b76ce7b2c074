"""preProcess() / removeRedundantPoints on the GPU (Dialog/PlaneDetect.h:448-512,
PCLViewer.cpp:781-805): NaN removal, translation to the centroid, redundancy removal with the
radius min_dist_between_points.  Runs in libdialog_amd.so (dlg_preprocess); no CPU path."""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _lib
from .sac import Context, _f32p, _i32p, _points, default_context


def preprocess(points, min_dist: float, translate: bool = True, ctx: Context | None = None):
    """-> (kept float32 [k,3] (translated when `translate`), input indices int32 [k],
    translation float32 [3])."""
    ctx = ctx or default_context()
    a, pts = _points(points)
    n = a.shape[0]
    out = np.empty((max(n, 1), 3), np.float32)
    idx = np.empty(max(n, 1), np.int32)
    tr = np.zeros(3, np.float32)
    k = C.c_int64(0)
    ctx.check(_lib.load().dlg_preprocess(ctx.h, C.byref(pts), int(bool(translate)),
                                         float(min_dist), _f32p(out), 12, _i32p(idx), n,
                                         C.byref(k), _f32p(tr)))
    return out[:k.value].copy(), idx[:k.value].copy(), tr


def remove_redundant_points(points, min_dist: float, ctx: Context | None = None):
    """on_removeRedundantPointsAction_triggered (PCLViewer.cpp:781-805): -> kept indices."""
    _, idx, _ = preprocess(points, min_dist, translate=False, ctx=ctx)
    return idx
