"""postProcessPlanes on the GPU (Dialog/PlaneDetect.h:1454-1579): plane refit, absorption of
leftover points by the planes' border polygons (isPointInPoly), clusterFilt of the rest.
Runs in libdialog_amd.so (dlg_post_process_planes / dlg_refit_planes / dlg_cluster_filter);
no CPU path.

A plane is a mapping (or object) with `coeff` (coeff.values: 3 or 4 floats, [0..2] = outward
normal), `points` (its points_set, [m, 3] float32) and `border` (its polygon, [b, 3] float32),
i.e. the reference's struct Plane (HeaderFile.h:81-88) minus the display fields.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass

import numpy as np

from . import _lib
from .sac import Context, _f32p, _i32p, _points, default_context


@dataclass
class PostProcessParams:
    """config.ini [PlaneDetect] defaults (T_dist_point_plane, radius_local, T_cluster_num)."""
    t_dist_point_plane: float = 0.1
    radius_local: float = 0.1
    t_cluster_num: int = 500
    plane_start_index: int = 0
    rand_seed: int = 0  # the srand(time(0)) value of isPointInPoly


def _get(plane, key):
    return plane[key] if isinstance(plane, dict) else getattr(plane, key)


def _xyz(a):
    a = np.asarray(a, np.float32)
    if a.size == 0:
        return np.zeros((0, 3), np.float32)
    if a.ndim == 1:
        a = a.reshape(-1, 3)
    return np.ascontiguousarray(a[:, :3])


class _PlaneArrays:
    """Keeps the concatenated host arrays alive while the C call reads them."""

    def __init__(self, planes):
        P = len(planes)
        self.coeffs = np.zeros((max(P, 1), 4), np.float32)
        pts, bor = [], []
        self.poff = np.zeros(P + 1, np.int64)
        self.boff = np.zeros(P + 1, np.int64)
        for k, pl in enumerate(planes):
            c = np.asarray(_get(pl, "coeff"), np.float32).ravel()
            self.coeffs[k, :min(4, c.size)] = c[:4]
            p = _xyz(_get(pl, "points"))
            b = _xyz(_get(pl, "border"))
            pts.append(p)
            bor.append(b)
            self.poff[k + 1] = self.poff[k] + p.shape[0]
            self.boff[k + 1] = self.boff[k] + b.shape[0]
        self.points = np.ascontiguousarray(np.concatenate(pts) if self.poff[-1] else
                                           np.zeros((1, 3), np.float32))
        self.borders = np.ascontiguousarray(np.concatenate(bor) if self.boff[-1] else
                                            np.zeros((1, 3), np.float32))
        self.s = _lib.Planes(P, _f32p(self.coeffs), _f32p(self.points), 12,
                             self.poff.ctypes.data_as(C.POINTER(C.c_int64)), _f32p(self.borders),
                             12, self.boff.ctypes.data_as(C.POINTER(C.c_int64)))


def plane_border(points, normal, alpha: float = 0.5) -> np.ndarray:
    """polyPointCloud (PlaneDetect.h:1376-1440) for one plane: its points projected on their
    least-squares plane, then a closed concave border of projected points oriented by `normal`
    (dlg_plane_border; the reference's qhull ConcaveHull is absent: parity unpinned) -> float32
    [B, 3] (B = 0: fewer than 3 points).  alpha: alpha_poly (config.txt: 0.5)."""
    a = np.ascontiguousarray(_xyz(points), np.float32)
    pts = _lib.Points(_f32p(a), a.shape[0], 12)
    pn = np.ascontiguousarray(normal, np.float32)[:3]
    L = _lib.load()
    n = C.c_int64()
    cap = max(a.shape[0], 16)
    out = np.zeros((cap, 3), np.float32)
    _lib.check(L.dlg_plane_border(C.byref(pts), _f32p(pn), float(alpha), _f32p(out), 12, cap,
                                  C.byref(n)))
    return out[:n.value].copy()


def refit_planes(planes):
    """PlaneDetect.h:1477-1498: computePointNormal of each plane's points, oriented like its
    previous normal -> float32 [P, 4]."""
    A = _PlaneArrays(planes)
    out = np.zeros((max(len(planes), 1), 4), np.float32)
    st = _lib.load().dlg_refit_planes(C.byref(A.s), _f32p(out))
    _lib.check(st)
    return out[:len(planes)].copy()


def post_process_planes(cloud, planes, params: PostProcessParams | None = None,
                        ctx: Context | None = None):
    """-> (coeffs float32 [P, 4], absorbed: list of ascending int32 cloud ids per plane,
    remaining: ascending int32 cloud ids of the new source_cloud)."""
    ctx = ctx or default_context()
    prm = params or PostProcessParams()
    a, pts = _points(cloud)
    n = a.shape[0]
    P = len(planes)
    A = _PlaneArrays(planes)
    cp = _lib.PostProcessParams(float(prm.t_dist_point_plane), float(prm.radius_local),
                                int(prm.t_cluster_num), int(prm.plane_start_index),
                                int(prm.rand_seed) & 0xffffffff)
    coeffs = np.zeros((max(P, 1), 4), np.float32)
    off = np.zeros(P + 1, np.int64)
    cap = max(n, 1)
    ids = np.empty(cap, np.int32)
    rem = np.empty(max(n, 1), np.int32)
    nrem = C.c_int64(0)
    L = _lib.load()
    i64p = C.POINTER(C.c_int64)
    while True:
        st = L.dlg_post_process_planes(ctx.h, C.byref(pts), C.byref(A.s), C.byref(cp),
                                       _f32p(coeffs), off.ctypes.data_as(i64p), _i32p(ids), cap,
                                       _i32p(rem), rem.size, C.byref(nrem))
        if st == _lib.DLG_ERR_CAPACITY and off[-1] > cap:
            cap = int(off[-1])
            ids = np.empty(cap, np.int32)
            continue
        ctx.check(st)
        break
    absorbed = [ids[off[k]:off[k + 1]].copy() for k in range(P)]
    return coeffs[:P].copy(), absorbed, rem[:nrem.value].copy()


def cluster_filter(points, radius: float, t_cluster_num: int, ctx: Context | None = None):
    """clusterFilt (PlaneDetect.h:1582-1655) -> ascending indices of the points kept."""
    ctx = ctx or default_context()
    a, pts = _points(points)
    n = a.shape[0]
    out = np.empty(max(n, 1), np.int32)
    k = C.c_int64(0)
    ctx.check(_lib.load().dlg_cluster_filter(ctx.h, C.byref(pts), float(radius),
                                             int(t_cluster_num), _i32p(out), n, C.byref(k)))
    return out[:k.value].copy()
