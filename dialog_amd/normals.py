"""Normal estimation and RegulateNormal on the GPU (Dialog/PlaneDetect.h:515-665).

Python mirror of the reference's normals stage: `estimate_normals` is estimateNormal()
(pcl::NormalEstimationOMP, radius r_for_estimate_normal, PlaneDetect.h:515-545) or the k = 20
NormalEstimation of PCLViewer.cpp:507-522; `regulate_normals` is the first-round branch of
regulateNormal() (PlaneDetect.h:586-646).  `NormalEstimation` keeps PCL's setter names.
Everything runs in libdialog_amd.so (dlg_estimate_normals / dlg_regulate_normals); there is no
CPU path.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _lib
from .sac import Context, _f32p, _points, default_context


NORMALS_PCL_FLOAT = 0
NORMALS_CENTRED_DOUBLE = 1


def estimate_normals(points, radius: float = 0.0, k: int = 0, viewpoint=(0.0, 0.0, 0.0),
                     ctx: Context | None = None, layout: str = "float4",
                     mode: str = "pcl") -> np.ndarray:
    """points float32 [N,3|4] -> float32 [N,4] (nx, ny, nz, curvature) for layout "float4", or
    [N,8] pcl::Normal records (normal_x/y/z, pad, curvature, pad x3) for layout "pcl".
    mode "pcl": PCL's float arithmetic (bit-exact with the oracle); "double": centred double
    moments (dlg_estimate_normals_ex)."""
    ctx = ctx or default_context()
    a, pts = _points(points)
    width = {"float4": 4, "pcl": 8}[layout]
    m = {"pcl": NORMALS_PCL_FLOAT, "double": NORMALS_CENTRED_DOUBLE}[mode]
    out = np.empty((a.shape[0], width), np.float32)
    vp = np.ascontiguousarray(viewpoint, np.float32)
    ctx.check(_lib.load().dlg_estimate_normals_ex(ctx.h, C.byref(pts), float(radius), int(k),
                                                  _f32p(vp), _f32p(out), 4 * width, m))
    return out


def regulate_normals(points, normals, seed_idx: int, seed_is_outward: bool, radius: float,
                     ctx: Context | None = None):
    """-> (normals copy with regulated signs, processed bool[N], number processed).  normals:
    float32 [N, >=3] records (only columns 0..2 change)."""
    ctx = ctx or default_context()
    a, pts = _points(points)
    nrm = np.array(normals, dtype=np.float32, order="C", copy=True)
    if nrm.ndim != 2 or nrm.shape[0] != a.shape[0] or nrm.shape[1] < 3:
        raise ValueError("normals must be float32 [N, >=3] matching points")
    proc = np.zeros(a.shape[0], np.uint8)
    cnt = C.c_int64(0)
    ctx.check(_lib.load().dlg_regulate_normals(
        ctx.h, C.byref(pts), _f32p(nrm), 4 * nrm.shape[1], int(seed_idx),
        int(bool(seed_is_outward)), float(radius), proc.ctypes.data_as(C.POINTER(C.c_uint8)),
        C.byref(cnt)))
    return nrm, proc.astype(bool), int(cnt.value)


def orient_normals_nn(points, normals, ref_points, ref_normals, ctx: Context | None = None):
    """regulateNormal() later-round branch (PlaneDetect.h:553-584): flip each normal to agree
    with its nearest backup point's normal.  Returns a copy (columns 0..2 change)."""
    ctx = ctx or default_context()
    a, pts = _points(points)
    r, rpts = _points(ref_points)
    nrm = np.array(normals, dtype=np.float32, order="C", copy=True)
    rn = np.ascontiguousarray(ref_normals, dtype=np.float32)
    if nrm.ndim != 2 or nrm.shape[0] != a.shape[0] or nrm.shape[1] < 3:
        raise ValueError("normals must be float32 [N, >=3] matching points")
    if rn.ndim != 2 or rn.shape[0] != r.shape[0] or rn.shape[1] < 3:
        raise ValueError("ref_normals must be float32 [M, >=3] matching ref_points")
    ctx.check(_lib.load().dlg_orient_normals_nn(ctx.h, C.byref(pts), _f32p(nrm), 4 * nrm.shape[1],
                                                C.byref(rpts), _f32p(rn), 4 * rn.shape[1]))
    return nrm


class NormalEstimation:
    """pcl::NormalEstimation(OMP)<PointXYZ, Normal> on the GPU."""

    def __init__(self, ctx: Context | None = None):
        self.ctx = ctx
        self.input = None
        self.radius = 0.0
        self.k = 0
        self.viewpoint = (0.0, 0.0, 0.0)

    def setInputCloud(self, xyz):
        self.input = np.ascontiguousarray(xyz, dtype=np.float32)

    def setRadiusSearch(self, r):
        self.radius, self.k = float(r), 0

    def setKSearch(self, k):
        self.k, self.radius = int(k), 0.0

    def setViewPoint(self, vx, vy, vz):
        self.viewpoint = (float(vx), float(vy), float(vz))

    def compute(self, layout="float4"):
        if self.input is None:
            raise ValueError("setInputCloud() first")
        return estimate_normals(self.input, self.radius, self.k, self.viewpoint, self.ctx, layout)

    set_input_cloud = setInputCloud
    set_radius_search = setRadiusSearch
    set_k_search = setKSearch
    set_view_point = setViewPoint
