"""ctypes wrapper for the C oracle (liborc.so) -- TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this module.
It is the checker, never the thing measured or shipped (see pcl_oracle.h for provenance and
pinning status: RNG pinned, PCL arithmetic "parity unpinned" -- restated from PCL 1.8).
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None


def build() -> str:
    path = os.path.join(_HERE, "liborc.so")
    src = os.path.join(_HERE, "pcl_oracle.c")
    if not os.path.exists(path) or os.path.getmtime(path) < os.path.getmtime(src):
        subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return path


SACMODEL_PLANE = 0
SACMODEL_NORMAL_PLANE = 11


class SacParams(C.Structure):
    _fields_ = [("threshold", C.c_double), ("max_iterations", C.c_int),
                ("probability", C.c_double), ("optimize", C.c_int),
                ("seed", C.c_uint32), ("refit_double", C.c_int), ("model", C.c_int),
                ("normal_distance_weight", C.c_double), ("normals", C.POINTER(C.c_float)),
                ("fast_qexp", C.c_int)]

QEXP_AUTO = -100000


class SacStats(C.Structure):
    _fields_ = [("iterations", C.c_int), ("skipped", C.c_int), ("draws", C.c_int64),
                ("best_sample", C.c_int32 * 3), ("coeff_unrefined", C.c_float * 4),
                ("n_unrefined", C.c_int64), ("has_model", C.c_int)]


class MT(C.Structure):
    _fields_ = [("mt", C.c_uint32 * 624), ("idx", C.c_int)]


def lib():
    global _LIB
    if _LIB is None:
        L = C.CDLL(build())
        fp = C.POINTER(C.c_float)
        i32p = C.POINTER(C.c_int32)
        i64p = C.POINTER(C.c_int64)
        L.orc_mt_seed.argtypes = [C.POINTER(MT), C.c_uint32]
        L.orc_mt_next.argtypes = [C.POINTER(MT)]
        L.orc_mt_next.restype = C.c_uint32
        L.orc_rnd.argtypes = [C.POINTER(MT)]
        L.orc_rnd.restype = C.c_int
        L.orc_plane_coefficients.argtypes = [fp, fp, fp, fp]
        L.orc_set_threads.argtypes = [C.c_int]
        L.orc_set_threads.restype = None
        L.orc_fast_qexp.argtypes = [fp, C.c_int64, i32p, C.c_int64]
        L.orc_fast_qexp.restype = C.c_int
        L.orc_refit_exact.argtypes = [fp, C.c_int64, i32p, C.c_int64, C.c_int, fp, fp]
        L.orc_refit_exact.restype = C.c_int
        L.orc_mom_digits.argtypes = [fp, C.c_int64, i32p, C.c_int64, C.c_int, i64p]
        L.orc_mom_digits.restype = None
        L.orc_refit_digits.argtypes = [i64p, C.c_int, fp, fp]
        L.orc_refit_digits.restype = C.c_int
        L.orc_plane_sample_good.argtypes = [fp, fp, fp]
        L.orc_thr_ceil.argtypes = [C.c_double]
        L.orc_thr_ceil.restype = C.c_float
        L.orc_sac_segment.argtypes = [fp, C.c_int64, C.c_int64, i32p, C.c_int64,
                                      C.POINTER(SacParams), fp, i32p, i64p, C.POINTER(SacStats)]
        L.orc_extract_planes.argtypes = [fp, C.c_int64, C.c_int64, C.POINTER(SacParams), C.c_int,
                                         C.c_int64, fp, i64p, i32p, C.POINTER(C.c_int)]
        L.orc_count_within.argtypes = [fp, C.c_int64, i32p, C.c_int64, fp, C.c_double]
        L.orc_count_within.restype = C.c_int64
        L.orc_mean_cov.argtypes = [fp, C.c_int64, i32p, C.c_int64, fp, fp]
        L.orc_eigen33.argtypes = [fp, fp, fp]
        L.orc_refit_double.argtypes = [fp, C.c_int64, i32p, C.c_int64, fp, fp]
        L.orc_count_within_np.argtypes = [fp, C.c_int64, fp, i32p, C.c_int64, fp, C.c_double,
                                          C.c_double]
        L.orc_count_within_np.restype = C.c_int64
        L.orc_normal_plane_dist.argtypes = [fp, fp, fp, C.c_double]
        L.orc_normal_plane_dist.restype = C.c_double
        L.orc_estimate_normals.argtypes = [fp, C.c_int64, C.c_int64, C.c_float, fp, fp]
        L.orc_estimate_normals_knn.argtypes = [fp, C.c_int64, C.c_int64, C.c_int, fp, fp]
        L.orc_estimate_normals_knn_brute.argtypes = [fp, C.c_int64, C.c_int64, C.c_int, fp, fp]
        L.orc_orient_normals_nn.argtypes = [fp, C.c_int64, C.c_int64, fp, fp, C.c_int64,
                                            C.c_int64, fp]
        L.orc_preprocess.argtypes = [fp, C.c_int64, C.c_int64, C.c_int, C.c_float, fp, i32p, fp]
        L.orc_preprocess.restype = C.c_int64
        L.orc_regulate_normals.argtypes = [fp, C.c_int64, C.c_int64, fp, C.c_int64, C.c_int,
                                           C.c_float, C.POINTER(C.c_uint8)]
        L.orc_regulate_normals.restype = C.c_int64
        u8p = C.POINTER(C.c_uint8)
        L.orc_msvc_rand.argtypes = [C.POINTER(C.c_uint32)]
        L.orc_msvc_rand.restype = C.c_uint32
        L.orc_is_point_in_poly.argtypes = [fp, fp, fp, C.c_int64, C.c_int64, C.c_float,
                                           C.c_uint32]
        L.orc_compute_point_normal.argtypes = [fp, C.c_int64, C.c_int64, fp, fp]
        L.orc_refit_planes.argtypes = [C.c_int, fp, fp, C.c_int64, i64p, fp]
        L.orc_cluster_filter.argtypes = [fp, C.c_int64, C.c_int64, C.c_float, C.c_int, u8p]
        L.orc_post_process_planes.argtypes = [
            fp, C.c_int64, C.c_int64, C.c_int, fp, fp, C.c_int64, i64p, fp, C.c_int64, i64p,
            C.c_float, C.c_int, C.c_uint32, C.c_float, C.c_int, fp, u8p, u8p]
        _LIB = L
    return _LIB


def _f(a):
    return a.ctypes.data_as(C.POINTER(C.c_float))


def _i32(a):
    return a.ctypes.data_as(C.POINTER(C.c_int32))


def _xyz(points):
    p = np.ascontiguousarray(points, dtype=np.float32)
    assert p.ndim == 2 and p.shape[1] in (3, 4)
    return p, p.shape[1]


def set_threads(n: int) -> None:
    """OpenMP threads of the oracle's countWithinDistance (1 = PCL's serial loop)."""
    lib().orc_set_threads(int(n))


def fast_qexp(points, indices=None) -> int:
    p, stride = _xyz(points)
    if indices is not None:
        idx = np.ascontiguousarray(indices, np.int32)
        return int(lib().orc_fast_qexp(_f(p), stride, _i32(idx), idx.shape[0]))
    return int(lib().orc_fast_qexp(_f(p), stride, None, p.shape[0]))


def refit_exact(points, indices, coeff_in, qexp):
    p, stride = _xyz(points)
    idx = np.ascontiguousarray(indices, np.int32)
    ci = np.ascontiguousarray(coeff_in, np.float32)
    co = np.zeros(4, np.float32)
    lib().orc_refit_exact(_f(p), stride, _i32(idx), idx.shape[0], int(qexp), _f(ci), _f(co))
    return co


def mom_digits(points, indices, qexp):
    """the fast refit's 25 int64 moment digits of points[indices] (sums over disjoint sets add)"""
    p, stride = _xyz(points)
    idx = np.ascontiguousarray(indices, np.int32)
    d = np.zeros(25, np.int64)
    lib().orc_mom_digits(_f(p), stride, _i32(idx), idx.shape[0], int(qexp),
                         d.ctypes.data_as(C.POINTER(C.c_int64)))
    return d


def refit_digits(digits, coeff_in, qexp):
    d = np.ascontiguousarray(digits, np.int64)
    ci = np.ascontiguousarray(coeff_in, np.float32)
    co = np.zeros(4, np.float32)
    lib().orc_refit_digits(d.ctypes.data_as(C.POINTER(C.c_int64)), int(qexp), _f(ci), _f(co))
    return co


def rnd_stream(n, seed=12345):
    g = MT()
    lib().orc_mt_seed(C.byref(g), seed)
    return np.array([lib().orc_rnd(C.byref(g)) for _ in range(n)], dtype=np.int64)


def mt_stream(n, seed=12345):
    g = MT()
    lib().orc_mt_seed(C.byref(g), seed)
    return np.array([lib().orc_mt_next(C.byref(g)) for _ in range(n)], dtype=np.uint64)


def params(threshold, max_iterations=50, probability=0.99, optimize=True, seed=12345,
           refit_double=False, normals=None, normal_distance_weight=0.1, refit="pcl",
           fast_qexp=None):
    """normals (float32 [N,4]: nx, ny, nz, curvature) selects SACMODEL_NORMAL_PLANE; the caller
    keeps the array alive for the call (params_keep).  refit: "pcl" (PCL float), "double" (the
    two-pass double LS reference; also refit_double=True) or "fast" (the product's
    DLG_REFIT_FAST, orc_refit_exact); fast_qexp overrides its quantum exponent."""
    mode = {"pcl": 0, "double": 1, "fast": 2}[refit]
    if refit_double:
        mode = 1
    prm = SacParams(float(threshold), int(max_iterations), float(probability),
                    int(bool(optimize)), int(seed), mode)
    prm.fast_qexp = QEXP_AUTO if fast_qexp is None else int(fast_qexp)
    if normals is not None:
        assert normals.dtype == np.float32 and normals.flags.c_contiguous and normals.shape[1] == 4
        prm.model = SACMODEL_NORMAL_PLANE
        prm.normal_distance_weight = float(normal_distance_weight)
        prm.normals = _f(normals)
    return prm


def _normals_arg(kw):
    if kw.get("normals") is not None:
        kw["normals"] = np.ascontiguousarray(kw["normals"], np.float32)
    return kw


def sac_segment(points, threshold, indices=None, **kw):
    """PCL SACSegmentation(PLANE, RANSAC).segment -> dict(coeff, inliers, stats...)."""
    p, stride = _xyz(points)
    n = p.shape[0]
    kw = _normals_arg(kw)
    prm = params(threshold, **kw)
    if indices is not None:
        idx = np.ascontiguousarray(indices, dtype=np.int32)
        nidx = idx.shape[0]
        idxp = _i32(idx)
    else:
        idx, nidx, idxp = None, n, None
    coeff = np.zeros(4, np.float32)
    inl = np.zeros(max(nidx, 1), np.int32)
    nin = C.c_int64(0)
    st = SacStats()
    ok = lib().orc_sac_segment(_f(p), n, stride, idxp, nidx, C.byref(prm), _f(coeff), _i32(inl),
                               C.byref(nin), C.byref(st))
    return dict(ok=bool(ok), coeff=coeff, inliers=inl[:nin.value].copy(),
                iterations=st.iterations, skipped=st.skipped, draws=st.draws,
                best_sample=np.array(st.best_sample[:], np.int32),
                coeff_unrefined=np.array(st.coeff_unrefined[:], np.float32),
                n_unrefined=st.n_unrefined)


def extract_planes(points, threshold, max_planes=20, min_inliers=0, **kw):
    p, stride = _xyz(points)
    n = p.shape[0]
    kw = _normals_arg(kw)
    prm = params(threshold, **kw)
    coeffs = np.zeros((max_planes, 4), np.float32)
    offs = np.zeros(max_planes + 1, np.int64)
    inl = np.zeros(max(n, 1), np.int32)
    npl = C.c_int(0)
    lib().orc_extract_planes(_f(p), n, stride, C.byref(prm), max_planes, int(min_inliers),
                             _f(coeffs), offs.ctypes.data_as(C.POINTER(C.c_int64)), _i32(inl),
                             C.byref(npl))
    k = npl.value
    return dict(coeffs=coeffs[:k].copy(), offsets=offs[:k + 1].copy(),
                inliers=inl[:offs[k]].copy(), n_planes=k)


def count_within_np(points, normals, coeff, threshold, lam=0.1):
    p, stride = _xyz(points)
    nrm = np.ascontiguousarray(normals, np.float32)
    c = np.ascontiguousarray(coeff, np.float32)
    return lib().orc_count_within_np(_f(p), stride, _f(nrm), None, p.shape[0], _f(c),
                                     float(threshold), float(lam))


def normal_plane_dist(coeff, point, normal, lam=0.1):
    c = np.ascontiguousarray(coeff, np.float32)
    p = np.ascontiguousarray(point, np.float32)
    n = np.ascontiguousarray(normal, np.float32)
    return lib().orc_normal_plane_dist(_f(c), _f(p), _f(n), float(lam))


def count_within(points, coeff, threshold, indices=None):
    p, stride = _xyz(points)
    c = np.ascontiguousarray(coeff, np.float32)
    if indices is None:
        return lib().orc_count_within(_f(p), stride, None, p.shape[0], _f(c), float(threshold))
    idx = np.ascontiguousarray(indices, np.int32)
    return lib().orc_count_within(_f(p), stride, _i32(idx), idx.shape[0], _f(c), float(threshold))


def plane_coefficients(p0, p1, p2):
    a = [np.ascontiguousarray(v, np.float32) for v in (p0, p1, p2)]
    c = np.zeros(4, np.float32)
    ok = lib().orc_plane_coefficients(_f(a[0]), _f(a[1]), _f(a[2]), _f(c))
    return bool(ok), c


def eigen33(cov):
    m = np.ascontiguousarray(cov, np.float32).reshape(9)
    ev = np.zeros(1, np.float32)
    v = np.zeros(3, np.float32)
    lib().orc_eigen33(_f(m), _f(ev), _f(v))
    return ev[0], v


def mean_cov(points, indices):
    p, stride = _xyz(points)
    idx = np.ascontiguousarray(indices, np.int32)
    cov = np.zeros(9, np.float32)
    cen = np.zeros(4, np.float32)
    lib().orc_mean_cov(_f(p), stride, _i32(idx), idx.shape[0], _f(cov), _f(cen))
    return cov, cen


def refit_double(points, indices, coeff_in):
    p, stride = _xyz(points)
    idx = np.ascontiguousarray(indices, np.int32)
    ci = np.ascontiguousarray(coeff_in, np.float32)
    co = np.zeros(4, np.float32)
    lib().orc_refit_double(_f(p), stride, _i32(idx), idx.shape[0], _f(ci), _f(co))
    return co


def thr_ceil(thr):
    return np.float32(lib().orc_thr_ceil(float(thr)))


def estimate_normals(points, radius, viewpoint=(0.0, 0.0, 0.0)):
    p, stride = _xyz(points)
    out = np.zeros((p.shape[0], 4), np.float32)
    vp = np.array(viewpoint, np.float32)
    lib().orc_estimate_normals(_f(p), p.shape[0], stride, float(radius), _f(vp), _f(out))
    return out


def estimate_normals_knn(points, k, viewpoint=(0.0, 0.0, 0.0), brute=False):
    """k-NN normals (grid search; brute=True: the O(n^2) definition it is checked against)."""
    p, stride = _xyz(points)
    out = np.zeros((p.shape[0], 4), np.float32)
    vp = np.array(viewpoint, np.float32)
    f = lib().orc_estimate_normals_knn_brute if brute else lib().orc_estimate_normals_knn
    f(_f(p), p.shape[0], stride, int(k), _f(vp), _f(out))
    return out


def regulate_normals(points, normals, seed_idx, seed_is_outward, radius):
    p, stride = _xyz(points)
    nrm = np.ascontiguousarray(normals, np.float32).copy()
    assert nrm.shape == (p.shape[0], 4)
    proc = np.zeros(p.shape[0], np.uint8)
    cnt = lib().orc_regulate_normals(_f(p), p.shape[0], stride, _f(nrm), int(seed_idx),
                                     int(bool(seed_is_outward)), float(radius),
                                     proc.ctypes.data_as(C.POINTER(C.c_uint8)))
    return nrm, proc.astype(bool), int(cnt)


def orient_normals_nn(points, normals, ref_points, ref_normals):
    p, stride = _xyz(points)
    r, rstride = _xyz(ref_points)
    nrm = np.ascontiguousarray(normals, np.float32).copy()
    rn = np.ascontiguousarray(ref_normals, np.float32)
    assert nrm.shape == (p.shape[0], 4) and rn.shape == (r.shape[0], 4)
    lib().orc_orient_normals_nn(_f(p), p.shape[0], stride, _f(nrm), _f(r), r.shape[0], rstride,
                                _f(rn))
    return nrm


def preprocess(points, min_dist, translate=True):
    p, stride = _xyz(points)
    n = p.shape[0]
    out = np.zeros((max(n, 1), 3), np.float32)
    idx = np.zeros(max(n, 1), np.int32)
    tr = np.zeros(3, np.float32)
    k = lib().orc_preprocess(_f(p), n, stride, int(bool(translate)), float(min_dist), _f(out),
                             _i32(idx), _f(tr))
    return out[:k].copy(), idx[:k].copy(), tr



# ---- postProcessPlanes (Dialog/PlaneDetect.h:1454-1579) ----
def _u8(a):
    return a.ctypes.data_as(C.POINTER(C.c_uint8))


def _i64(a):
    return a.ctypes.data_as(C.POINTER(C.c_int64))


def _concat(arrs):
    off = np.zeros(len(arrs) + 1, np.int64)
    for i, a in enumerate(arrs):
        off[i + 1] = off[i] + len(a)
    cat = (np.concatenate([np.asarray(a, np.float32).reshape(-1, 3) for a in arrs])
           if off[-1] else np.zeros((1, 3), np.float32))
    return np.ascontiguousarray(cat, np.float32), off


def msvc_rand(n, seed):
    st = C.c_uint32(seed)
    return [lib().orc_msvc_rand(C.byref(st)) for _ in range(n)]


def is_point_in_poly(p, coeff, border, t_dist, seed):
    q = np.ascontiguousarray(p, np.float32)
    c = np.ascontiguousarray(coeff, np.float32)
    b = np.ascontiguousarray(border, np.float32).reshape(-1, 3)
    return bool(lib().orc_is_point_in_poly(_f(q), _f(c), _f(b), b.shape[0], 3, float(t_dist),
                                           int(seed) & 0xffffffff))


def compute_point_normal(points):
    p, stride = _xyz(points)
    out = np.zeros(4, np.float32)
    curv = np.zeros(1, np.float32)
    lib().orc_compute_point_normal(_f(p), p.shape[0], stride, _f(out), _f(curv))
    return out, float(curv[0])


def refit_planes(coeffs, plane_points):
    pts, off = _concat(plane_points)
    c = np.ascontiguousarray(coeffs, np.float32).reshape(-1, 4)
    out = np.zeros_like(c)
    lib().orc_refit_planes(c.shape[0], _f(c), _f(pts), 3, _i64(off), _f(out))
    return out


def cluster_filter(points, radius, t_cluster_num):
    p, stride = _xyz(points)
    ok = np.zeros(max(p.shape[0], 1), np.uint8)
    lib().orc_cluster_filter(_f(p), p.shape[0], stride, float(radius), int(t_cluster_num), _u8(ok))
    return ok[:p.shape[0]].astype(bool)


def post_process_planes(cloud, coeffs, plane_points, borders, t_dist, plane_start, seed,
                        radius_local, t_cluster_num):
    """Returns (coeffs_out (P,4), absorbed: list of ascending cloud ids per plane,
    remaining: ascending cloud ids kept in source_cloud)."""
    p, stride = _xyz(cloud)
    n = p.shape[0]
    c = np.ascontiguousarray(coeffs, np.float32).reshape(-1, 4)
    P = c.shape[0]
    pts, poff = _concat(plane_points)
    bor, boff = _concat(borders)
    out = np.zeros_like(c)
    ab = np.zeros(max(P * n, 1), np.uint8)
    rem = np.zeros(max(n, 1), np.uint8)
    lib().orc_post_process_planes(_f(p), n, stride, P, _f(c), _f(pts), 3, _i64(poff), _f(bor), 3,
                                  _i64(boff), float(t_dist), int(plane_start),
                                  int(seed) & 0xffffffff, float(radius_local),
                                  int(t_cluster_num), _f(out), _u8(ab), _u8(rem))
    ab = ab[:P * n].reshape(P, n) if n else np.zeros((P, 0), np.uint8)
    absorbed = [np.nonzero(ab[k])[0].astype(np.int32) for k in range(P)]
    return out, absorbed, np.nonzero(rem[:n])[0].astype(np.int32)
