"""Host-side mirror of PCL's SACSegmentation interface over the MI355X C ABI.

`SACSegmentation` keeps the PCL 1.8 names, argument meanings and failure behaviour of
pcl::SACSegmentation<pcl::PointXYZ> as the reference calls it (Dialog/SimplifyVerticesSize.cpp:
62-67, 86-87): setModelType / setMethodType / setDistanceThreshold / setMaxIterations /
setProbability / setOptimizeCoefficients / setInputCloud / setIndices / segment().  segment()
returns (inliers, coefficients); "no model" is an empty inlier list and empty coefficients, as in
PCL.  `extract_planes` is the sequential extract-and-remove loop that fills the reference's
plane_clouds slot (Dialog/PlaneDetect.h:100, :667-1355).
"""
from __future__ import annotations

import atexit
import ctypes as C
import threading
import weakref

import numpy as np

from . import _lib
from ._lib import DLG_REFIT_FAST, DLG_REFIT_PCL, DLG_SACMODEL_PLANE, DialogError  # noqa: F401

SACMODEL_PLANE = 0
SACMODEL_NORMAL_PLANE = 11
SAC_RANSAC = 0


# Live device objects, closed at interpreter exit before the HIP runtime's own static destructors
# run (a hipFree after runtime teardown crashes).  Clouds first, then contexts.
_LIVE_CLOUDS: "weakref.WeakSet" = weakref.WeakSet()
_LIVE_CTXS: "weakref.WeakSet" = weakref.WeakSet()


@atexit.register
def _close_all():
    for obj in list(_LIVE_CLOUDS):
        try:
            obj.close()
        except Exception:
            pass
    for obj in list(_LIVE_CTXS):
        try:
            obj.close()
        except Exception:
            pass


def _f32p(a):
    return a.ctypes.data_as(C.POINTER(C.c_float))


def _i32p(a):
    return a.ctypes.data_as(C.POINTER(C.c_int32))


def _points(xyz):
    """float32 [N,3] or [N,4] (pcl::PointXYZ layout) -> (keepalive array, Points struct)."""
    a = np.ascontiguousarray(xyz, dtype=np.float32)
    if a.ndim != 2 or a.shape[1] not in (3, 4):
        raise ValueError("points must be float32 [N,3] or [N,4]")
    return a, _lib.Points(_f32p(a), a.shape[0], 4 * a.shape[1])


class Context:
    """One HIP device (+ optional rank communicator).  Not thread-safe: one per host thread."""

    def __init__(self, device: int = 0, _handle=None):
        self._L = _lib.load()
        if _handle is not None:
            self.h = _handle
        else:
            h = C.c_void_p()
            _lib.check(self._L.dlg_ctx_create(C.byref(h), int(device)), None)
            self.h = h
        r, w, d = C.c_int(), C.c_int(), C.c_int()
        _lib.check(self._L.dlg_ctx_info(self.h, C.byref(r), C.byref(w), C.byref(d)), self.h)
        self.rank, self.world, self.device = r.value, w.value, d.value
        _LIVE_CTXS.add(self)

    @classmethod
    def distributed(cls, device, rank, world, unique_id: bytes):
        L = _lib.load()
        h = C.c_void_p()
        buf = C.create_string_buffer(bytes(unique_id), 128)
        _lib.check(L.dlg_ctx_create_dist(C.byref(h), int(device), int(rank), int(world), buf), None)
        return cls(_handle=h)

    @staticmethod
    def unique_id() -> bytes:
        L = _lib.load()
        buf = C.create_string_buffer(128)
        _lib.check(L.dlg_get_unique_id(buf), None)
        return buf.raw

    @classmethod
    def loopback_group(cls, world: int, device: int = 0):
        L = _lib.load()
        arr = (C.c_void_p * world)()
        _lib.check(L.dlg_ctx_create_loopback_group(arr, int(world), int(device)), None)
        return [cls(_handle=C.c_void_p(arr[r])) for r in range(world)]

    def close(self):
        if getattr(self, "h", None) is not None and self.h.value:
            self._L.dlg_ctx_destroy(self.h)
            self.h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def check(self, status):
        _lib.check(status, self.h)

    def set_option(self, option: int, value: int):
        """dlg_ctx_set_option: choose among equivalent device paths (identical results)."""
        self.check(self._L.dlg_ctx_set_option(self.h, int(option), int(value)))

    def get_option(self, option: int) -> int:
        v = C.c_int64()
        self.check(self._L.dlg_ctx_get_option(self.h, int(option), C.byref(v)))
        return v.value

    def prune_stats(self, reset: bool = False) -> dict:
        """The pruned scoring kernel's work counters (needs DLG_OPT_PRUNE_STATS = 1)."""
        a = (C.c_uint64 * 8)()
        self.check(self._L.dlg_prune_stats(self.h, a, int(bool(reset))))
        return {"workgroups": a[0], "list_entries": a[1], "tiles": a[2], "blocks": a[3], "pairs": a[4],
                "redecided_blocks": a[5], "wg_ticks_sum": a[6], "wg_ticks_max": a[7]}

    def set_profiling(self, on=True):
        """on: True / 1 = all timing events, 2 = without the PCL refit walk's, False / 0 = none."""
        self.check(self._L.dlg_set_profiling(self.h, int(on)))

    def synchronize(self):
        self.check(self._L.dlg_synchronize(self.h))

    def barrier(self):
        self.check(self._L.dlg_barrier(self.h))

    def float_sums(self, xyz, cin=(0.0, 0.0, 1.0, 0.0), reps=1, walk_stats=False):
        """dlg_float_sums: DLG_REFIT_PCL's device sums (fsum.hip) over xyz (n x 3 float32, list
        order) and the float refit of cin -> (sums[9], coeff[4], uncertain, ms_per_call), plus
        the walk's per-chain counters [9, 8] when walk_stats."""
        a = np.ascontiguousarray(xyz, np.float32).reshape(-1, 3)
        ci = np.ascontiguousarray(cin, np.float32)
        sums = np.zeros(9, np.float32)
        co = np.zeros(4, np.float32)
        unc, ms = C.c_int(), C.c_double()
        ws = np.zeros((9, 8), np.int64) if walk_stats else None
        self.check(self._L.dlg_float_sums(self.h, _f32p(a), C.c_int64(a.shape[0]), _f32p(ci),
                                          int(reps), _f32p(sums), _f32p(co), C.byref(unc),
                                          C.byref(ms),
                                          ws.ctypes.data_as(C.POINTER(C.c_int64)) if walk_stats
                                          else None))
        if walk_stats:
            return sums, co, bool(unc.value), ms.value, ws
        return sums, co, bool(unc.value), ms.value

    def allreduce_max(self, v: float) -> float:
        x = C.c_double(float(v))
        self.check(self._L.dlg_allreduce_max_f64(self.h, C.byref(x)))
        return x.value


class Cloud:
    """Device-resident active point list (this rank's shard)."""

    def __init__(self, ctx: Context, xyz, indices=None, id_base: int = 0):
        self.ctx = ctx
        arr, pts = _points(xyz)
        h = C.c_void_p()
        if indices is not None:
            idx = np.ascontiguousarray(indices, dtype=np.int32)
            ctx.check(ctx._L.dlg_cloud_upload(ctx.h, C.byref(pts), _i32p(idx), idx.shape[0],
                                              int(id_base), C.byref(h)))
            self.n = idx.shape[0]
        else:
            ctx.check(ctx._L.dlg_cloud_upload(ctx.h, C.byref(pts), None, 0, int(id_base),
                                              C.byref(h)))
            self.n = arr.shape[0]
        self.h = h
        _LIVE_CLOUDS.add(self)

    def build_spatial(self):
        """Morton-ordered copy for the pruned scoring kernel (automatic for >= 131072 points)."""
        self.ctx.check(self.ctx._L.dlg_cloud_build_spatial(self.ctx.h, self.h))

    def drop_spatial(self):
        """release the Morton copy (resets the cloud); build_spatial() builds it again."""
        self.ctx.check(self.ctx._L.dlg_cloud_drop_spatial(self.h))

    def reset(self):
        self.ctx.check(self.ctx._L.dlg_cloud_reset(self.h))

    def set_normals(self, normals):
        """setInputNormals: float32 [N,4] (nx, ny, nz, curvature) or [N,8] pcl::Normal records,
        one per uploaded point.  Resets the cloud."""
        a = np.ascontiguousarray(normals, dtype=np.float32)
        if a.ndim != 2 or a.shape[1] not in (4, 8):
            raise ValueError("normals must be float32 [N,4] or [N,8]")
        self.ctx.check(self.ctx._L.dlg_cloud_set_normals(self.ctx.h, self.h, _f32p(a), a.shape[0],
                                                         4 * a.shape[1]))

    def estimate_normals(self, radius: float = 0.0, k: int = 0, viewpoint=(0.0, 0.0, 0.0),
                         mode: str = "pcl", copy_out: bool = False):
        """dlg_cloud_estimate_normals: estimateNormal() on this cloud's own device copy, the
        normals attached to the cloud (as set_normals; the cloud is reset) with no host round
        trip.  mode "pcl" (bit-exact PCL arithmetic) or "double".  copy_out: also return them
        as float32 [N,4] (nx, ny, nz, curvature)."""
        m = {"pcl": 0, "double": 1}[mode]
        vp = np.ascontiguousarray(viewpoint, np.float32)
        n = self.n
        out = np.empty((n, 4), np.float32) if copy_out else None
        self.ctx.check(self.ctx._L.dlg_cloud_estimate_normals(
            self.ctx.h, self.h, float(radius), int(k), _f32p(vp), m,
            _f32p(out) if copy_out else None, 16))
        return out

    def regulate_normals(self, seed_idx: int, seed_is_outward: bool, radius: float,
                         copy_out: bool = False):
        """dlg_cloud_regulate_normals: regulateNormal() (PlaneDetect.h:586-646) on this cloud's
        device copy and its attached normals, no host round trip; the regulated normals replace
        the attached ones (the cloud is reset).  -> (processed bool[N], number processed,
        normals float32 [N,4] when copy_out else None)."""
        n = self.n
        proc = np.zeros(max(n, 1), np.uint8)
        cnt = C.c_int64(0)
        out = np.empty((n, 4), np.float32) if copy_out else None
        self.ctx.check(self.ctx._L.dlg_cloud_regulate_normals(
            self.ctx.h, self.h, int(seed_idx), int(bool(seed_is_outward)), float(radius),
            proc.ctypes.data_as(C.POINTER(C.c_uint8)), C.byref(cnt),
            _f32p(out) if copy_out else None, 16))
        return proc[:n].astype(bool), int(cnt.value), out

    @property
    def n_active(self):
        v = C.c_int64()
        self.ctx.check(self.ctx._L.dlg_cloud_active(self.h, C.byref(v)))
        return v.value

    def close(self):
        if getattr(self, "h", None) is not None and self.h.value:
            if self.ctx.h.value:  # a closed context already released the device
                self.ctx._L.dlg_cloud_destroy(self.h)
            self.h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def shard_range(n_global: int, rank: int, world: int):
    """dlg_shard_range: the part [lo, hi) of an n_global-point cloud rank `rank` uploads (its
    contiguous shard; the whole cloud on every rank when shards would fall below the Morton-copy
    cut-off -- those clouds then run hypothesis-sharded by default) -> (lo, hi, replicated)."""
    L = _lib.load()
    lo, hi, rep = C.c_int64(), C.c_int64(), C.c_int()
    _lib.check(L.dlg_shard_range(int(n_global), int(rank), int(world), C.byref(lo), C.byref(hi),
                                 C.byref(rep)))
    return lo.value, hi.value, bool(rep.value)


def make_params(threshold=0.0, max_iterations=50, probability=0.99, optimize=True, seed=12345,
                refit_mode=DLG_REFIT_PCL, hypotheses_per_launch=0, gather_inliers=True,
                model=SACMODEL_PLANE, normal_distance_weight=0.1):
    L = _lib.load()
    p = _lib.SacParams()
    L.dlg_sac_params_default(C.byref(p))
    p.threshold = float(threshold)
    p.max_iterations = int(max_iterations)
    p.probability = float(probability)
    p.optimize = int(bool(optimize))
    p.seed = int(seed)
    p.refit_mode = int(refit_mode)
    p.hypotheses_per_launch = int(hypotheses_per_launch)
    p.gather_inliers = int(bool(gather_inliers))
    p.model = int(model)
    p.normal_distance_weight = float(normal_distance_weight)
    return p


def _stats_dict(st):
    return dict(iterations=st.iterations, skipped=st.skipped, has_model=bool(st.has_model),
                launches=st.launches, draws=st.draws,
                best_sample=np.array(st.best_sample[:], np.int32),
                coeff_unrefined=np.array(st.coeff_unrefined[:], np.float32),
                n_unrefined=st.n_unrefined, n_active=st.n_active, tests=st.tests,
                tests_scored=st.tests_scored, score_ms=st.score_ms)


def segment_cloud(cloud: Cloud, params, capacity=None):
    """One SACSegmentation::segment over the cloud's active list -> (inliers, coeff, stats)."""
    ctx = cloud.ctx
    cap = int(capacity if capacity is not None else max(cloud.n_active * max(ctx.world, 1), 1))
    inl = np.empty(max(cap, 1), np.int32)
    coeff = np.zeros(4, np.float32)
    n = C.c_int64()
    st = _lib.SacStats()
    ctx.check(ctx._L.dlg_sac_segment(ctx.h, cloud.h, C.byref(params), _f32p(coeff), _i32p(inl),
                                     cap, C.byref(n), C.byref(st)))
    return inl[:n.value], coeff, _stats_dict(st)  # a view: the buffer is this call's own


def extract_planes(cloud: Cloud, params, max_planes=20, min_inliers=0, capacity=None, out=None):
    """Sequential extract-and-remove -> dict(coeffs [P,4], offsets [P+1], inliers, stats).

    `out`: optional caller-owned int32 buffer for the inlier ids (reused across calls, like a
    std::vector the caller keeps); `inliers` is then a view of it."""
    ctx = cloud.ctx
    if out is not None:
        if out.dtype != np.int32 or not out.flags.c_contiguous or out.ndim != 1:
            raise ValueError("out must be a contiguous 1-D int32 array")
        inl, cap = out, int(out.size)
    else:
        cap = int(capacity if capacity is not None else max(cloud.n_active * max(ctx.world, 1), 1))
        inl = np.empty(max(cap, 1), np.int32)
    coeffs = np.zeros((max(max_planes, 1), 4), np.float32)
    offs = np.zeros(max_planes + 1, np.int64)
    npl = C.c_int()
    xs = _lib.ExtractStats()
    ctx.check(ctx._L.dlg_extract_planes(ctx.h, cloud.h, C.byref(params), int(max_planes),
                                        int(min_inliers), _f32p(coeffs),
                                        offs.ctypes.data_as(C.POINTER(C.c_int64)), _i32p(inl), cap,
                                        C.byref(npl), C.byref(xs)))
    k = npl.value
    stats = dict(rounds=xs.rounds, tests=xs.tests, tests_scored=xs.tests_scored,
                 score_launches=xs.score_launches, score_ms=xs.score_ms, select_ms=xs.select_ms,
                 wall_ms=xs.wall_ms, lean_rounds=xs.lean_rounds, spec_misses=xs.spec_misses,
                 pcl_host_checks=xs.pcl_host_checks, refit_walk_ms=xs.refit_walk_ms,
                 refit_repair_ms=xs.refit_repair_ms, refit_repairs=xs.refit_repairs,
                 refit_rebase_ms=xs.refit_rebase_ms)
    return dict(coeffs=coeffs[:k].copy(), offsets=offs[:k + 1].copy(),
                inliers=inl[:offs[k]], n_planes=k, stats=stats)


class RansacControl:
    """The host half of RandomSampleConsensus::computeModel (dlg_sac_control_*; no device).

    next() -> int32 [D, 3] global list positions of the next batch of draws (PCL's RNG and
    drawIndexSample swaps); consume(counts, good) replays computeModel over the batch and returns
    (batch index of a new best or -1, finished).  This is the replay dlg_sac_segment runs around
    its scoring kernel; point-sharded ranks each run one on the global N and summed counts.
    """

    def __init__(self, params, n_active_global: int, max_batch: int = 0):
        self._L = _lib.load()
        h = C.c_void_p()
        _lib.check(self._L.dlg_sac_control_create(C.byref(h), C.byref(params),
                                                  int(n_active_global), int(max_batch)))
        self.h = h
        self.n = int(n_active_global)

    def next(self) -> np.ndarray:
        d = C.c_int()
        st = self._L.dlg_sac_control_next(self.h, None, 0, C.byref(d))
        if d.value == 0:
            return np.zeros((0, 3), np.int32)
        if st != _lib.DLG_ERR_CAPACITY:
            _lib.check(st)
        pos = np.empty(3 * d.value, np.int32)
        _lib.check(self._L.dlg_sac_control_next(self.h, _i32p(pos), pos.size, C.byref(d)))
        return pos.reshape(-1, 3)

    def consume(self, counts, good):
        c = np.ascontiguousarray(counts, np.int32)
        g = np.ascontiguousarray(good, np.int32)
        if c.shape != g.shape:
            raise ValueError("counts and good differ in length")
        b, f = C.c_int(), C.c_int()
        _lib.check(self._L.dlg_sac_control_consume(self.h, _i32p(c), _i32p(g), c.shape[0],
                                                   C.byref(b), C.byref(f)))
        return b.value, bool(f.value)

    def result(self):
        st = _lib.SacStats()
        bd = C.c_int64()
        _lib.check(self._L.dlg_sac_control_result(self.h, C.byref(st), C.byref(bd)))
        r = _stats_dict(st)
        r["best_draw"] = bd.value
        return r

    def close(self):
        if self.h:
            self._L.dlg_sac_control_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


_default_ctx = threading.local()


def default_context() -> Context:
    c = getattr(_default_ctx, "ctx", None)
    if c is None:
        c = Context(0)
        _default_ctx.ctx = c
    return c


class SACSegmentation:
    """pcl::SACSegmentation<pcl::PointXYZ> (SACMODEL_PLANE, SAC_RANSAC) on the GPU."""

    def __init__(self, ctx: Context | None = None):
        self.ctx = ctx
        self.model_type = -1
        self.method_type = -1
        self.threshold = 0.0
        self.max_iterations = 50
        self.probability = 0.99
        self.optimize = True
        self.refit_mode = DLG_REFIT_PCL
        self.input = None
        self.indices = None
        self.last_stats = None

    _models = (SACMODEL_PLANE,)

    def _attach(self, cloud):
        pass

    # PCL setters (camelCase as in the reference's call sites) ------------------------------
    def setModelType(self, m):
        self.model_type = int(m)

    def setMethodType(self, m):
        self.method_type = int(m)

    def setDistanceThreshold(self, t):
        self.threshold = float(t)

    def setMaxIterations(self, n):
        self.max_iterations = int(n)

    def setProbability(self, p):
        self.probability = float(p)

    def setOptimizeCoefficients(self, b):
        self.optimize = bool(b)

    def setInputCloud(self, xyz):
        self.input = np.ascontiguousarray(xyz, dtype=np.float32)

    def setIndices(self, idx):
        self.indices = None if idx is None else np.ascontiguousarray(idx, dtype=np.int32)

    def setRefitMode(self, mode):
        self.refit_mode = int(mode)

    def segment(self):
        """-> (inliers int32[], coefficients float32[4] or [] when no model was found)."""
        if self.input is None:
            raise ValueError("setInputCloud() first")
        if self.model_type not in self._models:
            raise ValueError(f"model type {self.model_type} not supported here "
                             "(PCL: initSACModel fails)")
        if self.method_type not in (SAC_RANSAC,):
            raise ValueError("only SAC_RANSAC is supported")
        ctx = self.ctx or default_context()
        params = make_params(self.threshold, self.max_iterations, self.probability, self.optimize,
                             refit_mode=self.refit_mode, model=self.model_type,
                             normal_distance_weight=getattr(self, "normal_distance_weight", 0.1))
        cloud = Cloud(ctx, self.input, indices=self.indices)
        try:
            self._attach(cloud)
            inl, coeff, st = segment_cloud(cloud, params)
        finally:
            cloud.close()
        self.last_stats = st
        if not st["has_model"]:
            return np.zeros(0, np.int32), np.zeros(0, np.float32)
        return inl, coeff

    # snake_case aliases
    set_model_type = setModelType
    set_method_type = setMethodType
    set_distance_threshold = setDistanceThreshold
    set_max_iterations = setMaxIterations
    set_probability = setProbability
    set_optimize_coefficients = setOptimizeCoefficients
    set_input_cloud = setInputCloud
    set_indices = setIndices


class SACSegmentationFromNormals(SACSegmentation):
    """pcl::SACSegmentationFromNormals<PointXYZ, Normal> (SACMODEL_NORMAL_PLANE, SAC_RANSAC)."""

    _models = (SACMODEL_PLANE, SACMODEL_NORMAL_PLANE)

    def __init__(self, ctx: Context | None = None):
        super().__init__(ctx)
        self.normals = None
        self.normal_distance_weight = 0.1

    def setInputNormals(self, normals):
        self.normals = np.ascontiguousarray(normals, dtype=np.float32)

    def setNormalDistanceWeight(self, w):
        self.normal_distance_weight = float(w)

    def _attach(self, cloud):
        if self.model_type == SACMODEL_NORMAL_PLANE:
            if self.normals is None:
                raise ValueError("setInputNormals() first (PCL: no input normals)")
            cloud.set_normals(self.normals)

    set_input_normals = setInputNormals
    set_normal_distance_weight = setNormalDistanceWeight
