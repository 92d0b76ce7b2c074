"""ctypes binding of include/dialog_ransac.h (libdialog_amd.so, built in-tree for gfx950).

No fallback: if the library is missing or no gfx950 device is visible, calls raise.
"""
from __future__ import annotations

import ctypes as C
import os

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "libdialog_amd.so")  # (A/B tooling rebinds it: tools/with_lib.py)

DLG_OK = 0
DLG_ERR_INTERNAL = 6
DLG_ERR_COMM = 4
DLG_ERR_CAPACITY = 5
DLG_SACMODEL_PLANE = 0
DLG_SACMODEL_NORMAL_PLANE = 11
DLG_REFIT_PCL = 0
DLG_REFIT_FAST = 1
ABI_VERSION = 5  # include/dialog_ransac.h DLG_ABI_VERSION: the structs below match that header

SYMBOLS = [
    "dlg_abi_version", "dlg_status_string", "dlg_sac_params_default", "dlg_ctx_create",
    "dlg_get_unique_id", "dlg_ctx_create_dist", "dlg_ctx_create_loopback_group", "dlg_ctx_destroy",
    "dlg_last_error", "dlg_ctx_info", "dlg_cloud_upload", "dlg_cloud_destroy", "dlg_cloud_reset",
    "dlg_cloud_active", "dlg_sac_segment", "dlg_sac_segment_host", "dlg_extract_planes",
    "dlg_set_profiling", "dlg_synchronize", "dlg_allreduce_max_f64", "dlg_barrier",
    "dlg_score_benchmark", "dlg_estimate_normals", "dlg_regulate_normals",
    "dlg_cloud_set_normals", "dlg_orient_normals_nn", "dlg_preprocess", "dlg_refit_planes",
    "dlg_post_process_planes", "dlg_cluster_filter", "dlg_sac_control_create",
    "dlg_sac_control_destroy", "dlg_sac_control_next", "dlg_sac_control_consume",
    "dlg_sac_control_result", "dlg_cloud_build_spatial", "dlg_ctx_set_option",
    "dlg_ctx_get_option", "dlg_prune_stats", "dlg_estimate_normals_ex", "dlg_cloud_drop_spatial",
    "dlg_abi_struct_size", "dlg_float_sums", "dlg_cloud_estimate_normals", "dlg_plane_border",
    "dlg_cloud_regulate_normals", "dlg_shard_range",
]

# context options (include/dialog_ransac.h): equivalent execution paths, identical results
DLG_OPT_PRUNE = 1
DLG_OPT_LEAN_ROUNDS = 2
DLG_OPT_SPEC_PICK = 3
DLG_OPT_PRUNE_NP = 4
DLG_OPT_SCORE_KERNEL = 5
DLG_OPT_PRUNE_STATS = 6
DLG_OPT_SELECT_TILE = 7
DLG_OPT_PCL_REFIT_DEVICE = 8
DLG_OPT_PRUNE_TILE_SCORER = 9
DLG_OPT_NORMALS_FUSED = 10
DLG_OPT_REGULATE_WAVE = 11
DLG_OPT_FS_POISON = 12
DLG_OPT_HYP_SHARD = 13
DLG_OPT_FS_ONE_WALK = 14
DLG_OPT_FS_SEGMENTS = 15
DLG_OPT_FAULT_INJECT = 16
DLG_OPT_SYNC_CHECK = 17
DLG_OPT_COMM_TIMEOUT_MS = 18
DLG_OPT_SEL1_TICKET = 19
DLG_OPT_BOUNDS_STREAM = 20
DLG_OPT_SPATIAL_CURVE = 21
DLG_OPT_FS_JOIN = 22
DLG_OPT_UNREFINED_LIST = 23
DLG_TILE_EXACT = 0
DLG_TILE_BF16 = 1
DLG_TILE_MFMA = 2
DLG_SCORE_EXACT = 0
DLG_SCORE_BF16 = 1
DLG_SCORE_PRUNED = 2


class Points(C.Structure):
    _fields_ = [("xyz", C.POINTER(C.c_float)), ("n", C.c_int64), ("stride_bytes", C.c_int64)]


class Planes(C.Structure):
    _fields_ = [("n_planes", C.c_int32), ("coeffs", C.POINTER(C.c_float)),
                ("points", C.POINTER(C.c_float)), ("points_stride_bytes", C.c_int64),
                ("point_offsets", C.POINTER(C.c_int64)), ("borders", C.POINTER(C.c_float)),
                ("borders_stride_bytes", C.c_int64), ("border_offsets", C.POINTER(C.c_int64))]


class PostProcessParams(C.Structure):
    _fields_ = [("t_dist_point_plane", C.c_float), ("radius_local", C.c_float),
                ("t_cluster_num", C.c_int32), ("plane_start_index", C.c_int32),
                ("rand_seed", C.c_uint32)]


class SacParams(C.Structure):
    _fields_ = [("threshold", C.c_double), ("max_iterations", C.c_int), ("probability", C.c_double),
                ("optimize", C.c_int), ("seed", C.c_uint32), ("model", C.c_int),
                ("normal_distance_weight", C.c_double), ("refit_mode", C.c_int),
                ("hypotheses_per_launch", C.c_int), ("gather_inliers", C.c_int)]


class SacStats(C.Structure):
    _fields_ = [("iterations", C.c_int), ("skipped", C.c_int), ("has_model", C.c_int),
                ("launches", C.c_int), ("draws", C.c_int64), ("best_sample", C.c_int32 * 3),
                ("coeff_unrefined", C.c_float * 4), ("n_unrefined", C.c_int64),
                ("n_active", C.c_int64), ("tests", C.c_int64), ("tests_scored", C.c_int64),
                ("score_ms", C.c_double)]


class ExtractStats(C.Structure):
    _fields_ = [("rounds", C.c_int), ("tests", C.c_int64), ("tests_scored", C.c_int64),
                ("score_launches", C.c_int), ("score_ms", C.c_double), ("select_ms", C.c_double),
                ("wall_ms", C.c_double), ("lean_rounds", C.c_int), ("spec_misses", C.c_int),
                ("pcl_host_checks", C.c_int), ("refit_walk_ms", C.c_double),
                ("refit_repair_ms", C.c_double), ("refit_repairs", C.c_int),
                ("refit_rebase_ms", C.c_double)]


_lib = None


def load():
    """Load libdialog_amd.so (building it first if it is missing)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        if LIB_PATH != os.path.join(HERE, "libdialog_amd.so"):
            raise RuntimeError(f"{LIB_PATH}: no such library")
        from . import build as _b
        _b.build()
    L = C.CDLL(LIB_PATH)
    if L.dlg_abi_version() != ABI_VERSION:
        raise RuntimeError(f"{LIB_PATH}: ABI version {L.dlg_abi_version()}, binding expects {ABI_VERSION}")
    vp = C.c_void_p
    pp = C.POINTER(C.c_void_p)
    i32p = C.POINTER(C.c_int32)
    i64p = C.POINTER(C.c_int64)
    fp = C.POINTER(C.c_float)
    L.dlg_abi_version.restype = C.c_int
    L.dlg_abi_struct_size.restype = C.c_int64
    L.dlg_abi_struct_size.argtypes = [C.c_int]
    L.dlg_status_string.restype = C.c_char_p
    L.dlg_status_string.argtypes = [C.c_int]
    L.dlg_sac_params_default.argtypes = [C.POINTER(SacParams)]
    L.dlg_sac_params_default.restype = None
    L.dlg_ctx_create.argtypes = [pp, C.c_int]
    L.dlg_get_unique_id.argtypes = [vp]
    L.dlg_ctx_create_dist.argtypes = [pp, C.c_int, C.c_int, C.c_int, vp]
    L.dlg_ctx_create_loopback_group.argtypes = [pp, C.c_int, C.c_int]
    L.dlg_ctx_destroy.argtypes = [vp]
    L.dlg_last_error.argtypes = [vp]
    L.dlg_last_error.restype = C.c_char_p
    L.dlg_ctx_info.argtypes = [vp, C.POINTER(C.c_int), C.POINTER(C.c_int), C.POINTER(C.c_int)]
    L.dlg_cloud_upload.argtypes = [vp, C.POINTER(Points), i32p, C.c_int64, C.c_int32, pp]
    L.dlg_cloud_destroy.argtypes = [vp]
    L.dlg_cloud_reset.argtypes = [vp]
    L.dlg_cloud_build_spatial.argtypes = [vp, vp]
    L.dlg_cloud_drop_spatial.argtypes = [vp]
    L.dlg_cloud_active.argtypes = [vp, i64p]
    L.dlg_sac_segment.argtypes = [vp, vp, C.POINTER(SacParams), fp, i32p, C.c_int64, i64p,
                                  C.POINTER(SacStats)]
    L.dlg_sac_segment_host.argtypes = [vp, C.POINTER(Points), i32p, C.c_int64,
                                       C.POINTER(SacParams), fp, i32p, C.c_int64, i64p,
                                       C.POINTER(SacStats)]
    L.dlg_extract_planes.argtypes = [vp, vp, C.POINTER(SacParams), C.c_int, C.c_int64, fp, i64p,
                                     i32p, C.c_int64, C.POINTER(C.c_int), C.POINTER(ExtractStats)]
    L.dlg_set_profiling.argtypes = [vp, C.c_int]
    L.dlg_synchronize.argtypes = [vp]
    L.dlg_allreduce_max_f64.argtypes = [vp, C.POINTER(C.c_double)]
    L.dlg_barrier.argtypes = [vp]
    L.dlg_score_benchmark.argtypes = [vp, vp, C.c_int, C.c_int, C.c_int, C.c_double,
                                      C.POINTER(C.c_double), i32p]
    L.dlg_float_sums.argtypes = [vp, fp, C.c_int64, fp, C.c_int, fp, fp, C.POINTER(C.c_int),
                                 C.POINTER(C.c_double), i64p]
    L.dlg_ctx_set_option.argtypes = [vp, C.c_int, C.c_int64]
    L.dlg_ctx_get_option.argtypes = [vp, C.c_int, i64p]
    L.dlg_prune_stats.argtypes = [vp, C.POINTER(C.c_uint64), C.c_int]
    L.dlg_preprocess.argtypes = [vp, C.POINTER(Points), C.c_int, C.c_float, fp, C.c_int64, i32p,
                                 C.c_int64, i64p, fp]
    L.dlg_orient_normals_nn.argtypes = [vp, C.POINTER(Points), fp, C.c_int64, C.POINTER(Points),
                                        fp, C.c_int64]
    L.dlg_cloud_set_normals.argtypes = [vp, vp, fp, C.c_int64, C.c_int64]
    L.dlg_cloud_estimate_normals.argtypes = [vp, vp, C.c_float, C.c_int, fp, C.c_int, fp,
                                             C.c_int64]
    L.dlg_plane_border.argtypes = [C.POINTER(Points), fp, C.c_float, fp, C.c_int64, C.c_int64,
                                   i64p]
    L.dlg_estimate_normals.argtypes = [vp, C.POINTER(Points), C.c_float, C.c_int, fp, fp, C.c_int64]
    L.dlg_estimate_normals_ex.argtypes = [vp, C.POINTER(Points), C.c_float, C.c_int, fp, fp,
                                          C.c_int64, C.c_int]
    L.dlg_regulate_normals.argtypes = [vp, C.POINTER(Points), fp, C.c_int64, C.c_int64, C.c_int,
                                       C.c_float, C.POINTER(C.c_uint8), i64p]
    L.dlg_cloud_regulate_normals.argtypes = [vp, vp, C.c_int64, C.c_int, C.c_float,
                                             C.POINTER(C.c_uint8), i64p, fp, C.c_int64]
    L.dlg_refit_planes.argtypes = [C.POINTER(Planes), fp]
    L.dlg_shard_range.argtypes = [C.c_int64, C.c_int, C.c_int, i64p, i64p, C.POINTER(C.c_int)]
    L.dlg_sac_control_create.argtypes = [pp, C.POINTER(SacParams), C.c_int64, C.c_int]
    L.dlg_sac_control_destroy.argtypes = [vp]
    L.dlg_sac_control_next.argtypes = [vp, i32p, C.c_int64, C.POINTER(C.c_int)]
    L.dlg_sac_control_consume.argtypes = [vp, i32p, i32p, C.c_int, C.POINTER(C.c_int),
                                          C.POINTER(C.c_int)]
    L.dlg_sac_control_result.argtypes = [vp, C.POINTER(SacStats), i64p]
    L.dlg_post_process_planes.argtypes = [vp, C.POINTER(Points), C.POINTER(Planes),
                                          C.POINTER(PostProcessParams), fp, i64p, i32p, C.c_int64,
                                          i32p, C.c_int64, i64p]
    L.dlg_cluster_filter.argtypes = [vp, C.POINTER(Points), C.c_float, C.c_int32, i32p,
                                     C.c_int64, i64p]
    for s in SYMBOLS:
        if s not in ("dlg_abi_version", "dlg_status_string", "dlg_sac_params_default",
                     "dlg_last_error", "dlg_abi_struct_size"):
            getattr(L, s).restype = C.c_int
    _lib = L
    return L


class DialogError(RuntimeError):
    def __init__(self, status, msg):
        super().__init__(f"dialog_amd error {status}: {msg}")
        self.status = status


def check(status, ctx=None):
    if status != DLG_OK:
        L = load()
        detail = L.dlg_last_error(ctx).decode(errors="replace")
        raise DialogError(status, f"{L.dlg_status_string(status).decode()}: {detail}")
