"""dialog_amd -- MI355X-native RANSAC plane segmentation for the czh55/Dialog plane stage.

The product path is libdialog_amd.so (hand-written gfx950 HIP kernels + C++ host driver behind the
C ABI in include/dialog_ransac.h).  This package holds the ctypes binding, a Python mirror of
PCL's SACSegmentation interface, the synthetic-cloud generator and PCD I/O.  There is no CPU
fallback: without the library or a gfx950 device every compute call raises.
"""
from .sac import (SAC_RANSAC, SACMODEL_NORMAL_PLANE, SACMODEL_PLANE, Cloud, Context,  # noqa: F401
                  RansacControl,
                  DialogError, SACSegmentation, SACSegmentationFromNormals, extract_planes,
                  make_params, segment_cloud, shard_range)
from .normals import (NormalEstimation, estimate_normals, orient_normals_nn,  # noqa: F401
                      regulate_normals)
from .preprocess import preprocess, remove_redundant_points  # noqa: F401
from .postprocess import (PostProcessParams, cluster_filter, plane_border,  # noqa: F401
                          post_process_planes, refit_planes)
from ._lib import DLG_REFIT_FAST, DLG_REFIT_PCL, LIB_PATH  # noqa: F401
from ._lib import (DLG_OPT_LEAN_ROUNDS, DLG_OPT_PCL_REFIT_DEVICE, DLG_OPT_PRUNE,  # noqa: F401
                   DLG_OPT_NORMALS_FUSED, DLG_OPT_PRUNE_NP, DLG_OPT_PRUNE_TILE_SCORER, DLG_TILE_BF16, DLG_TILE_EXACT, DLG_TILE_MFMA,
                   DLG_OPT_PRUNE_STATS, DLG_OPT_SCORE_KERNEL, DLG_OPT_SELECT_TILE,
                   DLG_OPT_REGULATE_WAVE, DLG_OPT_SPEC_PICK, DLG_OPT_FS_POISON, DLG_OPT_HYP_SHARD, DLG_OPT_FS_ONE_WALK, DLG_OPT_FS_SEGMENTS,
                   DLG_OPT_FAULT_INJECT, DLG_OPT_SYNC_CHECK, DLG_OPT_COMM_TIMEOUT_MS, DLG_OPT_SEL1_TICKET,
                   DLG_OPT_BOUNDS_STREAM, DLG_OPT_SPATIAL_CURVE, DLG_OPT_FS_JOIN, DLG_OPT_UNREFINED_LIST, DLG_ERR_COMM, DLG_ERR_INTERNAL, DLG_SCORE_BF16,
                   DLG_SCORE_EXACT, DLG_SCORE_PRUNED)

__all__ = ["Context", "Cloud", "SACSegmentation", "extract_planes", "segment_cloud", "make_params",
           "SACMODEL_PLANE", "SACMODEL_NORMAL_PLANE", "SAC_RANSAC", "DLG_REFIT_PCL",
           "DLG_REFIT_FAST", "DialogError", "LIB_PATH", "NormalEstimation", "estimate_normals",
           "regulate_normals", "SACSegmentationFromNormals", "orient_normals_nn",
           "preprocess", "remove_redundant_points", "PostProcessParams", "post_process_planes",
           "refit_planes", "cluster_filter", "RansacControl"]
