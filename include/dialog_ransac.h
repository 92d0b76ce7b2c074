/*
 * dialog_ransac.h -- C ABI of the MI355X-native RANSAC plane-segmentation path.
 *
 * Drop-in boundary for czh55/Dialog's plane stage.  The reference has no FFI of its own: its
 * plane stage is a header "module" of free functions over globals (Dialog/PlaneDetect.h:143-211,
 * source_cloud :104, source_normal :107, plane_clouds :100) that calls PCL.  These entry points
 * replace the PCL calls that sit under PlaneDetect.h's functions:
 *
 *   dlg_sac_segment      <- pcl::SACSegmentation<PointXYZ>::segment(PointIndices&, ModelCoefficients&)
 *                           with SACMODEL_PLANE / SAC_RANSAC (reference call pattern
 *                           Dialog/SimplifyVerticesSize.cpp:62-67, :86-87)
 *   dlg_extract_planes   <- the segmentation slot Dialog/PlaneDetect.h:667-1355 (createPS ..
 *                           mergePlanes) re-filled by sequential extract-and-remove RANSAC, the
 *                           analogue of the re-run loop PCLViewer.cpp:1120-1177 /
 *                           PlaneDetect.h:1500-1573; output feeds plane_clouds (PlaneDetect.h:100)
 *   dlg_estimate_normals <- estimateNormal(), Dialog/PlaneDetect.h:515-545
 *                           (pcl::NormalEstimationOMP, radius r_for_estimate_normal)
 *   dlg_regulate_normals <- regulateNormal(), Dialog/PlaneDetect.h:547-665
 *
 * Conventions: inputs are borrowed for the duration of a call; outputs go to caller buffers
 * (capacity given; DLG_ERR_CAPACITY + required size when too small).  No exceptions cross the
 * ABI.  "No model" is DLG_OK with *n_inliers == 0 and a zeroed coefficient vector (the C++ shim
 * maps it to PCL's empty indices/values).  One context per host thread; calls block until the
 * device work of the call has finished.  Every compute entry point runs on the GPU: there is no
 * CPU fallback, and creating a context without a usable HIP device fails with DLG_ERR_NO_DEVICE.
 */
#ifndef DIALOG_RANSAC_H
#define DIALOG_RANSAC_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* 2: dlg_extract_stats gained lean_rounds, spec_misses, pcl_host_checks; dlg_score_benchmark's
 * 4th argument is a DLG_SCORE_* kernel; execution paths are context options, not environment
 * variables.  3: dlg_extract_stats gained refit_walk_ms; dlg_float_sums, dlg_cloud_estimate_normals
 * and dlg_plane_border were added; dlg_cloud_drop_spatial keeps the copy's buffers.
 * 4: dlg_extract_stats gained refit_repair_ms (refit_walk_ms is k_fs_walk alone on every rank);
 * DLG_OPT_FS_POISON; dlg_cloud_regulate_normals; DLG_OPT_HYP_SHARD; DLG_OPT_FS_ONE_WALK;
 * dlg_extract_stats gained refit_repairs; dlg_prune_stats fills 8 counters; DLG_OPT_FS_SEGMENTS;
 * the tile-scorer option's getter returns the value set.
 * 5: a failing rank aborts its group (peers return DLG_ERR_COMM); DLG_OPT_FAULT_INJECT,
 * DLG_OPT_SYNC_CHECK, DLG_OPT_COMM_TIMEOUT_MS, DLG_OPT_SEL1_TICKET, DLG_OPT_BOUNDS_STREAM;
 * DLG_OPT_SPATIAL_CURVE, DLG_OPT_FS_JOIN, DLG_OPT_UNREFINED_LIST (same ABI version: added options);
 * DLG_OPT_HYP_SHARD defaults to -1 (automatic); dlg_shard_range */
#define DLG_ABI_VERSION 5

typedef enum {
  DLG_OK = 0,
  DLG_ERR_INVALID = 1,    /* bad argument */
  DLG_ERR_HIP = 2,        /* HIP runtime error */
  DLG_ERR_NO_DEVICE = 3,  /* no usable gfx950 device */
  DLG_ERR_COMM = 4,       /* RCCL / communicator error; several ranks: the group was aborted
                             (a peer's call failed -- dlg_last_error names the rank and its
                             error -- or a wait timed out).  An aborted group stays aborted:
                             destroy its contexts */
  DLG_ERR_CAPACITY = 5,   /* output buffer too small; required size reported */
  DLG_ERR_INTERNAL = 6
} dlg_status;

/* pcl::SacModel values (pcl/sample_consensus/model_types.h) */
enum { DLG_SACMODEL_PLANE = 0, DLG_SACMODEL_NORMAL_PLANE = 11 };
/* refit of the winning model (SampleConsensusModelPlane::optimizeModelCoefficients) */
enum {
  DLG_REFIT_PCL = 0,   /* PCL's float refit: computeMeanAndCovarianceMatrix's single-pass float
                          sums in list order + float eigen33, bit-exact with PCL.  The sums run
                          on the device, exactly (fsum.hpp); several ranks hand the chains'
                          values from rank to rank in list order (RCCL send/recv) */
  DLG_REFIT_FAST = 1   /* NOT PCL's arithmetic: exact integer moments of the inliers + a double
                          Jacobi solve (the least-squares plane to within float rounding; order-
                          and rank-count-independent).  Its planes differ from PCL's by up to
                          ~1e-4 and can change which plane a later extract round picks */
};

typedef struct dlg_ctx dlg_ctx;
typedef struct dlg_cloud dlg_cloud;

/* Host points, borrowed.  stride_bytes 16 = pcl::PointXYZ (x, y, z, pad), 12 = packed xyz. */
typedef struct {
  const float* xyz;
  int64_t n;
  int64_t stride_bytes;
} dlg_points;

typedef struct {
  double threshold;            /* setDistanceThreshold */
  int max_iterations;          /* setMaxIterations (PCL default 50) */
  double probability;          /* setProbability (PCL default 0.99) */
  int optimize;                /* setOptimizeCoefficients (PCL default 1) */
  uint32_t seed;               /* 12345u = PCL's non-random seed */
  int model;                   /* DLG_SACMODEL_PLANE | DLG_SACMODEL_NORMAL_PLANE (needs normals) */
  double normal_distance_weight; /* SACSegmentationFromNormals::setNormalDistanceWeight (0.1) */
  int refit_mode;              /* DLG_REFIT_PCL (default) | DLG_REFIT_FAST */
  int hypotheses_per_launch;   /* upper bound of one scoring launch; 0 = 4096 */
  int gather_inliers;          /* multi-rank: 1 = every rank receives the global inlier list */
} dlg_sac_params;

typedef struct {
  int iterations;              /* RandomSampleConsensus iterations_ at exit */
  int skipped;
  int has_model;
  int launches;                /* scoring launches */
  int64_t draws;               /* drawIndexSample calls */
  int32_t best_sample[3];      /* global indices of the winning triple */
  float coeff_unrefined[4];
  int64_t n_unrefined;         /* inliers of the unrefined model */
  int64_t n_active;            /* points the model was fitted on (all ranks) */
  int64_t tests;               /* point-plane tests PCL's loop evaluates (iterations x n_active) */
  int64_t tests_scored;        /* point-plane tests the GPU scored (>= tests: batch tail) */
  double score_ms;             /* device time of the scoring launches (HIP events) */
} dlg_sac_stats;

typedef struct {
  int rounds;                  /* segment() calls */
  int64_t tests;
  int64_t tests_scored;
  int score_launches;
  double score_ms;             /* sum of scoring-kernel device time */
  double select_ms;            /* sum of select/compact/moments device time */
  double wall_ms;              /* host wall time of the call */
  int lean_rounds;             /* rounds that took the single-pass (lean-list) select */
  int spec_misses;             /* speculative device picks the host replay overturned */
  int pcl_host_checks;         /* device PCL refits whose tail the host recomputed (an eigen33
                                  transcendental near a float rounding boundary) */
  double refit_walk_ms;        /* of select_ms: the device PCL refit's chain walks (k_fs_walk,
                                  latency-bound sequential chains), lean rounds */
  double refit_repair_ms;      /* several ranks: the PCL refit's repair phase on the stream (the
                                  exactness checks and the repair walks, k_fs_repair), summed
                                  over the rounds */
  int refit_repairs;           /* several ranks: the PCL refit's repair steps summed over the
                                  rounds (hand-over: W - 1 a round; DLG_OPT_FS_ONE_WALK 2: the
                                  parallel repair iterations) */
  double refit_rebase_ms;      /* several ranks, rank > 0, DLG_OPT_FS_ONE_WALK 0 / 2: the time
                                  between the first walk's end and the second walk's start (the
                                  allgather of the walks' ends + the rebase kernels); refit_walk_ms
                                  then holds the two walks alone */
} dlg_extract_stats;

void dlg_sac_params_default(dlg_sac_params* p);   /* PCL SACSegmentation defaults */
const char* dlg_status_string(dlg_status s);
int dlg_abi_version(void);
/* sizeof of the ABI's structs, for bindings to check their layouts: 0 dlg_points, 1 dlg_sac_params,
 * 2 dlg_sac_stats, 3 dlg_extract_stats, 4 dlg_planes, 5 dlg_postprocess_params; -1 otherwise */
int64_t dlg_abi_struct_size(int which);

/* ---- contexts ------------------------------------------------------------------------------ */
dlg_status dlg_ctx_create(dlg_ctx** out, int device);
/* one process per GPU: rank/world over RCCL (xGMI).  unique_id: 128 bytes from dlg_get_unique_id
 * on rank 0, distributed out of band (e.g. torch.distributed gloo).  world 1 with a NULL id is a
 * plain context; world 1 with an id runs a 1-rank RCCL communicator. */
dlg_status dlg_get_unique_id(void* unique_id_128);
dlg_status dlg_ctx_create_dist(dlg_ctx** out, int device, int rank, int world,
                               const void* unique_id_128);
/* in-process group of `world` ranks sharing one device, one host thread per rank (test and
 * rehearsal of the sharded path on a single GPU); the group's contexts must be driven
 * concurrently, rank r from its own thread. */
dlg_status dlg_ctx_create_loopback_group(dlg_ctx** out_array, int world, int device);
dlg_status dlg_ctx_destroy(dlg_ctx* ctx);
const char* dlg_last_error(const dlg_ctx* ctx);
dlg_status dlg_ctx_info(const dlg_ctx* ctx, int* rank, int* world, int* device);

/* ---- device-resident clouds (this rank's contiguous shard of the global index order) -------- */
/* The active list starts as point xyz[k] for k = indices[i] (pcl setIndices(); any order,
 * duplicates allowed) or k = 0..n-1 when indices is NULL; its global id is id_base + k.
 * Multi-rank: each rank uploads its contiguous shard with id_base = the shard's first global id;
 * the global active list is the concatenation of the ranks' lists in rank order. */
dlg_status dlg_cloud_upload(dlg_ctx* ctx, const dlg_points* pts, const int32_t* indices,
                            int64_t n_indices, int32_t id_base, dlg_cloud** out);
dlg_status dlg_cloud_destroy(dlg_cloud* cloud);
/* re-activate every point of the cloud (undo extract-and-remove) */
dlg_status dlg_cloud_reset(dlg_cloud* cloud);
/* Morton-ordered copy of the cloud's finite points + tile bounding spheres for the pruned
 * scoring kernel (same counts, fewer evaluated tests).  Built by dlg_cloud_upload for clouds of
 * >= 131072 points (context option DLG_OPT_PRUNE: 0 never, 1 always); this forces it for any cloud
 * (call right after upload or dlg_cloud_reset).  Kept in step by SACMODEL_PLANE extraction. */
dlg_status dlg_cloud_build_spatial(dlg_ctx* ctx, dlg_cloud* cloud);
/* drop the Morton copy (the exhaustive scoring kernels take over until it is built again; its
 * device buffers are kept for the next build and freed by dlg_cloud_destroy); resets the cloud to
 * all points active.  With dlg_cloud_build_spatial it times the index build on device-resident
 * points. */
dlg_status dlg_cloud_drop_spatial(dlg_cloud* cloud);
dlg_status dlg_cloud_active(const dlg_cloud* cloud, int64_t* n_active_local);
/* SACSegmentationFromNormals::setInputNormals: one normal record per uploaded point (n = the
 * dlg_points n of dlg_cloud_upload; the cloud's indices select from it like from the points).
 * stride_bytes 16 = (nx, ny, nz, curvature), >= 32 = pcl::Normal (curvature at byte 16).
 * Required by DLG_SACMODEL_NORMAL_PLANE; resets the cloud to all points active. */
dlg_status dlg_cloud_set_normals(dlg_ctx* ctx, dlg_cloud* cloud, const float* normals, int64_t n,
                                 int64_t stride_bytes);

/* ---- RANSAC ----------------------------------------------------------------------------------- */
/* SACSegmentation::segment on the cloud's active points (not removed).  inliers_out receives
 * global ids in active-list order (this rank's part, or all ranks' if gather_inliers). */
dlg_status dlg_sac_segment(dlg_ctx* ctx, dlg_cloud* cloud, const dlg_sac_params* prm,
                           float coeff_out[4], int32_t* inliers_out, int64_t cap,
                           int64_t* n_inliers, dlg_sac_stats* stats);

/* Host-buffer convenience: upload, segment, free (PCL setInputCloud + setIndices + segment). */
dlg_status dlg_sac_segment_host(dlg_ctx* ctx, const dlg_points* pts, const int32_t* indices,
                                int64_t n_indices, const dlg_sac_params* prm, float coeff_out[4],
                                int32_t* inliers_out, int64_t cap, int64_t* n_inliers,
                                dlg_sac_stats* stats);

/* Sequential extract-and-remove: round r runs segment() on the remaining points (RNG reseeded,
 * shuffled list = remaining list), records the plane and removes its inliers.  Stops when fewer
 * than max(3, min_inliers) points remain, when no model is found, or when a plane has fewer than
 * min_inliers inliers (not recorded).  coeffs_out: 4*max_planes floats; offsets_out:
 * max_planes+1 (offsets into inliers_out); inliers_out capacity `cap` ids. */
dlg_status dlg_extract_planes(dlg_ctx* ctx, dlg_cloud* cloud, const dlg_sac_params* prm,
                              int max_planes, int64_t min_inliers, float* coeffs_out,
                              int64_t* offsets_out, int32_t* inliers_out, int64_t cap,
                              int* n_planes, dlg_extract_stats* stats);

/* ---- normals (Dialog/PlaneDetect.h:515-665) -------------------------------------------------- */
/* pcl::NormalEstimation(OMP)::compute on every point of pts (estimateNormal(),
 * PlaneDetect.h:515-545): neighbours = radius search (k_nn == 0, radius > 0; PCL's radius
 * r_for_estimate_normal, config.txt:4) or the k_nn nearest (k_nn in 1..64; PCLViewer.cpp:507-522
 * uses 20), as KdTreeFLANN returns them; normal = eigenvector of the smallest eigenvalue of the
 * neighbourhood covariance, curvature = lambda0 / (lambda0 + lambda1 + lambda2), flipped towards
 * viewpoint (NULL = origin).  < 3 neighbours or a non-finite point -> NaN normal and curvature.
 * normals_out: n records of out_stride_bytes: 16 = (nx, ny, nz, curvature); >= 32 = pcl::Normal
 * (normal_x/y/z at bytes 0-11, curvature at byte 16, other fields zeroed). */
dlg_status dlg_estimate_normals(dlg_ctx* ctx, const dlg_points* pts, float radius, int k_nn,
                                const float viewpoint[3], float* normals_out,
                                int64_t out_stride_bytes);
/* dlg_estimate_normals with an arithmetic mode:
 *   DLG_NORMALS_PCL_FLOAT (what dlg_estimate_normals uses): PCL 1.8's computePointNormal --
 *     computeMeanAndCovarianceMatrix's single-pass float sums over the neighbours in FLANN's
 *     (d2, index) order, pcl::eigen33 in float, curvature |lambda0 / trace| in float, the
 *     viewpoint flip; bit-exact with the oracle's restatement of it
 *   DLG_NORMALS_CENTRED_DOUBLE: the same neighbourhoods, moments centred on the query in double
 *     and eigen33 in double (better conditioned far from the origin; not PCL's rounding) */
enum { DLG_NORMALS_PCL_FLOAT = 0, DLG_NORMALS_CENTRED_DOUBLE = 1 };
dlg_status dlg_estimate_normals_ex(dlg_ctx* ctx, const dlg_points* pts, float radius, int k_nn,
                                   const float viewpoint[3], float* normals_out,
                                   int64_t out_stride_bytes, int mode);
/* estimateNormal() on a cloud already on the device (the C5 chain: normals fused ahead of the
 * NORMAL_PLANE segmentation without a host round trip): the normals of dlg_estimate_normals_ex
 * (same neighbourhoods, same arithmetic for `mode`) over the cloud's uploaded points, attached
 * to the cloud as dlg_cloud_set_normals would attach them (the cloud is reset).  normals_out
 * (nullable): also copied out, records of out_stride_bytes as dlg_estimate_normals writes them.
 * One rank only: a context of a communicator with world > 1 holds a shard, whose points near the
 * cut would lose the neighbours on other ranks (PCL's normals are over the whole cloud), so it
 * gets DLG_ERR_INVALID -- estimate the normals over the whole cloud (dlg_estimate_normals_ex) and
 * attach each rank's slice with dlg_cloud_set_normals. */
dlg_status dlg_cloud_estimate_normals(dlg_ctx* ctx, dlg_cloud* cloud, float radius, int k_nn,
                                      const float viewpoint[3], int mode, float* normals_out,
                                      int64_t out_stride_bytes);
/* regulateNormal() first-round branch (PlaneDetect.h:586-646): flip the seed normal unless
 * seed_is_outward (is_norm_direction_valid), then BFS over radius-`radius` neighbourhoods
 * (r_for_regulate_normal, config.txt:9) in PCL's queue order, flipping each newly reached normal
 * whose float dot with the normal of the point that reached it is < 0.  normals_inout: n records
 * of stride_bytes (>= 12, multiple of 4); only normal_x/y/z are written.  processed_out
 * (nullable): n bytes, 1 = reached (isProcessed).  seed_idx < 0 is PCL's "invalid point index":
 * DLG_OK, nothing changed, *n_processed = 0. */
dlg_status dlg_regulate_normals(dlg_ctx* ctx, const dlg_points* pts, float* normals_inout,
                                int64_t stride_bytes, int64_t seed_idx, int seed_is_outward,
                                float radius, uint8_t* processed_out, int64_t* n_processed);

/* regulateNormal() first-round branch on a cloud's device copy and the normals attached to it
 * (dlg_cloud_estimate_normals or dlg_cloud_set_normals): the same BFS as dlg_regulate_normals
 * over the cloud's uploaded points, with no host round trip; the flipped normals replace the
 * attached ones (so a following SACMODEL_NORMAL_PLANE extraction uses them) and the cloud is
 * reset.  seed_idx indexes the cloud's points (upload order; with setIndices, the index list's
 * order).  processed_out (nullable): one byte per point; normals_out (nullable): the regulated
 * normals, stride 16 (x, y, z, curvature) or >= 32 (pcl::Normal).  One rank only. */
dlg_status dlg_cloud_regulate_normals(dlg_ctx* ctx, dlg_cloud* cloud, int64_t seed_idx,
                                      int seed_is_outward, float radius, uint8_t* processed_out,
                                      int64_t* n_processed, float* normals_out,
                                      int64_t out_stride_bytes);

/* regulateNormal() later-round branch (PlaneDetect.h:553-584, !isFirstPostProcess): each point
 * of pts takes the orientation of its nearest neighbour in the backup cloud ref_pts
 * (KdTreeFLANN::nearestKSearch k = 1; equidistant neighbours -> lowest index): its normal flips
 * when Vector3f(n).dot(Vector3f(n_ref)) < 0.  Only normal_x/y/z of normals_inout are written. */
dlg_status dlg_orient_normals_nn(dlg_ctx* ctx, const dlg_points* pts, float* normals_inout,
                                 int64_t stride_bytes, const dlg_points* ref_pts,
                                 const float* ref_normals, int64_t ref_stride_bytes);

/* ---- preprocessing (Dialog/PlaneDetect.h:448-512, PCLViewer.cpp:781-805) -------------------- */
/* preProcess(): pcl::removeNaNFromPointCloud, then (translate != 0) the translation of the cloud
 * to its centroid (sequential float sums / float(n), as the reference; translation[3] receives
 * it), then the redundancy removal: walking the points in order, a point is kept unless an
 * already kept point lies within min_dist (KdTreeFLANN radius test), i.e. the index-ordered
 * maximal independent set of the radius graph.  out_xyz: the kept (translated) points in input
 * order, records of out_stride_bytes (12 = xyz, 16 = pcl::PointXYZ with pad 1.0); out_index: their
 * input index.  *n_out = kept points (also on DLG_ERR_CAPACITY when cap is too small).  With
 * translate = 0 this is on_removeRedundantPointsAction_triggered (PCLViewer.cpp:781-805). */
dlg_status dlg_preprocess(dlg_ctx* ctx, const dlg_points* pts, int translate, float min_dist,
                          float* out_xyz, int64_t out_stride_bytes, int32_t* out_index,
                          int64_t cap, int64_t* n_out, float translation[3]);

/* ---- postProcessPlanes (Dialog/PlaneDetect.h:1454-1579) ------------------------------------ */
/* The final planes (plane_clouds_final, HeaderFile.h:98; struct Plane HeaderFile.h:81-88) as
 * borrowed host arrays: plane k owns points[point_offsets[k] .. point_offsets[k + 1]) (its
 * points_set) and border vertices [border_offsets[k] .. border_offsets[k + 1]) (its border, the
 * ConcaveHull polygon of polyPlanes, PlaneDetect.h:1358-1436), records of *_stride_bytes (12 or
 * >= 16, multiple of 4).  coeffs: 4 floats per plane (coeff.values; only [0..2], the outward
 * normal, is read). */
typedef struct {
  int32_t n_planes;
  const float* coeffs;
  const float* points;
  int64_t points_stride_bytes;
  const int64_t* point_offsets;  /* n_planes + 1 */
  const float* borders;
  int64_t borders_stride_bytes;
  const int64_t* border_offsets; /* n_planes + 1 */
} dlg_planes;

/* config.ini [PlaneDetect] values and the call's state (PlaneDetect.h:86-90, 1453) */
typedef struct {
  float t_dist_point_plane;  /* T_dist_point_plane: isPointInPoly's plane-distance gate */
  float radius_local;        /* radius_local: clusterFilt neighbourhood radius (>= 0) */
  int32_t t_cluster_num;     /* T_cluster_num: clusters of <= this many points are dropped */
  int32_t plane_start_index; /* planes [plane_start_index, n_planes) may absorb points */
  uint32_t rand_seed;        /* the srand(time(0)) value isPointInPoly reseeds rand() with */
} dlg_postprocess_params;

/* polyPlanes() -> polyPointCloud() (PlaneDetect.h:1358-1440) for one plane, so the four-file
 * polygon hand-off (PCLViewer.cpp:1341-1396) can run from RANSAC output alone: the plane's points
 * (its points_set) projected onto their least-squares plane (pcl::computePointNormal, PCL float
 * arithmetic) as projPoint2Plane does, then pcl::ConcaveHull's alpha shape (alpha = alpha_poly,
 * config.txt:28) restated step by step (PCA frame, Delaunay triangulation, circumradius filter,
 * boundary edges, PCL's polygon walk; dialog_amd/csrc/alpha_shape.hpp): the triangles, the alpha
 * filter and the boundary are qhull's ("QJ") on the committed fixtures.  The reference takes
 * polygons[0]; qhull's facet order, which decides that, is unpinned, so the border is the
 * boundary polygon of largest area.  Orientation as the reference: reversed when
 * normalize(normalize(p1 - p0) x normalize(p2 - p1)) . pn < 0.  border_out: up to cap records of
 * out_stride_bytes (>= 12; xyz first); *n_out = vertices (0: fewer than 3 points or no polygon),
 * also reported with DLG_ERR_CAPACITY.  Host arithmetic; no context.  The C++ shim's
 * dialog::polyPointCloud / dialog::polyPlanes wrap it (include/dialog/sac_segmentation.hpp). */
dlg_status dlg_plane_border(const dlg_points* plane_pts, const float pn[3], float alpha,
                            float* border_out, int64_t out_stride_bytes, int64_t cap,
                            int64_t* n_out);

/* PlaneDetect.h:1477-1498: coeffs_out[4k..4k+3] = pcl::computePointNormal of plane k's points
 * (float sums in list order, eigen33, d = -n.centroid; NaN with < 3 points), negated when its
 * dot with the previous normal coeffs[4k..4k+2] is < 0.  Host arithmetic (sequential float sums
 * are sequential by definition); no context needed. */
dlg_status dlg_refit_planes(const dlg_planes* planes, float* coeffs_out);

/* postProcessPlanes() minus its display/bookkeeping: (1) refit as dlg_refit_planes; (2) every
 * plane point marks its nearest cloud point processed (KdTreeFLANN nearestKSearch k = 1, ties ->
 * lowest index); (3) each unprocessed cloud point joins every plane k >= plane_start_index whose
 * isPointInPoly (PlaneDetect.h:1891-1964, after srand(rand_seed)) accepts it; (4) clusterFilt
 * (PlaneDetect.h:1582-1655) on the points still unprocessed.  Outputs: coeffs_out (4 per plane);
 * absorbed_offsets[n_planes + 1] and absorbed_ids: per plane, the ascending cloud indices it
 * absorbed (the shim appends those points to points_set); remaining_ids: ascending cloud indices
 * that form the new source_cloud.  Sizes are reported (absorbed_offsets[n_planes],
 * *n_remaining) also on DLG_ERR_CAPACITY.  A plane taking part in (3) must have >= 1 border
 * vertex (the reference divides by the border size).  Exact duplicate points are assumed absent
 * (preProcess removes them): clusterFilt's "skip the first neighbour" then skips the point
 * itself, and its BFS clusters are the connected components computed here. */
dlg_status dlg_post_process_planes(dlg_ctx* ctx, const dlg_points* cloud, const dlg_planes* planes,
                                   const dlg_postprocess_params* params, float* coeffs_out,
                                   int64_t* absorbed_offsets, int32_t* absorbed_ids,
                                   int64_t absorbed_cap, int32_t* remaining_ids,
                                   int64_t remaining_cap, int64_t* n_remaining);

/* clusterFilt() alone (PlaneDetect.h:1582-1655): ascending indices of the points whose
 * radius-`radius` connected component has more than t_cluster_num points. */
dlg_status dlg_cluster_filter(dlg_ctx* ctx, const dlg_points* pts, float radius,
                              int32_t t_cluster_num, int32_t* kept_ids, int64_t cap,
                              int64_t* n_kept);

/* ---- host-side RANSAC control (no device) ----------------------------------------------------
 * The sequential half of RandomSampleConsensus::computeModel [PCL-1.8 ext] that dlg_sac_segment
 * runs on the host, exported on its own so that a caller with another scorer -- and the
 * multi-rank CPU tests -- drive exactly the replay the GPU path uses:
 *   dlg_sac_control_next    <- SampleConsensusModel::getSamples/drawIndexSample (the RNG and the
 *                              swaps on the persistent shuffled index copy) for the next batch:
 *                              3 list positions per draw into the N_active-long global list;
 *   dlg_sac_control_consume <- computeModel's loop over the batch's (isSampleGood, count) pairs:
 *                              1000 bad draws in a row end it, strict '>' keeps the first best,
 *                              k = log(1-p)/log(1-w^3), the max_iterations break.
 * A batch must be consumed before the next one is drawn.  Point-sharded ranks each run one
 * controller on the global N and the summed counts and so take identical decisions. */
typedef struct dlg_sac_control dlg_sac_control;
dlg_status dlg_sac_control_create(dlg_sac_control** out, const dlg_sac_params* prm,
                                  int64_t n_active_global, int max_batch /* 0 = 4096 */);
dlg_status dlg_sac_control_destroy(dlg_sac_control* ctl);
/* *n_draws = size of the next batch (0 once the loop has ended); DLG_ERR_CAPACITY if
 * cap < 3 * *n_draws (nothing is drawn) */
dlg_status dlg_sac_control_next(dlg_sac_control* ctl, int32_t* positions_out, int64_t cap,
                                int* n_draws);
/* counts/good of the batch just drawn, in draw order; *best_in_batch = draw index of a new best
 * (-1: unchanged), *finished = 1 once computeModel's loop has ended */
dlg_status dlg_sac_control_consume(dlg_sac_control* ctl, const int32_t* counts,
                                   const int32_t* good, int n_draws, int* best_in_batch,
                                   int* finished);
/* iterations, draws, has_model, n_unrefined (best count), n_active, tests; best_draw = global
 * draw index (over all batches) of the winning hypothesis, -1 without a model */
dlg_status dlg_sac_control_result(const dlg_sac_control* ctl, dlg_sac_stats* st,
                                  int64_t* best_draw);

/* ---- profiling ------------------------------------------------------------------------------ */
/* Kernel-level HIP-event timing on the context's stream (bench roofline); off by default.
 * enable 1: the scoring launches, the select phase and the PCL refit walk; 2: without the walk's
 * events (each timing event on a dispatch costs the stream a few microseconds). */
dlg_status dlg_set_profiling(dlg_ctx* ctx, int enable);
dlg_status dlg_synchronize(dlg_ctx* ctx);
/* Scoring-kernel micro-benchmark (kernel A/B on the device): D random plane hypotheses through
 * the same gather/build path, `kernel` (DLG_SCORE_EXACT, DLG_SCORE_BF16 or DLG_SCORE_PRUNED, the
 * last needing the cloud's Morton copy) launched `reps` times on the cloud's active points;
 * returns the mean device time per launch and (optional) the counts of the last launch. */
dlg_status dlg_score_benchmark(dlg_ctx* ctx, dlg_cloud* cloud, int D, int kernel, int reps,
                               double threshold, double* ms_per_launch, int32_t* counts_out);
/* DLG_REFIT_PCL's device refit (fsum.hip) on caller data, for tests and measurement: the nine
 * sequential float sums of pcl::computeMeanAndCovarianceMatrix's dense branch (accu[0..8] =
 * xx, xy, xz, yy, yz, zz, x, y, z in list order) over n points (xyz: 3 floats each), then
 * optimizeModelCoefficients' float eigen33 refit of cin.  sums_out[9] and coeff_out[4] are the
 * device's bits; *uncertain = 1 when an eigen33 transcendental could not be rounded for certain
 * (the extraction then takes the host's value).  reps >= 1 launches are timed: *ms_per_call.
 * walk_stats (optional, the last call's; 8 int64 per chain, several counters packed):
 *   [0] windows walked record by record;
 *   [1] bits 0-31 speculation passes, bits 32-63 table lookups missed: no table built yet;
 *   [2] bits 0-31 passes needing the full lemma, bits 32-63 table lookups missed: lead out of
 *       the table's range;
 *   [3] bits 0-23 chunks stepped alone, bits 24-63 five 8-bit saturating buckets of the missed
 *       leads (|lead| < 128, < 512, < 4096, larger, not an exact multiple of the quantum);
 *   [4] bits 0-31 reruns, bits 32-63 table lookups missed: entry dropped by the builder;
 *   [5] shader clocks of the walk; [6] shader clocks of its integer stepping;
 *   [7] bits 0-31 windows passed by their summaries, bits 32-63 windows passed by a table. */
dlg_status dlg_float_sums(dlg_ctx* ctx, const float* xyz, int64_t n, const float cin[4], int reps,
                          float sums_out[9], float coeff_out[4], int* uncertain,
                          double* ms_per_call, int64_t* walk_stats /* nullable: [9][8] */);
/* Execution-path options of a context.  Every setting gives identical results (planes, inliers,
 * counts): they only choose among equivalent device paths, for tests and measurement.  There are
 * no environment switches in the library. */
enum {
  DLG_OPT_PRUNE = 1,        /* Morton copy + pruned countWithinDistance: -1 (default) clouds of
                               >= 131072 points, 0 never, 1 every cloud (applies at upload) */
  DLG_OPT_LEAN_ROUNDS = 2,  /* 1 (default): single-pass selects driven by the Morton copy in
                               SACMODEL_PLANE extraction, in every refit mode and at any rank
                               count (PCL refit on N > 1 ranks: each rank walks its shard's float
                               chains); 0: two-pass */
  DLG_OPT_SPEC_PICK = 3,    /* 1 (default): device-side computeModel decision for probability-1
                               rounds (host replay confirms it); 0: host decision only */
  DLG_OPT_PRUNE_NP = 4,     /* 1 (default): pruned SACMODEL_NORMAL_PLANE scoring; 0: exhaustive */
  DLG_OPT_SCORE_KERNEL = 5, /* exhaustive scorer (no Morton copy): DLG_SCORE_BF16 (default) or
                               DLG_SCORE_EXACT */
  DLG_OPT_PRUNE_STATS = 6,  /* 1: count the pruned kernel's work (dlg_prune_stats); 0 (default) */
  DLG_OPT_SELECT_TILE = 7,  /* points per tile of the lean rounds' single-pass selects: 4096,
                               8192 or 16384 (default) */
  DLG_OPT_PCL_REFIT_DEVICE = 8, /* DLG_REFIT_PCL: 1 (default) the float sums on the
                               device, exact (fsum.hpp); 0 gathered and summed on the host; 2 as 1,
                               the host recomputing every refit's tail from the sums; 3 as 2 and
                               every round's select redone with the host's plane (test) */
  DLG_OPT_PRUNE_TILE_SCORER = 9, /* the pruned plane scorer's (tile, plane) pairs:
                               DLG_TILE_EXACT (default) PCL-order f32 with lanes as planes, or
                               DLG_TILE_BF16 32x32 bf16 matrix-core blocks + band re-decision
                               (NORMAL_PLANE: DLG_TILE_EXACT lanes as planes with the prefilter
                               verdicts as bits, DLG_TILE_BF16 round 4's lanes-as-points scorer).
                               (A/B-only variants of the first, same counts: 11, 14 with 1, 4
                               planes per lane, 12 packed f32 tests, 15..17 item-claim orders;
                               the getter returns the value set) */
  DLG_OPT_NORMALS_FUSED = 10, /* PCL-float radius normals: 1 (default) search, (d2, index) order
                               and sums in one fused pass; 0: the chunked count / fill / sort /
                               sum pipeline */
  DLG_OPT_REGULATE_WAVE = 11, /* RegulateNormal's claim pass: 1 (default) one wave per frontier
                               node over its packed candidate cells; 0: one thread per (node,
                               cell) */
  DLG_OPT_FS_POISON = 12,   /* tests only: 1 fills the PCL float-sum walk's window tables with
                               garbage entries stamped for the next launch whenever its scratch
                               is laid out, before the clear; 0 (default) */
  DLG_OPT_HYP_SHARD = 13,   /* several ranks, small clouds (SURVEY 8(e)'s fallback): 1 = every
                               rank uploads the WHOLE cloud (id_base 0) and dlg_sac_segment /
                               dlg_extract_planes split each batch's hypotheses over the ranks
                               (rank r scores its slice, the counts are allreduced; the rest of
                               the round runs on every rank alike: same results as one rank).
                               0: point sharding (each rank uploads its shard).  -1 (default):
                               hypothesis sharding exactly when every rank holds the same cloud
                               (same ids and extent), decided once per cloud -- the layout
                               dlg_shard_range hands out when point shards would be too small */
  DLG_OPT_FS_ONE_WALK = 14, /* several ranks, PCL float refit (same sums every way): 0 (default)
                               = walk, rebase every rank on the guess the walks propagate, walk
                               again, then hand the exact chain ends rank to rank (each repair a
                               few windows long); 1 = no rebase: the repairs start from the
                               double-prefix guesses (the round-4 protocol, A/B only); 2 = 0 with
                               parallel repair iterations and host checks instead of the
                               hand-over (tests and A/B only) */
  DLG_OPT_FS_SEGMENTS = 15, /* one rank, PCL float refit: walkers per float chain, 1..16 (default
                               8): the chain's windows in segments walked at once from the refined
                               guesses, then joined in order (a segment whose guess was not its
                               exact start is walked again until it meets its recorded walk); 1 =
                               one walker per chain.  Same sums every way */
  DLG_OPT_FAULT_INJECT = 16, /* tests only: k > 0 = this rank fails (DLG_ERR_INTERNAL) in the
                               middle of extract round k - 1, after the round's scoring; 0
                               (default).  Exercises the group abort: every peer returns
                               DLG_ERR_COMM naming the failed rank */
  DLG_OPT_SYNC_CHECK = 17,  /* several ranks, debug: 1 = after every extract round the ranks
                               allgather (round, inliers, coefficient bits, collectives issued)
                               and fail the call (aborting the group) on any mismatch; 0 (default) */
  DLG_OPT_COMM_TIMEOUT_MS = 18, /* several ranks: a host wait on the group (a stream holding an
                               RCCL collective, a round's results) that makes no progress for this
                               long aborts the group (DLG_ERR_COMM on every rank); 0 = no limit;
                               default 600000 */
  DLG_OPT_SEL1_TICKET = 19, /* single-pass select tiles numbered by an atomic ticket taken at
                               dispatch (a tile's predecessors are then always resident, so the
                               look-back completes even beside other contexts' spinning selects on
                               the same device) or by workgroup index (complete in index order
                               while the launch has the device to itself): -1 (default) tickets
                               while another context of this process uses the same device, 1
                               always, 0 never */
  DLG_OPT_BOUNDS_STREAM = 20, /* lean rounds: 1 = the survivors' sphere bounds on a second stream
                               beside the list pass (event-ordered both ways); 0 (default) */
  DLG_OPT_SPATIAL_CURVE = 21, /* the spatial copy's point order (tiles of 32 consecutive points):
                               1 (default) = Hilbert curve, 0 = Morton (Z-order, rounds 1-5).
                               Same results either way; Hilbert tiles are more compact (no Z
                               jumps inside a tile), so fewer (tile, plane) pairs pass the
                               sphere tests.  Applies to clouds built after the change */
  DLG_OPT_FS_JOIN = 22,      /* one rank, PCL float refit, segmented walk: 1 (default) = the last
                               of a chain's segment walkers to finish joins the chain's segments in
                               the walk's own launch; 0 = the joins as a launch of their own
                               (round 5).  Same sums either way */
  DLG_OPT_UNREFINED_LIST = 23 /* lean rounds, PCL float refit: the unrefined plane's inliers in
                               list order by 1 (default) = one pass over the active list (k_ulist:
                               pristine coordinates gathered by index, look-back compaction); 0 =
                               stamps from the Morton copy's near tiles into a bitmap + its
                               compaction (rounds 3-5).  Same inliers either way */
};
enum { DLG_TILE_EXACT = 0, DLG_TILE_BF16 = 1, DLG_TILE_MFMA = 2 };
enum { DLG_SCORE_EXACT = 0, DLG_SCORE_BF16 = 1, DLG_SCORE_PRUNED = 2 };
dlg_status dlg_ctx_set_option(dlg_ctx* ctx, int option, int64_t value);
dlg_status dlg_ctx_get_option(const dlg_ctx* ctx, int option, int64_t* value);
/* the pruned scoring kernel's counters since DLG_OPT_PRUNE_STATS was set (or the last reset):
 * [0] workgroups (DLG_TILE_EXACT), [1] super-tile list entries tested against tile spheres, [2] tiles visited,
 * [3] 32x32 blocks (DLG_TILE_EXACT: 64-lane passes) scored, [4] (tile, plane) pairs scored,
 * [5] blocks with a band re-decision (DLG_TILE_BF16 only), [6] / [7] (DLG_TILE_EXACT) the sum
 * and the maximum of the workgroups' spans in 100 MHz clock ticks (load balance) */
dlg_status dlg_prune_stats(dlg_ctx* ctx, uint64_t out[8], int reset);

/* The shard of an n_global-point cloud rank `rank` of `world` should upload:
 * the contiguous range [*lo, *hi) of the global order, or -- when a shard would fall below the
 * 131072-point Morton-copy cut-off (the pruned scorer's minimum) and world > 1 -- the whole cloud
 * [0, n_global) on every rank, which DLG_OPT_HYP_SHARD's default (-1) then runs hypothesis-
 * sharded.  *replicated = 1 in that case.  Host arithmetic; no context. */
dlg_status dlg_shard_range(int64_t n_global, int rank, int world, int64_t* lo, int64_t* hi,
                           int* replicated);

/* max over ranks of a host double (bench timing) and a barrier; no-ops for world == 1 */
dlg_status dlg_allreduce_max_f64(dlg_ctx* ctx, double* value);
dlg_status dlg_barrier(dlg_ctx* ctx);

#ifdef __cplusplus
}
#endif
#endif /* DIALOG_RANSAC_H */
