/*
 * pcl_oracle.h -- TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of the PCL-1.8 arithmetic behind the RANSAC plane path that
 * the MI355X product (dialog_amd/) replaces.  Only tests/, __graft_entry__.smoke()
 * and bench.py's cpu_baseline leg may load this; the product never links it.
 *
 * Provenance / pinning status (see DESIGN.md "Oracle"):
 *   - The reference (czh55/Dialog) has no RANSAC plane code and no tests; the
 *     arithmetic lives in third-party PCL 1.8 (+ Eigen 3.3, Boost 1.64), which is
 *     not vendored under /root/reference and cannot be built here.
 *     Reference call sites: Dialog/SimplifyVerticesSize.cpp:62-67 (SACSegmentation),
 *     Dialog/PlaneDetect.h:529-535 (NormalEstimationOMP), PlaneDetect.h:547-665
 *     (regulateNormal).
 *   - PINNED: the RNG stream (mt19937 seeded 12345u) against libstdc++
 *     std::mt19937 and numpy's MT19937 (tests/golden/rng_kat.json).
 *   - UNPINNED ("parity unpinned" for the PCL arithmetic): op order of Eigen's SSE
 *     predux, PCL's RANSAC loop and eigen33 are restated from the published PCL
 *     1.8 / Eigen 3.3 sources; no reference output exists to check them against.
 *     A second, independent numpy restatement (oracle/numpy_twin.py) cross-checks
 *     this C code bit-for-bit.
 */
#ifndef DIALOG_PCL_ORACLE_H
#define DIALOG_PCL_ORACLE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- Boost.Random mt19937 + uniform_int<>(0, INT_MAX) (SampleConsensusModel::rnd) ---- */
typedef struct { uint32_t mt[624]; int idx; } orc_mt19937;
void     orc_mt_seed(orc_mt19937* g, uint32_t seed);
uint32_t orc_mt_next(orc_mt19937* g);
int      orc_rnd(orc_mt19937* g);          /* == mt() >> 1 (bucket size 2, never rejects) */

/* ---- SampleConsensusModelPlane primitives (pcl/sample_consensus/impl/sac_model_plane.hpp) ---- */
int   orc_plane_sample_good(const float p0[3], const float p1[3], const float p2[3]);
int   orc_plane_coefficients(const float p0[3], const float p1[3], const float p2[3], float c[4]);
float orc_plane_abs_dist(const float c[4], float x, float y, float z);
/* smallest float >= thr: (double)|d| < thr  <=>  |d| < orc_thr_ceil(thr) */
float orc_thr_ceil(double thr);

/* ---- pcl::computeMeanAndCovarianceMatrix (float, single pass, index order) + eigen33 ---- */
unsigned orc_mean_cov(const float* xyz, int64_t stride, const int32_t* idx, int64_t n,
                      float cov[9], float centroid[4]);
void orc_compute_roots(const float m[9], float roots[3]);
void orc_eigen33(const float m[9], float* eval, float evec[3]);
/* double-precision twin (fast-mode reference): two-pass centroid + covariance, eigen33 in double */
void orc_eigen33_d(const double m[9], double* eval, double evec[3]);
int  orc_refit_double(const float* xyz, int64_t stride, const int32_t* idx, int64_t n,
                      const float coeff_in[4], float coeff_out[4]);
/* the product's DLG_REFIT_FAST restated (dialog_amd/csrc/exact_refit.hpp definition) */
int  orc_fast_qexp(const float* xyz, int64_t stride, const int32_t* idx, int64_t n);
int  orc_refit_exact(const float* xyz, int64_t stride, const int32_t* idx, int64_t n, int qexp,
                     const float coeff_in[4], float coeff_out[4]);
/* its two halves: the 25 int64 moment digits of a point set (exact_refit.hpp layout; digit sums
 * of disjoint sets add), and the refit from summed digits (the multi-rank protocol) */
void orc_mom_digits(const float* xyz, int64_t stride, const int32_t* idx, int64_t n, int qexp,
                    int64_t digits[25]);
int  orc_refit_digits(const int64_t digits[25], int qexp, const float coeff_in[4], float coeff_out[4]);
/* threads of countWithinDistance (OpenMP; default 1 = PCL's serial loop) */
void orc_set_threads(int n);
int  orc_get_threads(void);

/* ---- SACSegmentation<PointXYZ>::segment with SACMODEL_PLANE / SAC_RANSAC, and
 *      SACSegmentationFromNormals with SACMODEL_NORMAL_PLANE ---- */
#define ORC_SACMODEL_PLANE 0
#define ORC_SACMODEL_NORMAL_PLANE 11
typedef struct {
  double   threshold;        /* setDistanceThreshold */
  int      max_iterations;   /* setMaxIterations (PCL default 50) */
  double   probability;      /* setProbability (default 0.99) */
  int      optimize;         /* setOptimizeCoefficients (default true) */
  uint32_t seed;             /* 12345u unless random_ */
  int      refit_double;     /* 0: PCL float refit; 1: two-pass double refit (LS reference);
                                2: the product's fast refit (exact moments, orc_refit_exact) */
  int      model;            /* ORC_SACMODEL_PLANE | ORC_SACMODEL_NORMAL_PLANE */
  double   normal_distance_weight;  /* setNormalDistanceWeight (PCL default 0.1) */
  const float* normals;      /* NORMAL_PLANE: 4 floats per point (nx, ny, nz, curvature) */
  int      fast_qexp;        /* refit_double 2: quantum exponent, ORC_QEXP_AUTO = from the
                                segmented points (extract: from the whole cloud) */
} orc_sac_params;
#define ORC_QEXP_AUTO (-100000)

typedef struct {
  int     iterations;        /* RandomSampleConsensus::iterations_ at exit */
  int     skipped;
  int64_t draws;             /* drawIndexSample calls */
  int32_t best_sample[3];    /* global indices of the winning triple */
  float   coeff_unrefined[4];
  int64_t n_unrefined;       /* inliers of the unrefined model */
  int     has_model;
} orc_sac_stats;

/* returns 1 if a model was found (PCL: computeModel true). inliers_out needs capacity n_idx
 * (or n_points when indices == NULL). "No model" leaves *n_inliers = 0 and coeff zeroed. */
int orc_sac_segment(const float* xyz, int64_t n_points, int64_t stride,
                    const int32_t* indices, int64_t n_idx, const orc_sac_params* prm,
                    float coeff[4], int32_t* inliers_out, int64_t* n_inliers, orc_sac_stats* st);

/* sequential extract-and-remove (analogue of the reference's re-run loop,
 * PCLViewer.cpp:1120-1177 / PlaneDetect.h:1500-1573): round r segments the ascending
 * remaining-index list (RNG reseeded each round), records the plane and removes its inliers.
 * Stops when fewer than max(3, min_inliers) points remain, when no model is found or when a
 * plane has fewer than min_inliers inliers (that plane is not recorded). */
int orc_extract_planes(const float* xyz, int64_t n_points, int64_t stride,
                       const orc_sac_params* prm, int max_planes, int64_t min_inliers,
                       float* coeffs /* 4*max_planes */, int64_t* offsets /* max_planes+1 */,
                       int32_t* inliers /* n_points */, int* n_planes);

/* NORMAL_PLANE distance of one point (|w d_normal + (1 - w) d_euclid|), and its count */
void orc_normalized4(const float v[3], float out[3]);
double orc_normal_plane_dist(const float c[4], const float p[3], const float nrm[4], double lambda);
int64_t orc_count_within_np(const float* xyz, int64_t stride, const float* normals,
                            const int32_t* idx, int64_t n, const float c[4], double thr,
                            double lambda);

/* count within distance for an arbitrary list of hypotheses (CPU baseline leg) */
int64_t orc_count_within(const float* xyz, int64_t stride, const int32_t* idx, int64_t n,
                         const float c[4], double thr);

/* ---- NormalEstimation (radius search) + flipNormalTowardsViewpoint; regulateNormal BFS ---- */
/* normals_out: 4 floats per point (nx, ny, nz, curvature); NaN when < 3 neighbours.
 * Neighbours: all j with dist2(i,j) < r*r (FLANN L2, ((dx^2+dy^2)+dz^2)), sorted by (dist2, j). */
void orc_estimate_normals(const float* xyz, int64_t n, int64_t stride, float radius,
                          const float vp[3], float* normals_out);
/* PlaneDetect.h:547-665 first-round branch: seed flip, BFS over radius neighbours (sorted). */
void orc_estimate_normals_knn_brute(const float* xyz, int64_t n, int64_t stride, int k_nn,
                                    const float vp[3], float* out);
void orc_estimate_normals_knn(const float* xyz, int64_t n, int64_t stride, int k_nn,
                              const float vp[3], float* out);
int64_t orc_regulate_normals(const float* xyz, int64_t n, int64_t stride, float* normals,
                             int64_t seed_idx, int seed_is_outward, float radius,
                             uint8_t* processed_out);

/* PlaneDetect.h:553-584: orientation from the nearest backup point (normals: 4 floats/point) */
void orc_orient_normals_nn(const float* xyz, int64_t n, int64_t stride, float* normals,
                           const float* ref_xyz, int64_t m, int64_t ref_stride,
                           const float* ref_normals);

/* PlaneDetect.h:448-512 preProcess(): NaN removal, centroid translation, redundancy removal */
int64_t orc_preprocess(const float* xyz, int64_t n, int64_t stride, int translate, float min_dist,
                       float* out_xyz, int32_t* out_index, float translation[3]);

/* ---- postProcessPlanes (PlaneDetect.h:1454-1579) and its parts ---- */
uint32_t orc_msvc_rand(uint32_t* state);  /* MSVC CRT rand() on an explicit state */
/* isPointInPoly (PlaneDetect.h:1891-1964) after srand(seed); border: nb vertices */
int orc_is_point_in_poly(const float p[3], const float coeff[4], const float* border, int64_t nb,
                         int64_t border_stride, float t_dist, uint32_t seed);
/* pcl::computePointNormal over all n points (features/normal_3d.h) [PCL-1.8 ext] */
int orc_compute_point_normal(const float* xyz, int64_t n, int64_t stride, float plane[4],
                             float* curvature);
void orc_refit_planes(int n_planes, const float* coeffs_in, const float* pts, int64_t stride,
                      const int64_t* offs, float* coeffs_out);
/* clusterFilt (PlaneDetect.h:1582-1655): valid[i] = 0 for clusters of <= t_cluster_num points */
void orc_cluster_filter(const float* xyz, int64_t n, int64_t stride, float radius,
                        int t_cluster_num, uint8_t* valid);
void orc_post_process_planes(const float* cloud, int64_t n, int64_t stride, int n_planes,
                             const float* coeffs_in, const float* pts, int64_t pts_stride,
                             const int64_t* pts_off, const float* border, int64_t border_stride,
                             const int64_t* border_off, float t_dist, int plane_start,
                             uint32_t seed, float radius_local, int t_cluster_num,
                             float* coeffs_out, uint8_t* absorbed, uint8_t* remaining);

#ifdef __cplusplus
}
#endif
#endif
