// dialog/sac_segmentation.hpp -- header-only C++ host shim over the C ABI (dialog_ransac.h).
//
// Keeps the interface the reference's code is written against:
//   * pcl::SACSegmentation<PointT> (setModelType / setMethodType / setDistanceThreshold /
//     setMaxIterations / setProbability / setOptimizeCoefficients / setInputCloud / setIndices /
//     segment(PointIndices&, ModelCoefficients&)), as called at
//     Dialog/SimplifyVerticesSize.cpp:62-67, :86-87 -> dialog::SACSegmentation<PointT>;
//   * the plane-stage slot of Dialog/PlaneDetect.h:667-1355 that fills
//     `plane_clouds` (PlaneDetect.h:100, struct Plane HeaderFile.h:81-88) ->
//     dialog::extractPlanes(cloud, params, planes) (sequential extract-and-remove RANSAC);
//   * pcl::SACSegmentationFromNormals (SACMODEL_NORMAL_PLANE) -> dialog::SACSegmentationFromNormals;
//   * estimateNormal() (PlaneDetect.h:515-545, pcl::NormalEstimationOMP with a radius; k = 20 at
//     PCLViewer.cpp:507-522) -> dialog::NormalEstimation<PointT, pcl::Normal>;
//   * regulateNormal() (PlaneDetect.h:547-665) -> dialog::regulateNormals (first round) and
//     dialog::orientNormalsToBackup (later rounds);
//   * preProcess() (PlaneDetect.h:448-512) -> dialog::preProcess.
// With real PCL available define DIALOG_HAVE_PCL before including; otherwise minimal
// layout-identical stand-ins for pcl::PointXYZ (16 B), pcl::Normal (32 B), pcl::PointCloud,
// pcl::ModelCoefficients and pcl::PointIndices are declared here.
// PCL failure behaviour is kept: segment() never throws for "no model" -- it prints an error in
// PCL_ERROR style and leaves inliers/coefficients empty.  Device/runtime errors throw
// dialog::Error (there is no CPU fallback).
#pragma once

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <memory>
#include <stdexcept>
#include <string>
#include <type_traits>
#include <vector>

#include "../dialog_ransac.h"

#ifdef DIALOG_HAVE_PCL
#include <pcl/ModelCoefficients.h>
#include <pcl/PointIndices.h>
#include <pcl/point_cloud.h>
#include <pcl/point_types.h>
#include <pcl/sample_consensus/method_types.h>
#include <pcl/sample_consensus/model_types.h>
#else
namespace pcl {
struct alignas(16) PointXYZ {
  float x, y, z, data_pad;
  PointXYZ() : x(0.f), y(0.f), z(0.f), data_pad(1.f) {}
  PointXYZ(float a, float b, float c) : x(a), y(b), z(c), data_pad(1.f) {}
};
struct alignas(16) Normal {
  float normal_x, normal_y, normal_z, data_pad;
  float curvature, pad_[3];
};
template <typename T>
struct PointCloud {
  typedef std::shared_ptr<PointCloud<T>> Ptr;
  typedef std::shared_ptr<const PointCloud<T>> ConstPtr;
  std::vector<T> points;
  uint32_t width = 0, height = 1;
  bool is_dense = true;
  size_t size() const { return points.size(); }
  void push_back(const T& p) { points.push_back(p); width = (uint32_t)points.size(); }
};
struct ModelCoefficients {
  typedef std::shared_ptr<ModelCoefficients> Ptr;
  std::vector<float> values;
};
struct PointIndices {
  typedef std::shared_ptr<PointIndices> Ptr;
  std::vector<int> indices;
};
enum SacModel { SACMODEL_PLANE = 0, SACMODEL_NORMAL_PLANE = 11 };
static const int SAC_RANSAC = 0;
}  // namespace pcl
#endif

static_assert(sizeof(pcl::PointXYZ) == 16, "pcl::PointXYZ must be 16 bytes (x, y, z, pad)");

namespace dialog {

struct Error : std::runtime_error {
  Error(dlg_status s, const std::string& m) : std::runtime_error(m), status(s) {}
  dlg_status status;
};

inline void check(dlg_status s, const dlg_ctx* c) {
  if (s != DLG_OK)
    throw Error(s, std::string(dlg_status_string(s)) + ": " + dlg_last_error(c));
}

// one device context per host thread (RAII)
class Context {
 public:
  explicit Context(int device = 0) { check(dlg_ctx_create(&c_, device), nullptr); }
  ~Context() { dlg_ctx_destroy(c_); }
  Context(const Context&) = delete;
  Context& operator=(const Context&) = delete;
  dlg_ctx* get() const { return c_; }
  static Context& thread_default() {
    thread_local Context ctx(0);
    return ctx;
  }

 private:
  dlg_ctx* c_ = nullptr;
};

template <typename PointT>
class SACSegmentation {
 public:
  typedef typename pcl::PointCloud<PointT>::ConstPtr PointCloudConstPtr;

  explicit SACSegmentation(Context* ctx = nullptr) : ctx_(ctx) { dlg_sac_params_default(&prm_); }

  void setInputCloud(const PointCloudConstPtr& cloud) { input_ = cloud; }
  void setIndices(const pcl::PointIndices::Ptr& idx) { indices_ = idx ? idx->indices : std::vector<int>(); has_idx_ = (bool)idx; }
  void setIndices(const std::vector<int>& idx) { indices_ = idx; has_idx_ = true; }
  void setModelType(int m) { model_ = m; }
  void setMethodType(int m) { method_ = m; }
  void setDistanceThreshold(double t) { prm_.threshold = t; }
  void setMaxIterations(int n) { prm_.max_iterations = n; }
  void setProbability(double p) { prm_.probability = p; }
  void setOptimizeCoefficients(bool b) { prm_.optimize = b ? 1 : 0; }
  // extension: DLG_REFIT_PCL (bit-exact with PCL, default) or DLG_REFIT_FAST
  void setRefitMode(int m) { prm_.refit_mode = m; }
  const dlg_sac_stats& lastStats() const { return stats_; }

  void segment(pcl::PointIndices& inliers, pcl::ModelCoefficients& coefficients) {
    inliers.indices.clear();
    coefficients.values.clear();
    if (!input_) {
      std::fprintf(stderr, "[dialog::SACSegmentation::segment] No input dataset given!\n");
      return;
    }
    if (model_ != pcl::SACMODEL_PLANE || method_ != pcl::SAC_RANSAC) {
      std::fprintf(stderr, "[dialog::SACSegmentation::segment] Error initializing the SAC model!\n");
      return;
    }
    prm_.model = DLG_SACMODEL_PLANE;
    dlg_ctx* c = (ctx_ ? ctx_ : &Context::thread_default())->get();
    dlg_points pts{input_->points.empty() ? nullptr : &input_->points[0].x,
                   (int64_t)input_->points.size(), (int64_t)sizeof(PointT)};
    const int64_t n = has_idx_ ? (int64_t)indices_.size() : pts.n;
    std::vector<int32_t> out((size_t)(n > 0 ? n : 1));
    std::vector<int32_t> idx32(indices_.begin(), indices_.end());
    float coeff[4];
    int64_t nin = 0;
    check(dlg_sac_segment_host(c, &pts, has_idx_ ? idx32.data() : nullptr, n, &prm_, coeff,
                               out.data(), (int64_t)out.size(), &nin, &stats_),
          c);
    if (!stats_.has_model) {
      std::fprintf(stderr, "[dialog::SACSegmentation::segment] Error segmenting the model! No solution found.\n");
      return;
    }
    inliers.indices.assign(out.begin(), out.begin() + nin);
    coefficients.values.assign(coeff, coeff + 4);
  }

 protected:
  Context* ctx_;
  dlg_sac_params prm_;
  dlg_sac_stats stats_{};
  PointCloudConstPtr input_;
  std::vector<int> indices_;
  bool has_idx_ = false;
  int model_ = -1, method_ = -1;
};

// pcl::SACSegmentationFromNormals<PointT, pcl::Normal>: SACMODEL_NORMAL_PLANE (or PLANE) with the
// input normals (one pcl::Normal per input point; setIndices selects from both)
template <typename PointT, typename PointNT = pcl::Normal>
class SACSegmentationFromNormals : public SACSegmentation<PointT> {
 public:
  typedef typename pcl::PointCloud<PointNT>::ConstPtr NormalsConstPtr;
  explicit SACSegmentationFromNormals(Context* ctx = nullptr) : SACSegmentation<PointT>(ctx) {}
  void setInputNormals(const NormalsConstPtr& normals) { normals_ = normals; }
  void setNormalDistanceWeight(double w) { weight_ = w; }

  void segment(pcl::PointIndices& inliers, pcl::ModelCoefficients& coefficients) {
    if (this->model_ != pcl::SACMODEL_NORMAL_PLANE) {
      SACSegmentation<PointT>::segment(inliers, coefficients);
      return;
    }
    inliers.indices.clear();
    coefficients.values.clear();
    if (!this->input_ || !normals_ || normals_->points.size() != this->input_->points.size()) {
      std::fprintf(stderr, "[dialog::SACSegmentationFromNormals::segment] No input dataset containing normals was given!\n");
      return;
    }
    if (this->method_ != pcl::SAC_RANSAC) {
      std::fprintf(stderr, "[dialog::SACSegmentationFromNormals::segment] Error initializing the SAC model!\n");
      return;
    }
    dlg_ctx* c = (this->ctx_ ? this->ctx_ : &Context::thread_default())->get();
    dlg_points pts{this->input_->points.empty() ? nullptr : &this->input_->points[0].x,
                   (int64_t)this->input_->points.size(), (int64_t)sizeof(PointT)};
    std::vector<int32_t> idx32(this->indices_.begin(), this->indices_.end());
    const int64_t n = this->has_idx_ ? (int64_t)idx32.size() : pts.n;
    dlg_cloud* cl = nullptr;
    check(dlg_cloud_upload(c, &pts, this->has_idx_ ? idx32.data() : nullptr, n, 0, &cl), c);
    std::unique_ptr<dlg_cloud, dlg_status (*)(dlg_cloud*)> guard(cl, dlg_cloud_destroy);
    check(dlg_cloud_set_normals(c, cl, normals_->points.empty() ? nullptr : &normals_->points[0].normal_x,
                                (int64_t)normals_->points.size(), (int64_t)sizeof(PointNT)),
          c);
    dlg_sac_params prm = this->prm_;
    prm.model = DLG_SACMODEL_NORMAL_PLANE;
    prm.normal_distance_weight = weight_;
    std::vector<int32_t> out((size_t)(n > 0 ? n : 1));
    float coeff[4];
    int64_t nin = 0;
    check(dlg_sac_segment(c, cl, &prm, coeff, out.data(), (int64_t)out.size(), &nin, &this->stats_), c);
    if (!this->stats_.has_model) {
      std::fprintf(stderr, "[dialog::SACSegmentationFromNormals::segment] Error segmenting the model! No solution found.\n");
      return;
    }
    inliers.indices.assign(out.begin(), out.begin() + nin);
    coefficients.values.assign(coeff, coeff + 4);
  }

 private:
  NormalsConstPtr normals_;
  double weight_ = 0.1;  // PCL default distance_weight_
};

// pcl::NormalEstimation(OMP)<PointT, pcl::Normal> (estimateNormal(), PlaneDetect.h:515-545)
template <typename PointT, typename PointNT = pcl::Normal>
class NormalEstimation {
 public:
  typedef typename pcl::PointCloud<PointT>::ConstPtr PointCloudConstPtr;
  explicit NormalEstimation(Context* ctx = nullptr) : ctx_(ctx) {}
  void setInputCloud(const PointCloudConstPtr& cloud) { input_ = cloud; }
  void setRadiusSearch(double r) { radius_ = r; k_ = 0; }
  void setKSearch(int k) { k_ = k; radius_ = 0.0; }
  void setViewPoint(float vx, float vy, float vz) { vp_[0] = vx; vp_[1] = vy; vp_[2] = vz; }
  // output: one PointNT per input point (NaN normal/curvature where < 3 neighbours)
  void compute(pcl::PointCloud<PointNT>& output) {
    output.points.clear();
    if (!input_) {
      std::fprintf(stderr, "[dialog::NormalEstimation::compute] No input dataset given!\n");
      return;
    }
    output.points.resize(input_->points.size());
    output.width = (uint32_t)output.points.size();
    output.height = 1;
    if (output.points.empty()) return;
    dlg_ctx* c = (ctx_ ? ctx_ : &Context::thread_default())->get();
    dlg_points pts{&input_->points[0].x, (int64_t)input_->points.size(), (int64_t)sizeof(PointT)};
    check(dlg_estimate_normals(c, &pts, (float)radius_, k_, vp_, &output.points[0].normal_x,
                               (int64_t)sizeof(PointNT)),
          c);
  }

 private:
  Context* ctx_;
  PointCloudConstPtr input_;
  double radius_ = 0.0;
  int k_ = 0;
  float vp_[3] = {0.f, 0.f, 0.f};
};

// regulateNormal() first round (PlaneDetect.h:586-646): returns the number of points reached;
// processed (optional) receives isProcessed[]
template <typename PointT, typename PointNT>
inline int64_t regulateNormals(const pcl::PointCloud<PointT>& cloud, pcl::PointCloud<PointNT>& normals,
                               int64_t selected_point_index, bool is_norm_direction_valid,
                               float r_for_regulate_normal, std::vector<uint8_t>* processed = nullptr,
                               Context* ctx = nullptr) {
  if (normals.points.size() != cloud.points.size()) throw Error(DLG_ERR_INVALID, "normals/cloud size mismatch");
  if (cloud.points.empty()) return 0;
  dlg_ctx* c = (ctx ? ctx : &Context::thread_default())->get();
  dlg_points pts{&cloud.points[0].x, (int64_t)cloud.points.size(), (int64_t)sizeof(PointT)};
  if (processed) processed->assign(cloud.points.size(), 0);
  int64_t count = 0;
  check(dlg_regulate_normals(c, &pts, &normals.points[0].normal_x, (int64_t)sizeof(PointNT),
                             selected_point_index, is_norm_direction_valid ? 1 : 0,
                             r_for_regulate_normal, processed ? processed->data() : nullptr, &count),
        c);
  return count;
}

// regulateNormal() later rounds (PlaneDetect.h:553-584): orientation from the nearest point of
// the backup cloud
template <typename PointT, typename PointNT>
inline void orientNormalsToBackup(const pcl::PointCloud<PointT>& cloud, pcl::PointCloud<PointNT>& normals,
                                  const pcl::PointCloud<PointT>& backup,
                                  const pcl::PointCloud<PointNT>& backup_normals, Context* ctx = nullptr) {
  if (normals.points.size() != cloud.points.size() || backup_normals.points.size() != backup.points.size())
    throw Error(DLG_ERR_INVALID, "normals/cloud size mismatch");
  if (cloud.points.empty()) return;
  dlg_ctx* c = (ctx ? ctx : &Context::thread_default())->get();
  dlg_points pts{&cloud.points[0].x, (int64_t)cloud.points.size(), (int64_t)sizeof(PointT)};
  dlg_points ref{backup.points.empty() ? nullptr : &backup.points[0].x, (int64_t)backup.points.size(),
                 (int64_t)sizeof(PointT)};
  check(dlg_orient_normals_nn(c, &pts, &normals.points[0].normal_x, (int64_t)sizeof(PointNT), &ref,
                              backup_normals.points.empty() ? nullptr : &backup_normals.points[0].normal_x,
                              (int64_t)sizeof(PointNT)),
        c);
}

// preProcess() (PlaneDetect.h:448-512) / removeRedundantPoints (PCLViewer.cpp:781-805): NaN
// removal, optional translation to the centroid (returned in *translation), redundancy removal
// with min_dist_between_points.  out: the kept points (translated); kept_index: their input index.
template <typename PointT>
inline void preProcess(const pcl::PointCloud<PointT>& cloud, bool translate, float min_dist,
                       pcl::PointCloud<PointT>& out, std::vector<int>* kept_index = nullptr,
                       float translation[3] = nullptr, Context* ctx = nullptr) {
  static_assert(sizeof(PointT) == 16, "preProcess writes pcl::PointXYZ records");
  out.points.clear();
  if (kept_index) kept_index->clear();
  if (cloud.points.empty()) return;
  dlg_ctx* c = (ctx ? ctx : &Context::thread_default())->get();
  dlg_points pts{&cloud.points[0].x, (int64_t)cloud.points.size(), (int64_t)sizeof(PointT)};
  out.points.resize(cloud.points.size());
  std::vector<int32_t> idx(cloud.points.size());
  int64_t n = 0;
  float tr[3];
  check(dlg_preprocess(c, &pts, translate ? 1 : 0, min_dist, &out.points[0].x, (int64_t)sizeof(PointT),
                       idx.data(), (int64_t)idx.size(), &n, tr),
        c);
  out.points.resize((size_t)n);
  out.width = (uint32_t)n;
  out.height = 1;
  if (kept_index) kept_index->assign(idx.begin(), idx.begin() + n);
  if (translation) { translation[0] = tr[0]; translation[1] = tr[1]; translation[2] = tr[2]; }
}

// The fields of the reference's struct Plane (HeaderFile.h:81-88) that postProcessPlanes reads
// and writes: points_set, coeff.values (3 = outward normal before the first post-process, 4
// after) and border (the polyPlanes polygon, PlaneDetect.h:1358-1436).
template <typename PointT>
struct PlaneSet {
  pcl::PointCloud<PointT> points_set;
  std::vector<float> coeff;
  pcl::PointCloud<PointT> border;
};

struct PostProcessParams {
  float t_dist_point_plane = 0.1f;  // config.ini [PlaneDetect] T_dist_point_plane
  float radius_local = 0.1f;        // radius_local (clusterFilt)
  int t_cluster_num = 500;          // T_cluster_num
  uint32_t rand_seed = 0;           // the time(0) value isPointInPoly seeds rand() with
};

// postProcessPlanes() (PlaneDetect.h:1454-1579) on the GPU: every plane's coeff becomes the
// oriented computePointNormal refit (4 values); planes [plane_start_index, size) absorb the
// cloud points inside their border polygon (appended to points_set in cloud order);
// source_cloud is replaced by the points left after clusterFilt; plane_start_index advances to
// planes.size() as in the reference (:1557-1558).
template <typename PointT>
inline void postProcessPlanes(pcl::PointCloud<PointT>& source_cloud,
                              std::vector<PlaneSet<PointT>>& planes, int& plane_start_index,
                              const PostProcessParams& pp, Context* ctx = nullptr) {
  dlg_ctx* c = (ctx ? ctx : &Context::thread_default())->get();
  const size_t np = planes.size();
  std::vector<float> coeffs(4 * (np ? np : 1), 0.0f), out(4 * (np ? np : 1), 0.0f);
  std::vector<PointT> pts, bor;
  std::vector<int64_t> poff(np + 1, 0), boff(np + 1, 0);
  for (size_t k = 0; k < np; ++k) {
    for (size_t j = 0; j < planes[k].coeff.size() && j < 4; ++j) coeffs[4 * k + j] = planes[k].coeff[j];
    pts.insert(pts.end(), planes[k].points_set.points.begin(), planes[k].points_set.points.end());
    bor.insert(bor.end(), planes[k].border.points.begin(), planes[k].border.points.end());
    poff[k + 1] = (int64_t)pts.size();
    boff[k + 1] = (int64_t)bor.size();
  }
  dlg_planes P{(int32_t)np, coeffs.data(), pts.empty() ? nullptr : &pts[0].x, (int64_t)sizeof(PointT),
               poff.data(), bor.empty() ? nullptr : &bor[0].x, (int64_t)sizeof(PointT), boff.data()};
  dlg_postprocess_params prm{pp.t_dist_point_plane, pp.radius_local, (int32_t)pp.t_cluster_num,
                             (int32_t)plane_start_index, pp.rand_seed};
  dlg_points cl{source_cloud.points.empty() ? nullptr : &source_cloud.points[0].x,
                (int64_t)source_cloud.points.size(), (int64_t)sizeof(PointT)};
  std::vector<int64_t> aoff(np + 1, 0);
  std::vector<int32_t> ids(source_cloud.points.size() ? source_cloud.points.size() : 1);
  std::vector<int32_t> rem(source_cloud.points.size() ? source_cloud.points.size() : 1);
  int64_t nrem = 0;
  dlg_status st = dlg_post_process_planes(c, &cl, &P, &prm, out.data(), aoff.data(), ids.data(),
                                          (int64_t)ids.size(), rem.data(), (int64_t)rem.size(), &nrem);
  if (st == DLG_ERR_CAPACITY && aoff[np] > (int64_t)ids.size()) {  // a point joined several planes
    ids.resize((size_t)aoff[np]);
    st = dlg_post_process_planes(c, &cl, &P, &prm, out.data(), aoff.data(), ids.data(),
                                 (int64_t)ids.size(), rem.data(), (int64_t)rem.size(), &nrem);
  }
  check(st, c);
  for (size_t k = 0; k < np; ++k) {
    planes[k].coeff.assign(out.begin() + 4 * k, out.begin() + 4 * k + 4);
    for (int64_t t = aoff[k]; t < aoff[k + 1]; ++t) planes[k].points_set.push_back(source_cloud.points[ids[t]]);
  }
  pcl::PointCloud<PointT> kept;
  kept.points.reserve((size_t)nrem);
  for (int64_t t = 0; t < nrem; ++t) kept.points.push_back(source_cloud.points[rem[t]]);
  kept.width = (uint32_t)kept.points.size();
  source_cloud = std::move(kept);
  plane_start_index = (int)np;
}

// Result of the plane stage for one plane: coefficients (a, b, c, d) and inlier ids.  The
// reference's struct Plane (HeaderFile.h:81-88) is filled from it by copying the inlier points
// into points_set and coeff.values (see INTEGRATION.md for the PlaneDetect.h adapter).
struct PlaneResult {
  float coeff[4];
  std::vector<int> indices;
};

struct ExtractParams {
  double threshold = 0.1;          // config.txt T_dist_point_plane (Dialog/config.txt:29)
  int64_t min_inliers = 500;       // config.txt T_num_of_single_plane (Dialog/config.txt:20)
  int max_planes = 64;
  int max_iterations = 1000;
  double probability = 0.99;
  int refit_mode = DLG_REFIT_PCL;
  // SACMODEL_NORMAL_PLANE when set: one pcl::Normal per cloud point
  const pcl::PointCloud<pcl::Normal>* normals = nullptr;
  double normal_distance_weight = 0.1;
};

template <typename PointT>
inline dlg_extract_stats extractPlanes(const pcl::PointCloud<PointT>& cloud, const ExtractParams& ep,
                                       std::vector<PlaneResult>& planes, Context* ctx = nullptr) {
  planes.clear();
  dlg_ctx* c = (ctx ? ctx : &Context::thread_default())->get();
  dlg_points pts{cloud.points.empty() ? nullptr : &cloud.points[0].x, (int64_t)cloud.points.size(),
                 (int64_t)sizeof(PointT)};
  dlg_cloud* cl = nullptr;
  check(dlg_cloud_upload(c, &pts, nullptr, 0, 0, &cl), c);
  std::unique_ptr<dlg_cloud, dlg_status (*)(dlg_cloud*)> guard(cl, dlg_cloud_destroy);
  dlg_sac_params prm;
  dlg_sac_params_default(&prm);
  if (ep.normals) {
    check(dlg_cloud_set_normals(c, cl, ep.normals->points.empty() ? nullptr : &ep.normals->points[0].normal_x,
                                (int64_t)ep.normals->points.size(), (int64_t)sizeof(pcl::Normal)),
          c);
    prm.model = DLG_SACMODEL_NORMAL_PLANE;
    prm.normal_distance_weight = ep.normal_distance_weight;
  }
  prm.threshold = ep.threshold;
  prm.max_iterations = ep.max_iterations;
  prm.probability = ep.probability;
  prm.refit_mode = ep.refit_mode;
  std::vector<float> coeffs(4 * (size_t)(ep.max_planes > 0 ? ep.max_planes : 1));
  std::vector<int64_t> offs((size_t)ep.max_planes + 1);
  std::vector<int32_t> ids(cloud.points.size() ? cloud.points.size() : 1);
  int np = 0;
  dlg_extract_stats xs{};
  check(dlg_extract_planes(c, cl, &prm, ep.max_planes, ep.min_inliers, coeffs.data(), offs.data(),
                           ids.data(), (int64_t)ids.size(), &np, &xs),
        c);
  for (int p = 0; p < np; ++p) {
    PlaneResult r;
    for (int k = 0; k < 4; ++k) r.coeff[k] = coeffs[4 * p + k];
    r.indices.assign(ids.begin() + offs[p], ids.begin() + offs[p + 1]);
    planes.push_back(std::move(r));
  }
  return xs;
}

// The plane stage's output for the reference's polyPlanes (PlaneDetect.h:1358-1440): one entry
// of `plane_clouds` (PlaneDetect.h:100) per RANSAC plane, PlaneT being the reference's struct
// Plane (HeaderFile.h:81-88: border, points_set, coeff, triangles_headfile).  As the reference's
// segmentation leaves it (PlaneDetect.h:997-999, 1094-1096): points_set = copies of the inlier
// points, border = null (polyPlanes builds the ConcaveHull border for every plane whose border is
// still null and skips the others, :1364), coeff.values = the 3 components of the plane normal
// pointing out of the object.  Orientation as the reference's (:1048-1050, 1086-1093): the
// regulated normal of the source point nearest plane->points[0] -- the first inlier itself --
// flips the normal when p_n . n < 0 (float dot in Eigen's Vector3f order; a NaN normal never
// flips).  Returns the number of planes appended.
template <typename PlaneT, typename Alloc, typename PointT, typename PointNT>
inline size_t fillPlaneClouds(const pcl::PointCloud<PointT>& cloud,
                              const pcl::PointCloud<PointNT>& normals,
                              const std::vector<PlaneResult>& found,
                              std::vector<PlaneT, Alloc>& plane_clouds) {
  if (normals.points.size() != cloud.points.size())
    throw Error(DLG_ERR_INVALID, "fillPlaneClouds: one normal per cloud point");
  size_t added = 0;
  for (const PlaneResult& pr : found) {
    if (pr.indices.empty()) continue;
    PlaneT pl;
    pl.points_set.reset(new pcl::PointCloud<PointT>);
    pl.points_set->points.reserve(pr.indices.size());
    for (int i : pr.indices) pl.points_set->push_back(cloud.points[(size_t)i]);
    const PointNT& nr = normals.points[(size_t)pr.indices[0]];
    const float dot = (nr.normal_x * pr.coeff[0] + nr.normal_y * pr.coeff[1]) + nr.normal_z * pr.coeff[2];
    const float sg = dot < 0.0f ? -1.0f : 1.0f;
    pl.coeff.values.assign({sg * pr.coeff[0], sg * pr.coeff[1], sg * pr.coeff[2]});
    plane_clouds.push_back(std::move(pl));
    ++added;
  }
  return added;
}

// polyPointCloud() (PlaneDetect.h:1376-1440) on dlg_plane_border: the plane's points projected
// onto their least-squares plane (pcl::computePointNormal + projPoint2Plane), the concave border
// of pcl::ConcaveHull (alpha shape of the projected points, alpha = alpha_poly, config.txt:28;
// the reference takes polygons[0], here the boundary polygon of largest area) appended to
// `border` in the reference's orientation (reversed when normalize(normalize(p1 - p0) x
// normalize(p2 - p1)) . pn < 0).  pn: any type with pn[0..2] (float[3], Eigen::Vector3f).  The
// input cloud is not modified (the reference projects a copy, :1367-1368).  A plane of fewer than
// 3 points gets no border.  Host arithmetic: replaces pcl::ConcaveHull (qhull) in polyPlanes.
template <typename PointT, typename Vec3>
inline void polyPointCloud(const pcl::PointCloud<PointT>& cloud, pcl::PointCloud<PointT>& border,
                           const Vec3& pn, float alpha_poly) {
  const int64_t n = (int64_t)cloud.points.size();
  static_assert(sizeof(PointT) >= 12, "PointT must start with float x, y, z");
  dlg_points pts{reinterpret_cast<const float*>(cloud.points.data()), n, (int64_t)sizeof(PointT)};
  const float v[3] = {(float)pn[0], (float)pn[1], (float)pn[2]};
  std::vector<PointT> out((size_t)std::max<int64_t>(n, 1));
  int64_t nb = 0;
  const dlg_status s = dlg_plane_border(&pts, v, alpha_poly, reinterpret_cast<float*>(out.data()),
                                        (int64_t)sizeof(PointT), n, &nb);
  if (s != DLG_OK) throw Error(s, std::string("dlg_plane_border: ") + dlg_status_string(s));
  for (int64_t i = 0; i < nb; ++i) {
    PointT q = PointT();
    q.x = out[(size_t)i].x; q.y = out[(size_t)i].y; q.z = out[(size_t)i].z;
    border.push_back(q);
  }
}

// polyPlanes() (PlaneDetect.h:1357-1374): every plane whose border is still null gets one from
// polyPointCloud over its points_set, oriented by its coeff.values[0..2] (the outward normal
// fillPlaneClouds stored); planes with a border are skipped, as in the reference.  PlaneT: the
// reference's struct Plane (HeaderFile.h:81-88).  Returns the number of borders built.
template <typename PlaneT, typename Alloc>
inline size_t polyPlanes(std::vector<PlaneT, Alloc>& plane_clouds, float alpha_poly) {
  size_t built = 0;
  for (PlaneT& pl : plane_clouds) {
    if (pl.border) continue;
    typedef typename std::remove_reference<decltype(*pl.points_set)>::type CloudT;
    pl.border.reset(new CloudT);
    if (!pl.points_set || pl.coeff.values.size() < 3) continue;
    const float pn[3] = {pl.coeff.values[0], pl.coeff.values[1], pl.coeff.values[2]};
    polyPointCloud(*pl.points_set, *pl.border, pn, alpha_poly);
    ++built;
  }
  return built;
}

}  // namespace dialog
