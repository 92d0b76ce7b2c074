// dialog/sac_segmentation.hpp -- header-only C++ host shim over the C ABI (dialog_ransac.h).
//
// Keeps the interface the reference's code is written against:
//   * pcl::SACSegmentation<PointT> (setModelType / setMethodType / setDistanceThreshold /
//     setMaxIterations / setProbability / setOptimizeCoefficients / setInputCloud / setIndices /
//     segment(PointIndices&, ModelCoefficients&)), as called at
//     Dialog/SimplifyVerticesSize.cpp:62-67, :86-87 -> dialog::SACSegmentation<PointT>;
//   * the plane-stage slot of Dialog/PlaneDetect.h:667-1355 that fills
//     `plane_clouds` (PlaneDetect.h:100, struct Plane HeaderFile.h:81-88) ->
//     dialog::extractPlanes(cloud, params, planes) (sequential extract-and-remove RANSAC).
// With real PCL available define DIALOG_HAVE_PCL before including; otherwise minimal
// layout-identical stand-ins for pcl::PointXYZ (16 B), pcl::Normal (32 B), pcl::PointCloud,
// pcl::ModelCoefficients and pcl::PointIndices are declared here.
// PCL failure behaviour is kept: segment() never throws for "no model" -- it prints an error in
// PCL_ERROR style and leaves inliers/coefficients empty.  Device/runtime errors throw
// dialog::Error (there is no CPU fallback).
#pragma once

#include <cstdint>
#include <cstdio>
#include <memory>
#include <stdexcept>
#include <string>
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

 private:
  Context* ctx_;
  dlg_sac_params prm_;
  dlg_sac_stats stats_{};
  PointCloudConstPtr input_;
  std::vector<int> indices_;
  bool has_idx_ = false;
  int model_ = -1, method_ = -1;
};

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

}  // namespace dialog
