// The PlaneDetect.h adapter of INTEGRATION.md §3 compiled against the shim's stand-in PCL types,
// with the reference's struct Plane (Dialog/HeaderFile.h:81-88) and its globals
// (source_cloud / source_normal PlaneDetect.h:104-107, plane_clouds PlaneDetect.h:100).  Run on
// the GPU by tests/test_gpu_parity.py: a closed box (six faces) -> estimateNormal (viewpoint at
// the box centre, then reversed: every normal outward, what regulateNormal() establishes) ->
// segmentPlanesRansac() -> the contract polyPlanes relies on (PlaneDetect.h:1364-1373): every
// plane has points, a null border (polyPlanes builds borders only where it is null), and
// coeff.values = 3 components pointing out of the box.  Orientation follows the reference's rule
// (PlaneDetect.h:1086-1093): the first inlier's normal decides, even against all the others.
#include <cmath>
#include <cstdio>
#include <memory>
#include <random>
#include <vector>

#include <dialog/sac_segmentation.hpp>

typedef pcl::PointXYZ PointT;
typedef pcl::PointCloud<PointT> PointCloudT;

struct Triangle_HeadFile {  // HeaderFile.h:74-79
  pcl::PointXYZ p_a, p_b, p_c;
};
struct Plane {  // HeaderFile.h:81-88
  PointCloudT::Ptr border;
  PointCloudT::Ptr points_set;
  pcl::ModelCoefficients coeff;
  std::vector<Triangle_HeadFile> triangles_headfile;
};

PointCloudT::Ptr source_cloud(new PointCloudT);
pcl::PointCloud<pcl::Normal>::Ptr source_normal(new pcl::PointCloud<pcl::Normal>);
std::vector<Plane> plane_clouds;
std::vector<dialog::PlaneResult> found;
float T_dist_point_plane = 0.02f;   // config.txt:29 (scaled to this cloud)
int T_num_of_single_plane = 500;    // config.txt:20
float r_for_estimate_normal = 0.1f; // config.txt:4

void estimateNormal(float vx, float vy, float vz) {  // PlaneDetect.h:515-545
  dialog::NormalEstimation<pcl::PointXYZ, pcl::Normal> ne;
  ne.setInputCloud(source_cloud);
  ne.setRadiusSearch(r_for_estimate_normal);
  ne.setViewPoint(vx, vy, vz);
  ne.compute(*source_normal);
}

void segmentPlanesRansac() {  // fills plane_clouds
  dialog::ExtractParams ep;
  ep.threshold = T_dist_point_plane;
  ep.min_inliers = T_num_of_single_plane;
  ep.max_iterations = 1000;
  dialog::extractPlanes(*source_cloud, ep, found);
  dialog::fillPlaneClouds(*source_cloud, *source_normal, found, plane_clouds);
}

int main() {
  const float cx = 3.f, cy = -2.f, cz = 1.5f, h = 1.f;  // box centre, half edge
  std::mt19937 g(7);
  std::uniform_real_distribution<float> u(-h, h);
  std::normal_distribution<float> eps(0.f, 0.002f);
  for (int f = 0; f < 6; ++f)
    for (int i = 0; i < 6000; ++i) {
      float p[3] = {u(g), u(g), u(g)};
      p[f / 2] = (f % 2 ? h : -h) + eps(g);
      source_cloud->push_back(PointT(cx + p[0], cy + p[1], cz + p[2]));
    }
  estimateNormal(cx, cy, cz);  // every normal points at the centre ...
  for (auto& n : source_normal->points) {  // ... reversed: outward (regulateNormal's job)
    n.normal_x = -n.normal_x; n.normal_y = -n.normal_y; n.normal_z = -n.normal_z;
  }
  segmentPlanesRansac();
  auto outward = [&](const Plane& pl) {  // the face centroid lies ~h along the outward normal
    double m[3] = {0, 0, 0};
    for (const auto& p : pl.points_set->points) { m[0] += p.x; m[1] += p.y; m[2] += p.z; }
    const double k = (double)pl.points_set->points.size();
    return pl.coeff.values[0] * (m[0] / k - cx) + pl.coeff.values[1] * (m[1] / k - cy) +
           pl.coeff.values[2] * (m[2] / k - cz);
  };
  int bad = 0;
  for (const Plane& pl : plane_clouds) {
    if (!pl.points_set || pl.points_set->points.empty() || pl.border || pl.coeff.values.size() != 3)
      ++bad;
    if (!(outward(pl) > 0.5)) ++bad;
  }
  // the first inlier's normal alone reversed: the reference's rule follows it (a majority vote
  // over the inliers would not)
  pcl::PointCloud<pcl::Normal> flipped = *source_normal;
  for (const auto& pr : found) {
    pcl::Normal& n = flipped.points[(size_t)pr.indices[0]];
    n.normal_x = -n.normal_x; n.normal_y = -n.normal_y; n.normal_z = -n.normal_z;
  }
  std::vector<Plane> inward;
  dialog::fillPlaneClouds(*source_cloud, flipped, found, inward);
  for (const Plane& pl : inward)
    if (!(outward(pl) < -0.5)) ++bad;
  std::printf("planes %zu bad %d\n", plane_clouds.size(), bad);
  return bad == 0 && plane_clouds.size() == 6 && inward.size() == 6 ? 0 : 1;
}
