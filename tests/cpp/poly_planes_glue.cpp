// The polygon stage of INTEGRATION.md §3d compiled against the shim with the reference's struct
// Plane (Dialog/HeaderFile.h:81-88) and its globals: a cloud read from argv[1] (float32 x, y, z
// records) -> estimateNormal -> segmentPlanesRansac() (GPU extract-and-remove + fillPlaneClouds)
// -> polyPlanes() (PlaneDetect.h:1357-1374), here dialog::polyPlanes over dlg_plane_border in
// place of pcl::ConcaveHull.  Writes argv[2]: per plane its points_set and its border (int64
// counts + float32 x, y, z), read by tests/test_borders.py, which checks the border vertices
// against qhull's alpha shape of the same points (the fixture logic of
// test_plane_border_vertex_set_pinned).
#include <cstdio>
#include <memory>
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
float T_dist_point_plane = 0.02f;  // config.txt:29
int T_num_of_single_plane = 500;   // config.txt:20
float r_for_estimate_normal = 0.3f;
float alpha_poly = 0.5f;           // config.txt:28

int main(int argc, char** argv) {
  if (argc < 3) return 2;
  FILE* f = std::fopen(argv[1], "rb");
  if (!f) return 3;
  float p[3];
  while (std::fread(p, 4, 3, f) == 3) source_cloud->push_back(PointT(p[0], p[1], p[2]));
  std::fclose(f);
  {  // estimateNormal (PlaneDetect.h:515-545)
    dialog::NormalEstimation<pcl::PointXYZ, pcl::Normal> ne;
    ne.setInputCloud(source_cloud);
    ne.setRadiusSearch(r_for_estimate_normal);
    ne.compute(*source_normal);
  }
  {  // segmentPlanesRansac
    std::vector<dialog::PlaneResult> found;
    dialog::ExtractParams ep;
    ep.threshold = T_dist_point_plane;
    ep.min_inliers = T_num_of_single_plane;
    ep.max_iterations = 1000;
    dialog::extractPlanes(*source_cloud, ep, found);
    dialog::fillPlaneClouds(*source_cloud, *source_normal, found, plane_clouds);
  }
  const size_t built = dialog::polyPlanes(plane_clouds, alpha_poly);  // polyPlanes()
  // a second call leaves them alone (the reference skips planes whose border is set, :1364)
  const size_t again = dialog::polyPlanes(plane_clouds, alpha_poly);
  FILE* o = std::fopen(argv[2], "wb");
  if (!o) return 4;
  const int64_t np = (int64_t)plane_clouds.size();
  std::fwrite(&np, 8, 1, o);
  for (const Plane& pl : plane_clouds) {
    for (const PointCloudT* c : {pl.points_set.get(), pl.border.get()}) {
      const int64_t k = (int64_t)c->points.size();
      std::fwrite(&k, 8, 1, o);
      for (const PointT& q : c->points) std::fwrite(&q.x, 4, 3, o);
    }
  }
  std::fclose(o);
  std::printf("planes %lld built %zu again %zu\n", (long long)np, built, again);
  return 0;
}
