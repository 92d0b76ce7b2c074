// Smoke program for the C++ host shim (include/dialog/sac_segmentation.hpp), written the way the
// reference calls PCL (Dialog/SimplifyVerticesSize.cpp:62-67).  Without a GPU it must fail loudly
// (exit 3 = no device); with one it prints "coeff a b c d n_inliers".
#include <dialog/sac_segmentation.hpp>

#include <cmath>
#include <cstdio>

int main(int argc, char** argv) {
  pcl::PointCloud<pcl::PointXYZ>::Ptr cloud(new pcl::PointCloud<pcl::PointXYZ>);
  for (int i = 0; i < 64; ++i)
    for (int j = 0; j < 64; ++j) cloud->push_back(pcl::PointXYZ(0.1f * i, 0.1f * j, 0.01f * std::sin(0.3f * i * j)));
  for (int k = 0; k < 500; ++k) cloud->push_back(pcl::PointXYZ(0.013f * k, 0.007f * k, 1.0f + 0.002f * k));
  try {
    dialog::SACSegmentation<pcl::PointXYZ> seg;
    seg.setOptimizeCoefficients(true);
    seg.setModelType(pcl::SACMODEL_PLANE);
    seg.setMethodType(pcl::SAC_RANSAC);
    seg.setDistanceThreshold(0.02);
    seg.setInputCloud(cloud);
    pcl::PointIndices inliers;
    pcl::ModelCoefficients coeff;
    seg.segment(inliers, coeff);
    if (coeff.values.size() != 4) return 4;
    std::printf("coeff %.9g %.9g %.9g %.9g %zu\n", coeff.values[0], coeff.values[1], coeff.values[2],
                coeff.values[3], inliers.indices.size());
    std::vector<dialog::PlaneResult> planes;
    dialog::ExtractParams ep;
    ep.threshold = 0.02;
    ep.min_inliers = 100;
    dialog::extractPlanes(*cloud, ep, planes);
    std::printf("planes %zu\n", planes.size());
    // normals stage: estimateNormal() + regulateNormal(), then the normal-plane model
    pcl::PointCloud<pcl::Normal>::Ptr normals(new pcl::PointCloud<pcl::Normal>);
    dialog::NormalEstimation<pcl::PointXYZ, pcl::Normal> ne;
    ne.setInputCloud(cloud);
    ne.setRadiusSearch(0.25);
    ne.compute(*normals);
    std::vector<uint8_t> processed;
    int64_t reached = dialog::regulateNormals(*cloud, *normals, 0, true, 0.25f, &processed);
    dialog::orientNormalsToBackup(*cloud, *normals, *cloud, *normals);
    dialog::SACSegmentationFromNormals<pcl::PointXYZ, pcl::Normal> segn;
    segn.setModelType(pcl::SACMODEL_NORMAL_PLANE);
    segn.setMethodType(pcl::SAC_RANSAC);
    segn.setDistanceThreshold(0.05);
    segn.setNormalDistanceWeight(0.1);
    segn.setInputCloud(cloud);
    segn.setInputNormals(normals);
    pcl::PointIndices inl_n;
    pcl::ModelCoefficients coeff_n;
    segn.segment(inl_n, coeff_n);
    std::printf("normals %zu reached %lld np_inliers %zu\n", normals->points.size(), (long long)reached,
                inl_n.indices.size());
    pcl::PointCloud<pcl::PointXYZ> pre;
    std::vector<int> kept;
    float tr[3];
    dialog::preProcess(*cloud, true, 0.15f, pre, &kept, tr);
    std::printf("preprocess %zu %zu\n", pre.points.size(), kept.size());
    // postProcessPlanes: the 64x64 sheet as one plane holding every other point, its square
    // border; the other half is absorbed, the 500-point line is one cluster of the rest
    std::vector<dialog::PlaneSet<pcl::PointXYZ>> ps(1);
    for (int i = 0; i < 64 * 64; i += 2) ps[0].points_set.push_back(cloud->points[i]);
    ps[0].coeff = {0.0f, 0.0f, 1.0f};
    ps[0].border.push_back(pcl::PointXYZ(-0.05f, -0.05f, 0.0f));
    ps[0].border.push_back(pcl::PointXYZ(6.35f, -0.05f, 0.0f));
    ps[0].border.push_back(pcl::PointXYZ(6.35f, 6.35f, 0.0f));
    ps[0].border.push_back(pcl::PointXYZ(-0.05f, 6.35f, 0.0f));
    pcl::PointCloud<pcl::PointXYZ> src = *cloud;
    int start = 0;
    dialog::PostProcessParams pp;
    pp.radius_local = 0.05f;
    pp.t_cluster_num = 10;
    dialog::postProcessPlanes(src, ps, start, pp);
    std::printf("postprocess %zu %zu %zu %d\n", ps[0].points_set.points.size(), src.points.size(),
                ps[0].coeff.size(), start);
    return 0;
  } catch (const dialog::Error& e) {
    std::fprintf(stderr, "dialog error: %s\n", e.what());
    return (int)e.status;
  }
}
