// grid_host.hpp -- host helpers of the neighbour-search grids (normals_host.cpp), shared by the
// normals, preProcess and postProcessPlanes drivers.
#pragma once

#include "driver.hpp"
#include "normals.hpp"

namespace dlg {

struct BBox {
  float lo[3], hi[3];
  bool any;
};

// bounding box of the finite points of (X, Y, Z)[0..n)
BBox bbox_of(dlg_ctx* c, const float* X, const float* Y, const float* Z, int n);
// points -> device SoA (nw.x/y/z) + bounding box of the finite points
BBox upload_points(dlg_ctx* c, const dlg_points* pts);
// grid with cell edge >= `cell` (grown until the key space fits 2^30 cells)
GridDesc make_grid(const BBox& b, double cell);
// builds grid level `lv` over (X, Y, Z) (default nw.x/y/z); returns the number of occupied
// cells (and the point-weighted mean occupancy sum(occ^2) / n in *pw_occ)
uint32_t build_grid(dlg_ctx* c, int n, const GridDesc& G, int lv, GridBufs* B,
                    const float* X = nullptr, const float* Y = nullptr, const float* Z = nullptr,
                    double* pw_occ = nullptr);
// k-nearest-neighbour grid hierarchy over nw.x/y/z
KnnLevels build_hierarchy(dlg_ctx* c, int n, const BBox& b, int k_nn);
void check_points(const dlg_points* pts);

}  // namespace dlg
