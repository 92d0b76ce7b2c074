// Test harness: the host alpha-shape module (dialog_amd/csrc/alpha_shape.hpp) behind plain C
// entry points, for tests/test_borders.py (compiled there with g++; no device).
#include <cstdint>
#include <cstring>

#include "../../dialog_amd/csrc/alpha_shape.hpp"

extern "C" {

// Delaunay triangles of n points (xy: 2 doubles each): writes up to cap triangles (3 ids each,
// counter-clockwise), returns the count
int64_t alpha_delaunay(const double* xy, int64_t n, int32_t* tri, int64_t cap) {
  const dlg::alpha::Tri2 T = dlg::alpha::Delaunay(xy, (int)n).run();
  const int64_t nt = (int64_t)T.tri.size() / 3;
  if (nt <= cap) std::memcpy(tri, T.tri.data(), sizeof(int32_t) * T.tri.size());
  return nt;
}

// kept triangles (flags per triangle of alpha_delaunay's order), the alpha shape's boundary
// vertices (point ids, first-met order) and PCL's polygon walk: returns the vertex count;
// poly_of[k] = the polygon of vertex position k (-1: in a run of < 3), order[k] = point id in
// walk order
int64_t alpha_boundary(const double* xy, int64_t n, double alpha, uint8_t* kept, int64_t kcap,
                       int32_t* verts, int32_t* order, int32_t* poly_of, int64_t vcap) {
  const dlg::alpha::Tri2 T = dlg::alpha::Delaunay(xy, (int)n).run();
  const dlg::alpha::AlphaShape S = dlg::alpha::alpha_shape(xy, T, alpha);
  if ((int64_t)S.kept.size() <= kcap) std::memcpy(kept, S.kept.data(), S.kept.size());
  const int64_t nv = (int64_t)S.av.size();
  if (nv <= vcap) {
    std::memcpy(verts, S.av.data(), sizeof(int32_t) * nv);
    for (int64_t k = 0; k < nv; ++k) { order[k] = -1; poly_of[k] = -1; }
    int64_t w = 0;
    for (size_t p = 0; p < S.polygons.size(); ++p)
      for (int32_t a : S.polygons[p]) {
        order[w] = S.av[a];
        poly_of[w] = (int32_t)p;
        ++w;
      }
  }
  return nv;
}

}  // extern "C"
