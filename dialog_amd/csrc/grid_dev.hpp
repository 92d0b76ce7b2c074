// grid_dev.hpp -- device helpers of the uniform neighbour-search grid (normals.hip,
// postprocess.hip): cell of a coordinate, cell key, occupied-cell table lookup, and the
// KdTreeFLANN squared distance.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

#include "normals.hpp"

namespace dlg {
namespace grid {

constexpr uint32_t kEmpty = 0xffffffffu;

__device__ __forceinline__ uint32_t hash_key(uint32_t k) {
  k ^= k >> 16;
  k *= 0x7feb352du;
  k ^= k >> 15;
  k *= 0x846ca68bu;
  k ^= k >> 16;
  return k;
}

__device__ __forceinline__ int cell_of(float v, float lo, float inv_cell, int g) {
  int c = (int)floorf((v - lo) * inv_cell);
  return c < 0 ? 0 : (c >= g ? g - 1 : c);
}

__device__ __forceinline__ uint32_t cell_key(const GridDesc& G, int x, int y, int z) {
  return (uint32_t)((z * G.g[1] + y) * G.g[0] + x);
}

// KdTreeFLANN L2: ((0 + dx^2) + dy^2) + dz^2 with d = query - point
__device__ __forceinline__ float flann_d2(float qx, float qy, float qz, float px, float py, float pz) {
  const float ex = qx - px, ey = qy - py, ez = qz - pz;
  return ((0.0f + ex * ex) + ey * ey) + ez * ez;
}

// [begin, end) of the sorted positions of cell key k (empty range if unoccupied)
__device__ __forceinline__ int2 cell_range(const uint32_t* __restrict__ tkeys,
                                           const int2* __restrict__ trange, uint32_t tmask,
                                           uint32_t k) {
  uint32_t h = hash_key(k) & tmask;
  while (true) {
    const uint32_t tk = tkeys[h];
    if (tk == k) return trange[h];
    if (tk == kEmpty) return make_int2(0, 0);
    h = (h + 1) & tmask;
  }
}

// the table slot of cell key k (-1 if unoccupied)
__device__ __forceinline__ int cell_slot(const uint32_t* __restrict__ tkeys, uint32_t tmask,
                                         uint32_t k) {
  uint32_t h = hash_key(k) & tmask;
  while (true) {
    const uint32_t tk = tkeys[h];
    if (tk == k) return (int)h;
    if (tk == kEmpty) return -1;
    h = (h + 1) & tmask;
  }
}

}  // namespace grid
}  // namespace dlg
