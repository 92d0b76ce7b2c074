// normals.hip -- neighbour-search normal estimation and RegulateNormal BFS on gfx950.
//
// Replaces Dialog/PlaneDetect.h:515-545 estimateNormal() (pcl::NormalEstimationOMP with
// setRadiusSearch(r_for_estimate_normal)), the k = 20 NormalEstimation of PCLViewer.cpp:507-522 /
// TriangularMeshing.h:28-35, and the BFS of PlaneDetect.h:547-665 regulateNormal().
//
// Neighbour search: a uniform grid with cells >= r, points sorted by cell key (hipCUB radix sort,
// stable, so deterministic), occupied cells in an open-addressing hash (key -> [begin, end) of the
// sorted order).  A radius query visits the 27 cells around its own; the neighbour test is the
// one KdTreeFLANN applies: d2 = ((0 + dx^2) + dy^2) + dz^2 in float with d = q - p, kept iff
// d2 < (float)(r * r).  Every candidate sits in exactly one cell, so nothing is double counted.
//
// Normals: covariance of the neighbourhood accumulated in double on coordinates centred at the
// query (PCL 1.8 sums raw float coordinates single-pass; that loses ~1e-3 relative accuracy away
// from the origin -- the result here is the better-conditioned value of the same quantity),
// pcl::eigen33 in double, curvature = |lambda0 / trace|, flipNormalTowardsViewpoint in float in
// PCL's order.  Fewer than 3 neighbours or a non-finite query -> NaN normal and curvature.
//
// RegulateNormal: level-synchronous BFS that reproduces PCL's sequential queue exactly.  In the
// sequential BFS a node is claimed by the first popped node (queue order) having it within
// r_regulate; levels are contiguous in the queue, so a node is claimed by the smallest queue
// position of the current level that reaches it (32-bit atomicMin), and the next level is
// ordered as PCL pushes it: by parent position (counting sort: children per parent, scanned),
// then by the parent's neighbour-list order (d2, index) (rank among the siblings).  All level
// state stays on the device; the host only polls the level size every 16 levels.
// A node flips iff dot(parent normal, node normal) < 0 in float, left to right (PlaneDetect.h:629).
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <cfloat>
#include <climits>
#include <cmath>
#include <cstdint>
#include <type_traits>

#include "grid_dev.hpp"
#include "host_math.hpp"
#include "normals.hpp"

namespace dlg {

namespace {

using namespace grid;

constexpr int kBS = 256;


// append val to out[] for every lane with pred: one global atomic per wavefront (a single
// hot counter serialises at the L2 when every lane hits it).  All lanes of the wave must call.
__device__ __forceinline__ void wave_append(bool pred, int32_t val, int32_t* __restrict__ out,
                                            uint32_t* __restrict__ counter) {
  const uint64_t m = __ballot(pred);
  if (m == 0) return;
  const int lane = threadIdx.x & 63;
  const int leader = __ffsll((unsigned long long)m) - 1;
  uint32_t base = 0;
  if (lane == leader) base = atomicAdd(counter, (uint32_t)__popcll(m));
  base = __shfl(base, leader, 64);
  const int below = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32),
                                              __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
  if (pred) out[base + below] = val;
}

__device__ __forceinline__ bool finite3(float x, float y, float z) {
  return isfinite(x) && isfinite(y) && isfinite(z);
}




// ---------------------------------------------------------------------------------------------
// bounding box of the finite points
__global__ __launch_bounds__(kBS) void k_bbox(const float* __restrict__ X, const float* __restrict__ Y,
                                              const float* __restrict__ Z, int n,
                                              float* __restrict__ partial) {
  float lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
  for (int i = blockIdx.x * kBS + threadIdx.x; i < n; i += gridDim.x * kBS) {
    const float x = X[i], y = Y[i], z = Z[i];
    if (!finite3(x, y, z)) continue;
    lo[0] = fminf(lo[0], x); lo[1] = fminf(lo[1], y); lo[2] = fminf(lo[2], z);
    hi[0] = fmaxf(hi[0], x); hi[1] = fmaxf(hi[1], y); hi[2] = fmaxf(hi[2], z);
  }
  __shared__ float s[6][kBS / 64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  for (int k = 0; k < 3; ++k) {
    float a = lo[k], b = hi[k];
    for (int o = 32; o > 0; o >>= 1) {
      a = fminf(a, __shfl_xor(a, o, 64));
      b = fmaxf(b, __shfl_xor(b, o, 64));
    }
    if (lane == 0) { s[k][w] = a; s[3 + k][w] = b; }
  }
  __syncthreads();
  if (threadIdx.x < 6) {
    const int k = threadIdx.x;
    float v = s[k][0];
    for (int t = 1; t < kBS / 64; ++t) v = k < 3 ? fminf(v, s[k][t]) : fmaxf(v, s[k][t]);
    partial[6 * blockIdx.x + k] = v;
  }
}

__global__ __launch_bounds__(kBS) void k_cell_keys(const float* __restrict__ X,
                                                   const float* __restrict__ Y,
                                                   const float* __restrict__ Z, int n, GridDesc G,
                                                   uint32_t* __restrict__ keys,
                                                   int32_t* __restrict__ idx,
                                                   float4* __restrict__ rec) {
  const int i = blockIdx.x * kBS + threadIdx.x;
  if (i >= n) return;
  const float x = X[i], y = Y[i], z = Z[i];
  if (rec) rec[i] = make_float4(x, y, z, 0.0f);  // (k_cells_build's gather source)
  uint32_t k = G.ncells;  // non-finite: sorted last, never inserted
  if (finite3(x, y, z))
    k = cell_key(G, cell_of(x, G.lo[0], G.inv_cell, G.g[0]), cell_of(y, G.lo[1], G.inv_cell, G.g[1]),
                 cell_of(z, G.lo[2], G.inv_cell, G.g[2]));
  keys[i] = k;
  idx[i] = i;
}

// sorted keys -> cell table (begin) + coordinates in sorted order
__global__ __launch_bounds__(kBS) void k_cells_build(
    const uint32_t* __restrict__ skeys, const int32_t* __restrict__ sidx, int n, uint32_t ncells,
    const float* __restrict__ X, const float* __restrict__ Y, const float* __restrict__ Z,
    uint32_t* __restrict__ tkeys, int2* __restrict__ trange, uint32_t tmask,
    float* __restrict__ sx, float* __restrict__ sy, float* __restrict__ sz,
    uint32_t* __restrict__ n_occupied, const float4* __restrict__ rec) {
  __shared__ uint32_t s_occ;
  const int t = blockIdx.x * kBS + threadIdx.x;
  if (threadIdx.x == 0) s_occ = 0u;
  __syncthreads();
  const bool in = t < n;
  const uint32_t k = in ? skeys[t] : ncells;
  const bool first = in && k != ncells && (t == 0 || skeys[t - 1] != k);
  // occupied-cell count: one global atomic per workgroup (a single hot address: one per
  // wavefront measured ~1 ms at 10M points)
  const unsigned long long b = __ballot(first);
  if ((threadIdx.x & 63) == 0 && b) atomicAdd(&s_occ, (uint32_t)__popcll(b));
  __syncthreads();
  if (threadIdx.x == 0 && s_occ) atomicAdd(n_occupied, s_occ);
  if (!in) return;
  const int i = sidx[t];
  if (rec) {  // (one 16-byte record per point instead of three scattered floats)
    const float4 v = rec[i];
    sx[t] = v.x;
    sy[t] = v.y;
    sz[t] = v.z;
  } else {
    sx[t] = X[i];
    sy[t] = Y[i];
    sz[t] = Z[i];
  }
  if (!first) return;
  uint32_t h = hash_key(k) & tmask;
  while (true) {
    const uint32_t prev = atomicCAS(&tkeys[h], kEmpty, k);
    if (prev == kEmpty) break;
    h = (h + 1) & tmask;
  }
  trange[h].x = t;
}

// the last point of each cell run writes the run's end (separate launch: the begin must exist)
// ... and adds occupancy^2 of its cell to sumsq (sum over points of their cell's occupancy: the
// point-weighted occupancy the k-NN cell size is tuned on; sparse outlier cells barely count)
__global__ __launch_bounds__(kBS) void k_cells_end(const uint32_t* __restrict__ skeys, int n,
                                                   uint32_t ncells, const uint32_t* __restrict__ tkeys,
                                                   int2* __restrict__ trange, uint32_t tmask,
                                                   unsigned long long* __restrict__ sumsq) {
  const int t = blockIdx.x * kBS + threadIdx.x;
  unsigned long long sq = 0;
  if (t < n) {
    const uint32_t k = skeys[t];
    if (k != ncells && !(t + 1 < n && skeys[t + 1] == k)) {
      uint32_t h = hash_key(k) & tmask;
      while (tkeys[h] != k) h = (h + 1) & tmask;
      trange[h].y = t + 1;
      const unsigned long long occ = (unsigned long long)(t + 1 - trange[h].x);
      sq = occ * occ;
    }
  }
  for (int o = 32; o > 0; o >>= 1) sq += __shfl_xor(sq, o, 64);
  // (one global atomic per workgroup on the single hot address)
  __shared__ unsigned long long s_sq;
  if (threadIdx.x == 0) s_sq = 0ull;
  __syncthreads();
  if ((threadIdx.x & 63) == 0 && sq) atomicAdd(&s_sq, sq);
  __syncthreads();
  if (threadIdx.x == 0 && s_sq) atomicAdd(sumsq, s_sq);
}


// ---- pcl::computeRoots / pcl::eigen33 (common/impl/eigen.hpp), in double ----
__device__ void roots2_d(double b, double c, double r[3]) {
  r[0] = 0.0;
  double d = b * b - 4.0 * c;
  if (d < 0.0) d = 0.0;
  const double sd = sqrt(d);
  r[2] = 0.5 * (b + sd);
  r[1] = 0.5 * (b - sd);
}

__device__ void compute_roots_d(const double m[9], double r[3]) {
  const double c0 = m[0] * m[4] * m[8] + 2.0 * m[1] * m[2] * m[5] - m[0] * m[5] * m[5] -
                    m[4] * m[2] * m[2] - m[8] * m[1] * m[1];
  const double c1 =
      m[0] * m[4] - m[1] * m[1] + m[0] * m[8] - m[2] * m[2] + m[4] * m[8] - m[5] * m[5];
  const double c2 = m[0] + m[4] + m[8];
  if (fabs(c0) < DBL_EPSILON) {
    roots2_d(c2, c1, r);
    return;
  }
  const double s_inv3 = 1.0 / 3.0, s_sqrt3 = sqrt(3.0);
  const double c2_over_3 = c2 * s_inv3;
  double a_over_3 = (c1 - c2 * c2_over_3) * s_inv3;
  if (a_over_3 > 0.0) a_over_3 = 0.0;
  const double half_b = 0.5 * (c0 + c2_over_3 * (2.0 * c2_over_3 * c2_over_3 - c1));
  double q = half_b * half_b + a_over_3 * a_over_3 * a_over_3;
  if (q > 0.0) q = 0.0;
  const double rho = sqrt(-a_over_3);
  const double theta = atan2(sqrt(-q), half_b) * s_inv3;
  const double ct = cos(theta), st = sin(theta);
  r[0] = c2_over_3 + 2.0 * rho * ct;
  r[1] = c2_over_3 - rho * (ct + s_sqrt3 * st);
  r[2] = c2_over_3 - rho * (ct - s_sqrt3 * st);
  double t;
  if (r[0] >= r[1]) { t = r[0]; r[0] = r[1]; r[1] = t; }
  if (r[1] >= r[2]) {
    t = r[1]; r[1] = r[2]; r[2] = t;
    if (r[0] >= r[1]) { t = r[0]; r[0] = r[1]; r[1] = t; }
  }
  if (r[0] <= 0.0) roots2_d(c2, c1, r);
}

// smallest eigenvalue / eigenvector of a symmetric 3x3 (row-major m)
__device__ void eigen33_d(const double mat[9], double* eval, double v[3]) {
  double scale = 0.0;
  for (int k = 0; k < 9; ++k) scale = fmax(scale, fabs(mat[k]));
  if (scale <= DBL_MIN) scale = 1.0;
  double m[9];
  for (int k = 0; k < 9; ++k) m[k] = mat[k] / scale;
  double r[3];
  compute_roots_d(m, r);
  *eval = r[0] * scale;
  m[0] -= r[0]; m[4] -= r[0]; m[8] -= r[0];
  // row0 x row1, row0 x row2, row1 x row2
  const double a0x = m[1] * m[5] - m[2] * m[4], a0y = m[2] * m[3] - m[0] * m[5], a0z = m[0] * m[4] - m[1] * m[3];
  const double a1x = m[1] * m[8] - m[2] * m[7], a1y = m[2] * m[6] - m[0] * m[8], a1z = m[0] * m[7] - m[1] * m[6];
  const double a2x = m[4] * m[8] - m[5] * m[7], a2y = m[5] * m[6] - m[3] * m[8], a2z = m[3] * m[7] - m[4] * m[6];
  const double l0 = a0x * a0x + a0y * a0y + a0z * a0z;
  const double l1 = a1x * a1x + a1y * a1y + a1z * a1z;
  const double l2 = a2x * a2x + a2y * a2y + a2z * a2z;
  double vx = a0x, vy = a0y, vz = a0z, l = l0;
  if (l1 > l) { vx = a1x; vy = a1y; vz = a1z; l = l1; }
  if (l2 > l) { vx = a2x; vy = a2y; vz = a2z; l = l2; }
  const double s = sqrt(l);
  v[0] = vx / s; v[1] = vy / s; v[2] = vz / s;
}

// centred double moments -> (normal, curvature), viewpoint flip in float (PCL order)
struct Moments {
  double s0 = 0, sx = 0, sy = 0, sz = 0, sxx = 0, sxy = 0, sxz = 0, syy = 0, syz = 0, szz = 0;
  __device__ __forceinline__ void add(float px, float py, float pz, float qx, float qy, float qz) {
    const double ax = (double)px - qx, ay = (double)py - qy, az = (double)pz - qz;
    s0 += 1.0;
    sx += ax; sy += ay; sz += az;
    sxx += ax * ax; sxy += ax * ay; sxz += ax * az;
    syy += ay * ay; syz += ay * az; szz += az * az;
  }
};

__device__ float4 finish_normal(const Moments& M, float qx, float qy, float qz, float vpx,
                                float vpy, float vpz) {
  if (M.s0 < 3.0) {
    const float qnan = __builtin_nanf("");
    return make_float4(qnan, qnan, qnan, qnan);
  }
  const double inv = 1.0 / M.s0;
  const double mx = M.sx * inv, my = M.sy * inv, mz = M.sz * inv;
  double cov[9];
  cov[0] = M.sxx * inv - mx * mx;
  cov[1] = M.sxy * inv - mx * my;
  cov[2] = M.sxz * inv - mx * mz;
  cov[4] = M.syy * inv - my * my;
  cov[5] = M.syz * inv - my * mz;
  cov[8] = M.szz * inv - mz * mz;
  cov[3] = cov[1]; cov[6] = cov[2]; cov[7] = cov[5];
  double ev, v[3];
  eigen33_d(cov, &ev, v);
  const double tr = cov[0] + cov[4] + cov[8];
  const float curv = tr != 0.0 ? (float)fabs(ev / tr) : 0.0f;
  float nx = (float)v[0], ny = (float)v[1], nz = (float)v[2];
  // pcl::flipNormalTowardsViewpoint: vp -= p; if (vp.dot(n) < 0) n *= -1
  const float vx = vpx - qx, vy = vpy - qy, vz = vpz - qz;
  const float cos_theta = vx * nx + vy * ny + vz * nz;
  if (cos_theta < 0.0f) { nx *= -1.0f; ny *= -1.0f; nz *= -1.0f; }
  return make_float4(nx, ny, nz, curv);
}

// one thread per query, queries taken in sorted-cell order so a wavefront shares its cells
__global__ __launch_bounds__(kBS) void k_normals_radius(
    const float* __restrict__ sx, const float* __restrict__ sy, const float* __restrict__ sz,
    const int32_t* __restrict__ sidx, int n, GridDesc G, const uint32_t* __restrict__ tkeys,
    const int2* __restrict__ trange, uint32_t tmask, float r2, float vpx, float vpy, float vpz,
    float4* __restrict__ normals) {
  const int t = blockIdx.x * kBS + threadIdx.x;
  if (t >= n) return;
  const float qx = sx[t], qy = sy[t], qz = sz[t];
  Moments M;
  if (finite3(qx, qy, qz)) {
    const int cx = cell_of(qx, G.lo[0], G.inv_cell, G.g[0]);
    const int cy = cell_of(qy, G.lo[1], G.inv_cell, G.g[1]);
    const int cz = cell_of(qz, G.lo[2], G.inv_cell, G.g[2]);
    for (int z = max(cz - 1, 0); z <= min(cz + 1, G.g[2] - 1); ++z)
      for (int y = max(cy - 1, 0); y <= min(cy + 1, G.g[1] - 1); ++y)
        for (int x = max(cx - 1, 0); x <= min(cx + 1, G.g[0] - 1); ++x) {
          const int2 rg = cell_range(tkeys, trange, tmask, cell_key(G, x, y, z));
          for (int u = rg.x; u < rg.y; ++u) {
            const float px = sx[u], py = sy[u], pz = sz[u];
            if (flann_d2(qx, qy, qz, px, py, pz) < r2) M.add(px, py, pz, qx, qy, qz);
          }
        }
  }
  normals[sidx[t]] = finish_normal(M, qx, qy, qz, vpx, vpy, vpz);
}

// k nearest neighbours over a grid hierarchy (cell_l = 2^l * cell_0, the top level has <= 2 cells
// per axis).  At level l the 27 cells around the query hold every point closer than cell_l, so if
// at least K candidates have d2 < cell_l^2 their K smallest (d2, index) are exactly FLANN's kNN
// set (anything unvisited is farther, ties included).  Otherwise the query moves up a level; at
// the top level the 27 cells are the whole cloud and every candidate counts.  One launch per
// level over the queries still open (compacted), so the few sparse outliers that climb do not
// hold back the wavefronts of the surface points, which finish at level 0.
// Queries are taken in the level's own cell order (qpos = sorted positions at level l; nullptr =
// all), so the lanes of a wavefront scan the same cells; a deferred query is flagged at its
// sorted position of level l + 1 and the next pass compacts the flags in that order.
// ---- PCL-float normals: pcl::computePointNormal as PCL 1.8 evaluates it -------------------
// computeMeanAndCovarianceMatrix (float, single pass over the neighbour list in FLANN's (d2,
// index) order), solvePlaneParameters (pcl::eigen33 in float, curvature = |lambda0 / trace| in
// float), flipNormalTowardsViewpoint (float, left to right).  Bit-exact with the oracle's
// restatement (orc_estimate_normals / _knn).
__device__ __forceinline__ void pcl_accu_add(float* a, float x, float y, float z) {
  a[0] += x * x; a[1] += x * y; a[2] += x * z;
  a[3] += y * y; a[4] += y * z; a[5] += z * z;
  a[6] += x;     a[7] += y;     a[8] += z;
}

__device__ float4 finish_normal_pcl(float* a, int cnt, float qx, float qy, float qz, float vpx,
                                    float vpy, float vpz) {
  if (cnt < 3) {
    const float qnan = __builtin_nanf("");
    return make_float4(qnan, qnan, qnan, qnan);
  }
  const float cf = (float)(size_t)cnt;
  for (int k = 0; k < 9; ++k) a[k] = a[k] / cf;
  float cov[9];
  cov[0] = a[0] - a[6] * a[6];
  cov[1] = a[1] - a[6] * a[7];
  cov[2] = a[2] - a[6] * a[8];
  cov[4] = a[3] - a[7] * a[7];
  cov[5] = a[4] - a[7] * a[8];
  cov[8] = a[5] - a[8] * a[8];
  cov[3] = cov[1]; cov[6] = cov[2]; cov[7] = cov[5];
  float ev, v[3];
  eigen33<float>(cov, &ev, v);
  const float eig_sum = cov[0] + cov[4] + cov[8];
  const float curv = eig_sum != 0.0f ? fabsf(ev / eig_sum) : 0.0f;
  float nx = v[0], ny = v[1], nz = v[2];
  const float vx = vpx - qx, vy = vpy - qy, vz = vpz - qz;
  const float cos_theta = vx * nx + vy * ny + vz * nz;
  if (cos_theta < 0.0f) { nx *= -1.0f; ny *= -1.0f; nz *= -1.0f; }
  return make_float4(nx, ny, nz, curv);
}

// radius search, pass 1: neighbour counts per query (sorted positions [q0, q0 + nq))
__global__ __launch_bounds__(kBS) void k_nbr_count(
    const float* __restrict__ sx, const float* __restrict__ sy, const float* __restrict__ sz,
    int q0, int nq, GridDesc G, const uint32_t* __restrict__ tkeys,
    const int2* __restrict__ trange, uint32_t tmask, float r2, int32_t* __restrict__ cnt) {
  const int i = blockIdx.x * kBS + threadIdx.x;
  if (i >= nq) return;
  const int t = q0 + i;
  const float qx = sx[t], qy = sy[t], qz = sz[t];
  int c = 0;
  if (finite3(qx, qy, qz)) {
    const int cx = cell_of(qx, G.lo[0], G.inv_cell, G.g[0]);
    const int cy = cell_of(qy, G.lo[1], G.inv_cell, G.g[1]);
    const int cz = cell_of(qz, G.lo[2], G.inv_cell, G.g[2]);
    for (int z = max(cz - 1, 0); z <= min(cz + 1, G.g[2] - 1); ++z)
      for (int y = max(cy - 1, 0); y <= min(cy + 1, G.g[1] - 1); ++y)
        for (int x = max(cx - 1, 0); x <= min(cx + 1, G.g[0] - 1); ++x) {
          const int2 rg = cell_range(tkeys, trange, tmask, cell_key(G, x, y, z));
#pragma unroll 4  // (the cell's loads issued together)
          for (int u = rg.x; u < rg.y; ++u)
            c += flann_d2(qx, qy, qz, sx[u], sy[u], sz[u]) < r2 ? 1 : 0;
        }
  }
  cnt[i] = c;
}

// pass 2: the neighbours as 64-bit keys (d2 bits << 32 | point index: (d2, index) order) at the
// query's offset
__global__ __launch_bounds__(kBS) void k_nbr_fill(
    const float* __restrict__ sx, const float* __restrict__ sy, const float* __restrict__ sz,
    const int32_t* __restrict__ sidx, int q0, int nq, GridDesc G,
    const uint32_t* __restrict__ tkeys, const int2* __restrict__ trange, uint32_t tmask, float r2,
    const int64_t* __restrict__ off, uint64_t* __restrict__ keys) {
  const int i = blockIdx.x * kBS + threadIdx.x;
  if (i >= nq) return;
  const int t = q0 + i;
  const float qx = sx[t], qy = sy[t], qz = sz[t];
  if (!finite3(qx, qy, qz)) return;
  uint64_t* out = keys + off[i];
  int c = 0;
  const int cx = cell_of(qx, G.lo[0], G.inv_cell, G.g[0]);
  const int cy = cell_of(qy, G.lo[1], G.inv_cell, G.g[1]);
  const int cz = cell_of(qz, G.lo[2], G.inv_cell, G.g[2]);
  for (int z = max(cz - 1, 0); z <= min(cz + 1, G.g[2] - 1); ++z)
    for (int y = max(cy - 1, 0); y <= min(cy + 1, G.g[1] - 1); ++y)
      for (int x = max(cx - 1, 0); x <= min(cx + 1, G.g[0] - 1); ++x) {
        const int2 rg = cell_range(tkeys, trange, tmask, cell_key(G, x, y, z));
#pragma unroll 4
        for (int u = rg.x; u < rg.y; ++u) {
          const float d2 = flann_d2(qx, qy, qz, sx[u], sy[u], sz[u]);
          if (d2 < r2)
            out[c++] = ((uint64_t)__float_as_uint(d2) << 32) | (uint32_t)sidx[u];
        }
      }
}

// v of lane (lane ^ S), S < 64, without LDS: DPP quad permutes (S = 1, 2), quad reversal then
// half-row mirror (4: l ^ 3 mirrored in 8 lanes is l ^ 4), row rotate by 8 (8), and gfx950's
// row / half-wave swaps (16, 32: the swap of v with itself leaves each lane's partner in one of
// the two results).  The whole wave must be active.
template <int S>
__device__ __forceinline__ uint32_t xor_lane(uint32_t v) {
  if constexpr (S == 1) {
    return __builtin_amdgcn_update_dpp(0u, v, 0xB1, 0xF, 0xF, false);  // quad_perm [1,0,3,2]
  } else if constexpr (S == 2) {
    return __builtin_amdgcn_update_dpp(0u, v, 0x4E, 0xF, 0xF, false);  // quad_perm [2,3,0,1]
  } else if constexpr (S == 4) {
    const uint32_t r = __builtin_amdgcn_update_dpp(0u, v, 0x1B, 0xF, 0xF, false);  // [3,2,1,0]
    return __builtin_amdgcn_update_dpp(0u, r, 0x141, 0xF, 0xF, false);  // row_half_mirror
  } else if constexpr (S == 8) {
    return __builtin_amdgcn_update_dpp(0u, v, 0x128, 0xF, 0xF, false);  // row_ror:8
  } else if constexpr (S == 16) {
    const auto r = __builtin_amdgcn_permlane16_swap(v, v, false, false);
    return (threadIdx.x & 16) ? r[0] : r[1];
  } else {
    static_assert(S == 32, "xor_lane: S in 1..32");
    const auto r = __builtin_amdgcn_permlane32_swap(v, v, false, false);
    return (threadIdx.x & 32) ? r[0] : r[1];
  }
}

template <int S>
__device__ __forceinline__ uint64_t xor_lane64(uint64_t v) {
  return (uint64_t)xor_lane<S>((uint32_t)v) | ((uint64_t)xor_lane<S>((uint32_t)(v >> 32)) << 32);
}

// one bitonic merge step at in-wave distance S over the E registers (blocks of `size` elements)
template <int E, int S>
__device__ __forceinline__ void bitonic_xstep(uint64_t (&v)[E], int size) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int j = 0; j < E; ++j) {
    const int e = lane + 64 * j;
    const bool up = (e & size) == 0;  // this element's block sorts ascending
    const bool take_min = ((lane & S) == 0) == up;  // the lower element keeps the min ascending
    const uint64_t o = xor_lane64<S>(v[j]);
    v[j] = (o < v[j]) == take_min ? o : v[j];
  }
}

// bitonic sort of 64 * E keys held E per lane (element e = lane + 64 j), ascending; the steps
// within a wave exchange through DPP / lane swaps (no LDS round trip per step)
template <int E>
__device__ __forceinline__ void wave_bitonic(uint64_t (&v)[E]) {
#pragma unroll
  for (int size = 2; size <= 64 * E; size <<= 1) {
#pragma unroll
    for (int stride = size >> 1; stride >= 64; stride >>= 1) {
      const int js = stride >> 6;
#pragma unroll
      for (int j = 0; j < E; ++j) {
        if ((j & js) == 0) {  // (j, j | js): both in this lane
          const bool up = ((j * 64) & size) == 0;
          uint64_t& a = v[j];
          uint64_t& b = v[j | js];
          const bool sw = up ? (a > b) : (a < b);
          if (sw) { const uint64_t t = a; a = b; b = t; }
        }
      }
    }
    if (size >= 64) bitonic_xstep<E, 32>(v, size);
    if (size >= 32) bitonic_xstep<E, 16>(v, size);
    if (size >= 16) bitonic_xstep<E, 8>(v, size);
    if (size >= 8) bitonic_xstep<E, 4>(v, size);
    if (size >= 4) bitonic_xstep<E, 2>(v, size);
    bitonic_xstep<E, 1>(v, size);
  }
}

template <int E>
__device__ __forceinline__ void sort_segment(uint64_t* seg, int k) {
  const int lane = threadIdx.x & 63;
  uint64_t v[E];
#pragma unroll
  for (int j = 0; j < E; ++j) {
    const int e = lane + 64 * j;
    v[j] = e < k ? seg[e] : ~0ull;
  }
  wave_bitonic<E>(v);
#pragma unroll
  for (int j = 0; j < E; ++j) {
    const int e = lane + 64 * j;
    if (e < k) seg[e] = v[j];
  }
}

// in-place heapsort by one lane (segments longer than 1024 keys: rare)
__device__ void heap_sort(uint64_t* a, int64_t n) {
  auto sift = [&](int64_t i, int64_t m) {
    for (;;) {
      int64_t c = 2 * i + 1;
      if (c >= m) break;
      if (c + 1 < m && a[c + 1] > a[c]) ++c;
      if (a[i] >= a[c]) break;
      const uint64_t t = a[i]; a[i] = a[c]; a[c] = t;
      i = c;
    }
  };
  for (int64_t i = n / 2 - 1; i >= 0; --i) sift(i, n);
  for (int64_t m = n - 1; m > 0; --m) {
    const uint64_t t = a[0]; a[0] = a[m]; a[m] = t;
    sift(0, m);
  }
}

// pass 3: sort each query's keys (one wave per query)
__global__ __launch_bounds__(kBS) void k_nbr_sort(int nq, const int32_t* __restrict__ cnt,
                                                  const int64_t* __restrict__ off,
                                                  uint64_t* __restrict__ keys) {
  const int wv = (blockIdx.x * kBS + threadIdx.x) >> 6;
  const int nw = (gridDim.x * kBS) >> 6;
  for (int i = wv; i < nq; i += nw) {
    const int k = cnt[i];
    if (k < 2) continue;
    uint64_t* seg = keys + off[i];
    if (k <= 64) sort_segment<1>(seg, k);
    else if (k <= 128) sort_segment<2>(seg, k);
    else if (k <= 256) sort_segment<4>(seg, k);
    else if (k <= 512) sort_segment<8>(seg, k);
    else if (k <= 1024) sort_segment<16>(seg, k);
    else if ((threadIdx.x & 63) == 0) heap_sort(seg, k);
  }
}

// pass 4: PCL's sums over the sorted neighbours, one thread per query
__global__ __launch_bounds__(kBS) void k_nbr_normals(
    const float* __restrict__ sx, const float* __restrict__ sy, const float* __restrict__ sz,
    const int32_t* __restrict__ sidx, int q0, int nq, const int32_t* __restrict__ cnt,
    const int64_t* __restrict__ off, const uint64_t* __restrict__ keys,
    const float* __restrict__ X, const float* __restrict__ Y, const float* __restrict__ Z,
    float vpx, float vpy, float vpz, float4* __restrict__ normals) {
  const int i = blockIdx.x * kBS + threadIdx.x;
  if (i >= nq) return;
  const int t = q0 + i;
  const int k = cnt[i];
  float a[9] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  const uint64_t* seg = keys + off[i];
  // sixteen neighbours' keys, then their 48 coordinate gathers, issued before any is summed (the
  // gathers are random over the cloud: one key -> coordinates latency per 16 terms, not per term);
  // the sums still run in list order
  constexpr int kB = 16;
  int e = 0;
  for (; e + kB <= k; e += kB) {
    int j[kB];
#pragma unroll
    for (int u = 0; u < kB; ++u) j[u] = (int)(uint32_t)seg[e + u];
    float px[kB], py[kB], pz[kB];
#pragma unroll
    for (int u = 0; u < kB; ++u) { px[u] = X[j[u]]; py[u] = Y[j[u]]; pz[u] = Z[j[u]]; }
#pragma unroll
    for (int u = 0; u < kB; ++u) pcl_accu_add(a, px[u], py[u], pz[u]);
  }
  for (; e < k; ++e) {
    const int j = (int)(uint32_t)seg[e];
    pcl_accu_add(a, X[j], Y[j], Z[j]);
  }
  normals[sidx[t]] = finish_normal_pcl(a, k, sx[t], sy[t], sz[t], vpx, vpy, vpz);
}

// The 27 cells around cell (cx, cy, cz) as 9 rows of contiguous sorted positions (a row's three
// x cells have consecutive keys), packed into one candidate list: rows[r] = row r's start in the
// list, rows[9 + r] = its offset to sorted positions, rows[18] = the list's length.  The whole
// wave calls it; rows is the wave's LDS table.
// cell_done (RegulateNormal's claim pass): cells whose points are all settled are left out (a
// row keeps the union of its other cells; a settled middle cell stays inside it)
__device__ __forceinline__ void nbr_rows(const GridDesc& G, const uint32_t* __restrict__ tkeys,
                                         const int2* __restrict__ trange, uint32_t tmask, int cx,
                                         int cy, int cz, int32_t* rows,
                                         const uint32_t* __restrict__ cell_done = nullptr) {
  const int lane = threadIdx.x & 63;
  // lanes 0..26 look up one cell each; a row's range is its cells' union (contiguous)
  int2 c = make_int2(INT_MAX, INT_MIN);
  if (lane < 27) {
    const int x = cx + lane % 3 - 1, y = cy + (lane / 3) % 3 - 1, z = cz + lane / 9 - 1;
    if (x >= 0 && y >= 0 && z >= 0 && x < G.g[0] && y < G.g[1] && z < G.g[2]) {
      const int h = cell_slot(tkeys, tmask, cell_key(G, x, y, z));
      if (h >= 0) {
        const int2 r = trange[h];
        if (r.y > r.x && !(cell_done && cell_done[h] >= (uint32_t)(r.y - r.x))) c = r;
      }
    }
  }
  int lo = c.x, hi = c.y;
#pragma unroll
  for (int o = 1; o <= 2; o <<= 1) {  // (min / max over each aligned triple of lanes)
    const int l2 = __shfl(lo, (lane / 3) * 3 + ((lane % 3 + o) % 3), 64);
    const int h2 = __shfl(hi, (lane / 3) * 3 + ((lane % 3 + o) % 3), 64);
    lo = min(lo, l2);
    hi = max(hi, h2);
  }
  const int rl = __shfl(lo, 3 * (lane < 9 ? lane : 0), 64);
  const int rh = __shfl(hi, 3 * (lane < 9 ? lane : 0), 64);
  const int2 rg = lane < 9 && rl < rh ? make_int2(rl, rh) : make_int2(0, 0);
  const int rlen = rg.y - rg.x;
  int incl = rlen;  // (lanes 0..8: inclusive prefix of the row lengths)
#pragma unroll
  for (int o = 1; o < 16; o <<= 1) {
    const int w = __shfl_up(incl, o, 64);
    if (lane >= o) incl += w;
  }
  const int excl = incl - rlen;
  __builtin_amdgcn_wave_barrier();
  if (lane < 9) {
    rows[lane] = excl;
    rows[9 + lane] = rg.x - excl;
  }
  if (lane == 8) rows[18] = incl;
  __builtin_amdgcn_wave_barrier();
}

// the sorted position of packed candidate v (row tables read from nbr_rows' LDS table)
__device__ __forceinline__ int nbr_pos(const int (&r_start)[9], const int (&r_off)[9], int v) {
  int u = v + r_off[0];
#pragma unroll
  for (int q = 1; q < 9; ++q) u = v >= r_start[q] ? v + r_off[q] : u;
  return u;
}

// ---- fused radius normals (PCL float): search, (d2, index) order and the sums in one pass ----
// One wave per query at a time, queries taken in runs of kFqRun consecutive sorted positions.
// Per query: the 27 cells around it are 9 runs of sorted positions (a row's three x cells have
// consecutive keys, so their ranges are contiguous; looked up when the query's cell changes),
// packed into one candidate list scanned 64 per step with FLANN's d2 and test (the neighbour
// set is KdTreeFLANN's); the passing ones are compacted into the wave's LDS buffer as
// keys (d2 bits << 32 | sorted position), sorted in registers by a wave bitonic sized to the
// count (64, 128, 256, 512 ... keys), reordered by the points' original index where d2 ties
// (FLANN's (d2, index) order: sorted positions follow the original index only within a cell),
// and the neighbours' coordinates gathered from the sorted keys and staged over the same buffer as
// (x, y, z) triplets in that order; lanes 0..8 then run computeMeanAndCovarianceMatrix's nine
// float chains in list order (each lane reading its chain's two operands at its own offsets).
// The sums of 64 queries are parked in LDS and finished (eigen33, curvature, viewpoint flip)
// with one query per lane.  Nothing per neighbour leaves the chip (the chunked pipeline writes,
// sorts and re-reads 8 bytes per neighbour).  A query with more than 64 EMAX neighbours goes to
// the overflow list for the next, wider launch.  Every LDS access of the shared buffer is a
// 32-bit word access or a memcpy (the keys and the coordinates alias).
constexpr int kFqRun = 16;
constexpr int kFqB = 4;  // candidate steps whose loads are in flight together
#define DLG_NBR_FUSED_ARGS                                                                        \
    const float *__restrict__ sx, const float *__restrict__ sy, const float *__restrict__ sz,     \
        const int32_t *__restrict__ sidx, int n, const int32_t *__restrict__ qlist,              \
        const uint32_t *__restrict__ qcount, GridDesc G, const uint32_t *__restrict__ tkeys,     \
        const int2 *__restrict__ trange, uint32_t tmask, float r2, float vpx, float vpy,         \
        float vpz, float4 *__restrict__ normals, int32_t *__restrict__ ovf,                      \
        uint32_t *__restrict__ ovf_count
template <int EMAX>
__device__ __forceinline__ void nbr_fused_body(DLG_NBR_FUSED_ARGS);

// the first pass (<= 512 neighbours) held to 128 VGPRs: four waves per SIMD, as many as its LDS
// allows; the wider pass (<= 1024) is LDS-limited to fewer waves anyway
template <int EMAX>
__global__ __launch_bounds__(kBS) __attribute__((amdgpu_waves_per_eu(4))) void k_nbr_fused(
    DLG_NBR_FUSED_ARGS) {
  nbr_fused_body<EMAX>(sx, sy, sz, sidx, n, qlist, qcount, G, tkeys, trange, tmask, r2, vpx,
                           vpy, vpz, normals, ovf, ovf_count);
}
template <int EMAX>
__global__ __launch_bounds__(kBS) void k_nbr_fused_wide(DLG_NBR_FUSED_ARGS) {
  nbr_fused_body<EMAX>(sx, sy, sz, sidx, n, qlist, qcount, G, tkeys, trange, tmask, r2, vpx,
                          vpy, vpz, normals, ovf, ovf_count);
}

__device__ __forceinline__ uint64_t lds_key(const uint32_t* buf, int e) {
  uint64_t k;
  __builtin_memcpy(&k, buf + 2 * e, 8);
  return k;
}
__device__ __forceinline__ void lds_set_key(uint32_t* buf, int e, uint64_t k) {
  __builtin_memcpy(buf + 2 * e, &k, 8);
}

// the wave's cnt (<= 64 E) keys in buf -> FLANN's (d2, original index) order, then the
// neighbours' (x, y, z) staged over the keys in that order (word 3 e + axis)
template <int E>
__device__ __forceinline__ void nbr_order_stage(uint32_t* buf, int cnt,
                                                const float* __restrict__ sx,
                                                const float* __restrict__ sy,
                                                const float* __restrict__ sz,
                                                const int32_t* __restrict__ sidx) {
  const int lane = threadIdx.x & 63;
  uint64_t v[E];
#pragma unroll
  for (int j = 0; j < E; ++j) {
    const int e = lane + 64 * j;
    v[j] = e < cnt ? lds_key(buf, e) : ~0ull;
  }
  wave_bitonic<E>(v);
  // (d2, sorted position) -> FLANN's (d2, original index): only equal-d2 runs can differ
  bool tie = false;
#pragma unroll
  for (int j = 0; j < E; ++j) {
    const uint64_t nxt = __shfl_down(v[j], 1, 64);
    const uint64_t nxt2 = j + 1 < E ? __shfl(v[j + 1 < E ? j + 1 : j], 0, 64) : ~0ull;
    const uint64_t w = lane == 63 ? nxt2 : nxt;
    const int e = lane + 64 * j;
    tie |= e + 1 < cnt && (v[j] >> 32) == (w >> 32);
  }
  if (__ballot(tie)) {
    // in registers: the entries re-sorted by (their equal-d2 run's first entry, original index,
    // entry) -- 10 + 32 + 10 bits -- and the entry index then finds each one's (d2, sorted
    // position) key, parked in LDS by entry
    static_assert(E <= 16, "entry indices fit 10 bits");
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int j = 0; j < E; ++j) lds_set_key(buf, lane + 64 * j, v[j]);
    __builtin_amdgcn_wave_barrier();
    uint64_t nk[E];
    int carry = 0;
#pragma unroll
    for (int j = 0; j < E; ++j) {
      const int e = lane + 64 * j;
      const uint64_t prev = e > 0 ? lds_key(buf, e - 1) : ~0ull;
      int rs = (e == 0 || (prev >> 32) != (v[j] >> 32)) ? e : 0;  // (a run starts here)
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {  // inclusive max-scan over the lanes: the run's start
        const int t = __shfl_up(rs, o, 64);
        if (lane >= o) rs = max(rs, t);
      }
      rs = max(rs, carry);
      carry = __shfl(rs, 63, 64);
      const uint32_t oi = e < cnt ? (uint32_t)sidx[(uint32_t)v[j]] : 0u;
      nk[j] = e < cnt ? ((uint64_t)rs << 42) | ((uint64_t)oi << 10) | (uint64_t)e : ~0ull;
    }
    wave_bitonic<E>(nk);
#pragma unroll
    for (int j = 0; j < E; ++j) {
      const int e = lane + 64 * j;
      v[j] = e < cnt ? lds_key(buf, (int)(nk[j] & 1023u)) : ~0ull;
    }
  }
  float x[E], y[E], z[E];
#pragma unroll
  for (int j = 0; j < E; ++j) {  // (every gather issued before the stores)
    const uint32_t u = (uint32_t)v[j];
    const bool in = lane + 64 * j < cnt;
    x[j] = in ? sx[u] : 0.0f;
    y[j] = in ? sy[u] : 0.0f;
    z[j] = in ? sz[u] : 0.0f;
  }
  __builtin_amdgcn_wave_barrier();  // (the keys are read: the triplets overwrite them)
#pragma unroll
  for (int j = 0; j < E; ++j) {
    const int e = lane + 64 * j;
    if (e < cnt) {
      buf[3 * e] = __float_as_uint(x[j]);
      buf[3 * e + 1] = __float_as_uint(y[j]);
      buf[3 * e + 2] = __float_as_uint(z[j]);
    }
  }
  __builtin_amdgcn_wave_barrier();
}

template <int EMAX>
__device__ __forceinline__ void nbr_fused_body(DLG_NBR_FUSED_ARGS) {
  constexpr int kCap = 64 * EMAX;
  constexpr int kW = kBS / 64;
  __shared__ __attribute__((aligned(16))) uint32_t s_buf[kW][3 * kCap];  // keys, then (x, y, z)
  __shared__ float s_sum[kW][9][64];  // parked sums: [chain][slot]
  __shared__ float4 s_q[kW][64];      // (query xyz, count) per slot
  __shared__ int32_t s_dst[kW][64];   // output point index per slot
  // the 27 cells around the current cell as 9 rows of contiguous sorted positions: row r's
  // start in the packed candidate list [r], its offset to sorted positions [9 + r], the list's
  // length [18]
  __shared__ int32_t s_rows[kW][20];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  uint32_t* buf = s_buf[wv];
  int32_t* rows = s_rows[wv];
  // lane c < 9 runs chain c: term = pa * pb, the coordinate sums (pb = 1: x * 1 = x exactly)
  // selecting 1 in place of a second operand
  const int sa = lane < 3 ? 0 : lane < 5 ? 1 : lane < 6 ? 2 : lane - 6;
  const int sb = lane == 0 ? 0 : (lane == 1 || lane == 3) ? 1 : (lane == 2 || lane == 4 || lane == 5) ? 2 : 3;
  const bool one_b = sb == 3;
  const int ob = one_b ? 0 : sb;
  int parked = 0;
  auto finish = [&]() {  // the parked queries, one per lane
    __builtin_amdgcn_wave_barrier();
    if (lane < parked) {
      float a[9];
#pragma unroll
      for (int k = 0; k < 9; ++k) a[k] = s_sum[wv][k][lane];
      const float4 q = s_q[wv][lane];
      normals[s_dst[wv][lane]] = finish_normal_pcl(a, __float_as_int(q.w), q.x, q.y, q.z, vpx, vpy, vpz);
    }
    __builtin_amdgcn_wave_barrier();
    parked = 0;
  };
  const int nq = qlist ? (int)*qcount : n;
  const int nruns = (nq + kFqRun - 1) / kFqRun;
  const int gw = (int)((blockIdx.x * kBS + threadIdx.x) >> 6), nw = (int)((gridDim.x * kBS) >> 6);
  for (int run = gw; run < nruns; run += nw) {
    int pcx = -1, pcy = -1, pcz = -1;
    const int i_end = min(nq, (run + 1) * kFqRun);
    for (int i = run * kFqRun; i < i_end; ++i) {
      const int t = qlist ? qlist[i] : i;
      const float qx = sx[t], qy = sy[t], qz = sz[t];
      if (!finite3(qx, qy, qz)) {
        if (lane == 0) {
          const float qn = __builtin_nanf("");
          normals[sidx[t]] = make_float4(qn, qn, qn, qn);
        }
        continue;
      }
      const int cx = cell_of(qx, G.lo[0], G.inv_cell, G.g[0]);
      const int cy = cell_of(qy, G.lo[1], G.inv_cell, G.g[1]);
      const int cz = cell_of(qz, G.lo[2], G.inv_cell, G.g[2]);
      if (cx != pcx || cy != pcy || cz != pcz) {
        pcx = cx; pcy = cy; pcz = cz;
        // lanes 0..26 look up one cell each; a row's range is its cells' union (contiguous)
        int2 c = make_int2(INT_MAX, INT_MIN);
        if (lane < 27) {
          const int x = cx + lane % 3 - 1, y = cy + (lane / 3) % 3 - 1, z = cz + lane / 9 - 1;
          if (x >= 0 && y >= 0 && z >= 0 && x < G.g[0] && y < G.g[1] && z < G.g[2]) {
            const int2 r = cell_range(tkeys, trange, tmask, cell_key(G, x, y, z));
            if (r.y > r.x) c = r;
          }
        }
        int lo = c.x, hi = c.y;
#pragma unroll
        for (int o = 1; o <= 2; o <<= 1) {  // (min / max over each aligned triple of lanes)
          const int l2 = __shfl(lo, (lane / 3) * 3 + ((lane % 3 + o) % 3), 64);
          const int h2 = __shfl(hi, (lane / 3) * 3 + ((lane % 3 + o) % 3), 64);
          lo = min(lo, l2);
          hi = max(hi, h2);
        }
        const int rl = __shfl(lo, 3 * (lane < 9 ? lane : 0), 64);
        const int rh = __shfl(hi, 3 * (lane < 9 ? lane : 0), 64);
        const int2 rg = lane < 9 && rl < rh ? make_int2(rl, rh) : make_int2(0, 0);
        const int rlen = rg.y - rg.x;
        int incl = rlen;  // (lanes 0..8: inclusive prefix of the row lengths)
#pragma unroll
        for (int o = 1; o < 16; o <<= 1) {
          const int w = __shfl_up(incl, o, 64);
          if (lane >= o) incl += w;
        }
        const int excl = incl - rlen;
        __builtin_amdgcn_wave_barrier();
        if (lane < 9) {
          rows[lane] = excl;
          rows[9 + lane] = rg.x - excl;
        }
        if (lane == 8) rows[18] = incl;
        __builtin_amdgcn_wave_barrier();
      }
      // (re-read per query: live only during the scan)
      int r_start[9], r_off[9];
#pragma unroll
      for (int q = 0; q < 9; ++q) {
        r_start[q] = rows[q];
        r_off[q] = rows[9 + q];
      }
      const int tot = rows[18];
      // the 9 rows' candidates as one packed list: position v of the list lies in row r, the
      // last row whose start P_r <= v, at sorted position v + (begin_r - P_r); row starts and
      // offsets are wave-uniform (scalars), recomputed when the query's cell changes.  64
      // positions per step, kFqB steps with their loads in flight together.
      int cnt = 0;
      for (int k0 = 0; k0 < tot; k0 += 64 * kFqB) {
        float d2[kFqB];
        int uu[kFqB];
#pragma unroll
        for (int j = 0; j < kFqB; ++j) {
          const int v = k0 + 64 * j + lane;
          int u = v + r_off[0];
#pragma unroll
          for (int q = 1; q < 9; ++q) u = v >= r_start[q] ? v + r_off[q] : u;
          uu[j] = u;
          d2[j] = INFINITY;
          if (v < tot) d2[j] = flann_d2(qx, qy, qz, sx[u], sy[u], sz[u]);
        }
#pragma unroll
        for (int j = 0; j < kFqB; ++j) {
          const bool in = d2[j] < r2;
          const uint64_t m = __ballot(in);
          const int p = cnt + __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32),
                                                        __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
          if (in && p < kCap)
            lds_set_key(buf, p, ((uint64_t)__float_as_uint(d2[j]) << 32) | (uint32_t)uu[j]);
          cnt += (int)__popcll(m);
        }
      }
      if (cnt > kCap) {  // (too many neighbours for this instantiation)
        if (lane == 0) ovf[atomicAdd(ovf_count, 1u)] = t;
        continue;
      }
      __builtin_amdgcn_wave_barrier();
      if (cnt <= 64) nbr_order_stage<1>(buf, cnt, sx, sy, sz, sidx);
      else if (cnt <= 128) nbr_order_stage<2>(buf, cnt, sx, sy, sz, sidx);
      else if (cnt <= 256 || EMAX < 8) nbr_order_stage<(EMAX < 4 ? EMAX : 4)>(buf, cnt, sx, sy, sz, sidx);
      else if (cnt <= 512 || EMAX < 16) nbr_order_stage<(EMAX < 8 ? EMAX : 8)>(buf, cnt, sx, sy, sz, sidx);
      else nbr_order_stage<EMAX>(buf, cnt, sx, sy, sz, sidx);
      // the nine chains, one per lane, in list order (PCL: accu[k] += term, float)
      float acc = 0.0f;
      if (lane < 9) {
        const uint32_t* ra = buf + sa;
        const uint32_t* rb = buf + ob;
#pragma unroll 8
        for (int e = 0; e < cnt; ++e) {
          const float pa = __uint_as_float(ra[3 * e]);
          const float pb = one_b ? 1.0f : __uint_as_float(rb[3 * e]);
          acc = acc + pa * pb;
        }
        s_sum[wv][lane][parked] = acc;
      }
      if (lane == 0) {
        s_q[wv][parked] = make_float4(qx, qy, qz, __int_as_float(cnt));
        s_dst[wv][parked] = sidx[t];
      }
      __builtin_amdgcn_wave_barrier();  // (the next query's keys overwrite the triplets)
      if (++parked == 64) finish();
    }
  }
  if (parked) finish();
}

constexpr int kKnnCap = 32;  // level 0: buffered candidates per query
template <int KP, bool PCLF, bool L0>
__global__ __launch_bounds__(kBS) void k_normals_knn(
    KnnLevels L, int l, const int32_t* __restrict__ qpos, int nq, const float* __restrict__ X,
    const float* __restrict__ Y, const float* __restrict__ Z, int K, float vpx, float vpy,
    float vpz, float4* __restrict__ normals, uint8_t* __restrict__ dflags, int64_t dstride,
    int lmax) {
  __shared__ uint32_t s_hist[L0 ? 8 : 1][kBS];        // level 0: 16 d2 buckets (16-bit halves)
  __shared__ int32_t s_buf[L0 ? kKnnCap : 1][kBS];    // level 0: the candidates of buckets <= B
  const int t = blockIdx.x * kBS + threadIdx.x;
  if (t >= nq) return;
  const int uq = qpos ? qpos[t] : t;
  const int qi = L.idx[l][uq];
  const float qx = L.sx[l][uq], qy = L.sy[l][uq], qz = L.sz[l][uq];
  const bool active = true;
  Moments M;
  bool defer = false;
  int jump = 1;  // levels up a deferred query goes
  if (active && finite3(qx, qy, qz)) {
    const GridDesc& G = L.G[l];
    const bool top = l == L.levels - 1;
    const float lim = top ? INFINITY : G.cell * G.cell;
    const float* __restrict__ sx = L.sx[l];
    const float* __restrict__ sy = L.sy[l];
    const float* __restrict__ sz = L.sz[l];
    const int32_t* __restrict__ sidx = L.idx[l];
    // the KP smallest (d2, index) so far, ascending, in registers (fully unrolled network)
    float bd[KP];
    int bi[KP];
#pragma unroll
    for (int j = 0; j < KP; ++j) { bd[j] = INFINITY; bi[j] = INT_MAX; }
    float kd = INFINITY;  // current K-th entry: the admission bound
    int ki = INT_MAX;
    int cnt = 0;          // candidates inside the level's guaranteed radius
    const int cx = cell_of(qx, G.lo[0], G.inv_cell, G.g[0]);
    const int cy = cell_of(qy, G.lo[1], G.inv_cell, G.g[1]);
    const int cz = cell_of(qz, G.lo[2], G.inv_cell, G.g[2]);
    // The 27 cells nearest first (own cell, faces, edges, corners); a cell is skipped when a
    // lower bound of its distance to the query reaches the radius, or exceeds the current K-th
    // distance once K candidates are held (then its candidates could neither count nor enter).
    // Per axis the bound is the query's distance to the shared cell face in units of the index
    // map's cell width, less 1e-4 of a cell for the map's rounding, and the squared sum is
    // scaled by (1 - 1e-5) before the compare (FLANN's d2 rounding): never above a point's d2.
    const float w = 1.0f / G.inv_cell;
    const float fx = (qx - G.lo[0]) * G.inv_cell - (float)cx;
    const float fy = (qy - G.lo[1]) * G.inv_cell - (float)cy;
    const float fz = (qz - G.lo[2]) * G.inv_cell - (float)cz;
    auto side = [&](float f, int d) {  // distance bound to the neighbour on side d, cell units
      const float v = d < 0 ? f : d > 0 ? 1.0f - f : 0.0f;
      return v > 1e-4f ? (v - 1e-4f) * w : 0.0f;
    };
    const float bx0 = side(fx, -1), bx1 = side(fx, 1), by0 = side(fy, -1), by1 = side(fy, 1);
    const float bz0 = side(fz, -1), bz1 = side(fz, 1);
    constexpr uint64_t kOrd[3] = {0x904416665151515ull, 0x1a9864a9261058ull, 0x2a2a20a8220ull};
    // cells nearest first, each skipped when its distance bound md fails keep(md)
    auto scan = [&](auto&& keep, auto&& visit) {
#pragma unroll 1
      for (int c3 = 0; c3 < 27; ++c3) {
        const uint32_t code = (uint32_t)(kOrd[c3 / 10] >> (6 * (c3 % 10))) & 63u;
        const int dx = (int)(code & 3u) - 1, dy = (int)((code >> 2) & 3u) - 1,
                  dz = (int)((code >> 4) & 3u) - 1;
        const int x = cx + dx, y = cy + dy, z = cz + dz;
        if (x < 0 || x >= G.g[0] || y < 0 || y >= G.g[1] || z < 0 || z >= G.g[2]) continue;
        const float ex = dx < 0 ? bx0 : dx > 0 ? bx1 : 0.0f;
        const float ey = dy < 0 ? by0 : dy > 0 ? by1 : 0.0f;
        const float ez = dz < 0 ? bz0 : dz > 0 ? bz1 : 0.0f;
        const float md = (ex * ex + ey * ey + ez * ez) * (1.0f - 1e-5f);
        if (md >= lim || !keep(md)) continue;
        const int2 rg = cell_range(L.tkeys[l], L.trange[l], L.tmask[l], cell_key(G, x, y, z));
        for (int u = rg.x; u < rg.y; ++u) visit(u, flann_d2(qx, qy, qz, sx[u], sy[u], sz[u]));
      }
    };
    auto insert = [&](float cd, int ci) {
      if (cd > kd || (cd == kd && ci > ki)) return;
#pragma unroll
      for (int j = 0; j < KP; ++j) {
        const bool lt = cd < bd[j] || (cd == bd[j] && ci < bi[j]);
        const float od = bd[j];
        const int oi = bi[j];
        bd[j] = lt ? cd : od;
        bi[j] = lt ? ci : oi;
        cd = lt ? od : cd;
        ci = lt ? oi : ci;
      }
#pragma unroll
      for (int j = 0; j < KP; ++j)
        if (j == K - 1) { kd = bd[j]; ki = bi[j]; }
    };
    bool direct = true;
    int B = 15;
    const float inv = L0 ? 16.0f / lim : 0.0f;
    auto bucket = [&](float d2) { const int bb = (int)(d2 * inv); return bb < 15 ? bb : 15; };
    if constexpr (L0) {
      // Level 0 (most queries): inside the scan the insertion network runs whenever any lane of
      // the wave admits a candidate, i.e. at nearly every one.  Instead (1) count the candidates
      // inside the radius in 16 buckets of d2 (LDS, 16-bit halves); (2) the first bucket B where
      // the count reaches K bounds the K-th distance: the candidates of buckets <= B (about K)
      // are buffered in LDS; (3) the network runs over the buffer only.  A bucket too dense for
      // the buffer takes the network inside the scan.
#pragma unroll
      for (int q = 0; q < 8; ++q) s_hist[q][threadIdx.x] = 0u;
      scan([](float) { return true; }, [&](int, float d2) {
        if (!(d2 < lim)) return;
        ++cnt;
        const int bb = bucket(d2);
        atomicAdd(&s_hist[bb >> 1][threadIdx.x], 1u << (16 * (bb & 1)));
      });
      direct = false;
      if (cnt >= K) {
        int cum = 0;
        for (int bb = 0; bb < 16; ++bb) {
          cum += (int)((s_hist[bb >> 1][threadIdx.x] >> (16 * (bb & 1))) & 0xFFFFu);
          if (cum >= K) { B = bb; break; }
        }
        // (a cell whose bound puts every candidate past bucket B: skipped)
        const float bmax = (float)(B + 1) * 1.0001f;
        int nb = 0;
        scan([&](float md) { return md * inv < bmax; }, [&](int u, float d2) {
          if (!(d2 < lim) || bucket(d2) > B) return;
          if (nb < kKnnCap) s_buf[nb][threadIdx.x] = u;
          ++nb;
        });
        if (nb <= kKnnCap) {
          for (int e = 0; e < nb; ++e) {
            const int u = s_buf[e][threadIdx.x];
            insert(flann_d2(qx, qy, qz, sx[u], sy[u], sz[u]), sidx[u]);
          }
        } else {
          direct = true;
        }
      }
    }
    if (direct) {
      scan([&](float md) { return !(md > kd); }, [&](int u, float d2) {
        if (!(d2 < lim)) return;
        if (!L0) ++cnt;
        if (!L0 || bucket(d2) <= B) insert(d2, sidx[u]);
      });
    }
    defer = cnt < K && !top;
    // (level 0, fewer than K/4 candidates: the radius holding K is more than twice this level's
    // on a surface, so level 1 would nearly always defer it again -- it goes to level 2.  Only
    // from level 0: above it the sparse queries are volume-like outliers, many of which level
    // l + 1 resolves, and a query scanned a level too coarse costs ~4x the candidates)
    if (L0 && cnt > 0 && cnt * 4 < K && l + 2 < L.levels - 1) jump = 2;
    // (level 0, fewer than K / 4 candidates: volume-like outliers, which C5's clouds resolve
    // three levels up -- level 2 deferred 86 % of the queries sent there to level 3, and the few
    // it kept cost a level build of ~1.1 ms)
    if (L0 && cnt * 4 < K && l + 3 < L.levels - 1) jump = 3;
    if (!defer) {
      const int m = cnt < K ? cnt : K;
      if constexpr (PCLF) {
        // PCL: float sums over the kNN list in (d2, index) order
        float a[9] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int j = 0; j < KP; ++j)
          if (j < m) {
            const int i = bi[j];
            pcl_accu_add(a, X[i], Y[i], Z[i]);
          }
        normals[qi] = finish_normal_pcl(a, m, qx, qy, qz, vpx, vpy, vpz);
        return;
      }
#pragma unroll
      for (int j = 0; j < KP; ++j)
        if (j < m) {
          const int i = bi[j];
          M.add(X[i], Y[i], Z[i], qx, qy, qz);
        }
    }
  }
  if (defer) {
    const int tl = l + jump < lmax ? l + jump : lmax;
    dflags[(int64_t)tl * dstride + qi] = 1;
  }
  else normals[qi] = PCLF ? finish_normal_pcl(nullptr, 0, qx, qy, qz, vpx, vpy, vpz)
                          : finish_normal(M, qx, qy, qz, vpx, vpy, vpz);
}

// The deferred levels (l > 0: mostly outliers, whose coarse cells can hold a plane's thousands of
// points): one WAVE per query instead of one lane.  The 27 cells are visited in k_normals_knn's
// order with its bounds; lanes take a cell's candidates 64 at a time (coalesced loads), and the
// admitted ones -- d2 < the level's radius and (d2, index) below the current K-th -- are merged
// into the wave's best keys (d2 bits << 32 | original index, lane j = the j-th) by a 128-key
// bitonic sort.  Same counts, same (d2, index) order, same K-th bound for skipping cells, so the
// same neighbour lists, deferrals and sums as the one-lane scan, whose wave waited for the lane
// with the densest cells.
// the normal from the wave's m best keys: lane j loads neighbour j (all at once), then the sums
// run over the list in (d2, index) order from registers (readlane), uniform in every lane; lane
// 0 stores
template <bool PCLF>
__device__ __forceinline__ void knn_finish(uint64_t best, int m, const float* __restrict__ X,
                                           const float* __restrict__ Y,
                                           const float* __restrict__ Z, float qx, float qy,
                                           float qz, float vpx, float vpy, float vpz,
                                           float4* __restrict__ out) {
  const int lane = threadIdx.x & 63;
  const int i = lane < m ? (int)(uint32_t)best : 0;
  const float x = X[i], y = Y[i], z = Z[i];
  auto rl = [](float v, int j) {
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), j));
  };
  if constexpr (PCLF) {
    float acc[9] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll 1
    for (int j = 0; j < m; ++j) pcl_accu_add(acc, rl(x, j), rl(y, j), rl(z, j));
    if (lane == 0) *out = finish_normal_pcl(acc, m, qx, qy, qz, vpx, vpy, vpz);
  } else {
    Moments M;
#pragma unroll 1
    for (int j = 0; j < m; ++j) M.add(rl(x, j), rl(y, j), rl(z, j), qx, qy, qz);
    if (lane == 0) *out = finish_normal(M, qx, qy, qz, vpx, vpy, vpz);
  }
}

constexpr int kKwB = 4;    // k_normals_knn_wave: candidate batches in flight
constexpr int kKwIns = 6;  // ... admitted candidates of a batch inserted one by one (more: a merge)

// one batch of 64 candidate keys (d2 bits << 32 | original index; ~0: none) into the wave's
// ascending best keys (lane j: the j-th) under the bound kth (the K-th best so far)
__device__ __forceinline__ void knn_admit(uint64_t key, int K, uint64_t& best, uint64_t& kth) {
  const int lane = threadIdx.x & 63;
  const bool adm = key < kth;
  uint64_t am = __ballot(adm);
  if (__popcll(am) > kKwIns) {  // many: one 128-key bitonic merge
    uint64_t v[2] = {best, adm ? key : ~0ull};
    wave_bitonic<2>(v);
    best = v[0];
    kth = __shfl(best, K - 1, 64);
  } else {
    while (am) {  // few: each inserted in place (rank by ballot, lanes above shift up)
      const int src = __builtin_ctzll(am);
      am &= am - 1;
      const uint64_t kv =
          ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(key >> 32), src) << 32) |
          (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)key, src);
      if (!(kv < kth)) continue;  // (uniform: the earlier insertions raised the bar)
      const int pos = (int)__popcll(__ballot(best < kv));
      const uint64_t up = __shfl_up(best, 1, 64);
      best = lane < pos ? best : lane == pos ? kv : up;
      kth = __shfl(best, K - 1, 64);
    }
  }
}
template <int KP, bool PCLF>
__global__ __launch_bounds__(kBS) void k_normals_knn_wave(
    KnnLevels L, int l, const int32_t* __restrict__ qpos, int nq, const float* __restrict__ X,
    const float* __restrict__ Y, const float* __restrict__ Z, int K, float vpx, float vpy,
    float vpz, float4* __restrict__ normals, uint8_t* __restrict__ dflags, int64_t dstride,
    int lmax) {
  static_assert(KP <= 64, "the K best live one per lane");
  const int lane = threadIdx.x & 63;
  const int wq = __builtin_amdgcn_readfirstlane((int)((blockIdx.x * kBS + threadIdx.x) >> 6));
  if (wq >= nq) return;
  const int uq = qpos ? qpos[wq] : wq;
  const int qi = L.idx[l][uq];
  const float qx = L.sx[l][uq], qy = L.sy[l][uq], qz = L.sz[l][uq];
  if (!finite3(qx, qy, qz)) {
    if (lane == 0) {
      Moments M;
      normals[qi] = PCLF ? finish_normal_pcl(nullptr, 0, qx, qy, qz, vpx, vpy, vpz)
                         : finish_normal(M, qx, qy, qz, vpx, vpy, vpz);
    }
    return;
  }
  const GridDesc& G = L.G[l];
  const bool top = l == L.levels - 1;
  const float lim = top ? INFINITY : G.cell * G.cell;
  const float* __restrict__ sx = L.sx[l];
  const float* __restrict__ sy = L.sy[l];
  const float* __restrict__ sz = L.sz[l];
  const int32_t* __restrict__ sidx = L.idx[l];
  uint64_t best = ~0ull;  // lane j: the j-th smallest key so far
  uint64_t kth = ~0ull;   // (uniform) the K-th smallest: the admission bound
  int cnt = 0;            // (uniform) candidates inside the level's guaranteed radius
  const int cx = cell_of(qx, G.lo[0], G.inv_cell, G.g[0]);
  const int cy = cell_of(qy, G.lo[1], G.inv_cell, G.g[1]);
  const int cz = cell_of(qz, G.lo[2], G.inv_cell, G.g[2]);
  const float w = 1.0f / G.inv_cell;
  const float fx = (qx - G.lo[0]) * G.inv_cell - (float)cx;
  const float fy = (qy - G.lo[1]) * G.inv_cell - (float)cy;
  const float fz = (qz - G.lo[2]) * G.inv_cell - (float)cz;
  auto side = [&](float f, int d) {
    const float v = d < 0 ? f : d > 0 ? 1.0f - f : 0.0f;
    return v > 1e-4f ? (v - 1e-4f) * w : 0.0f;
  };
  const float bx0 = side(fx, -1), bx1 = side(fx, 1), by0 = side(fy, -1), by1 = side(fy, 1);
  const float bz0 = side(fz, -1), bz1 = side(fz, 1);
  constexpr uint64_t kOrd[3] = {0x904416665151515ull, 0x1a9864a9261058ull, 0x2a2a20a8220ull};
#pragma unroll 1
  for (int c3 = 0; c3 < 27; ++c3) {
    const uint32_t code = (uint32_t)(kOrd[c3 / 10] >> (6 * (c3 % 10))) & 63u;
    const int dx = (int)(code & 3u) - 1, dy = (int)((code >> 2) & 3u) - 1,
              dz = (int)((code >> 4) & 3u) - 1;
    const int x = cx + dx, y = cy + dy, z = cz + dz;
    if (x < 0 || x >= G.g[0] || y < 0 || y >= G.g[1] || z < 0 || z >= G.g[2]) continue;
    const float ex = dx < 0 ? bx0 : dx > 0 ? bx1 : 0.0f;
    const float ey = dy < 0 ? by0 : dy > 0 ? by1 : 0.0f;
    const float ez = dz < 0 ? bz0 : dz > 0 ? bz1 : 0.0f;
    const float md = (ex * ex + ey * ey + ez * ez) * (1.0f - 1e-5f);
    const float kd = __uint_as_float((uint32_t)(kth >> 32));  // (+inf bits... NaN until K held)
    if (md >= lim || (kth != ~0ull && md > kd)) continue;
    const int2 rg = cell_range(L.tkeys[l], L.trange[l], L.tmask[l], cell_key(G, x, y, z));
    const int a = __builtin_amdgcn_readfirstlane(rg.x), b = __builtin_amdgcn_readfirstlane(rg.y);
    // kKwB batches of 64 candidates per step, every load issued before the first d2 (a cell of
    // a coarse level holds hundreds of a plane's points: the steps are latency-bound)
#pragma unroll 1
    for (int u0 = a; u0 < b; u0 += 64 * kKwB) {
      float px[kKwB], py[kKwB], pz[kKwB];
      int32_t pi[kKwB];
#pragma unroll
      for (int j = 0; j < kKwB; ++j) {
        const int u = u0 + 64 * j + lane;
        const bool valid = u < b;
        px[j] = valid ? sx[u] : INFINITY;
        py[j] = valid ? sy[u] : 0.0f;
        pz[j] = valid ? sz[u] : 0.0f;
        pi[j] = valid ? sidx[u] : 0;
      }
#pragma unroll
      for (int j = 0; j < kKwB; ++j) {
        const float d2 = flann_d2(qx, qy, qz, px[j], py[j], pz[j]);  // (+inf past the end)
        const bool in = d2 < lim;
        cnt += (int)__popcll(__ballot(in));
        const uint64_t key = in ? ((uint64_t)__float_as_uint(d2) << 32) | (uint32_t)pi[j] : ~0ull;
        knn_admit(key, K, best, kth);
      }
    }
  }
  const bool defer = cnt < K && !top;
  if (defer) {
    const int tl = lmax;  // (the launch passes the level deferrals go to)
    if (lane == 0) dflags[(int64_t)tl * dstride + qi] = 1;
    return;
  }
  knn_finish<PCLF>(best, cnt < K ? cnt : K, X, Y, Z, qx, qy, qz, vpx, vpy, vpz, normals + qi);
}

__global__ __launch_bounds__(kBS) void k_inverse_perm(const int32_t* __restrict__ idx, int n,
                                                      int32_t* __restrict__ pos_of) {
  const int u = blockIdx.x * kBS + threadIdx.x;
  if (u < n) pos_of[idx[u]] = u;
}

// nearest neighbour of external queries over the grid hierarchy (same level rule as
// k_normals_knn with K = 1); a non-finite query gets nn = -1
__global__ __launch_bounds__(kBS) void k_nn1(KnnLevels L, int l, const int32_t* __restrict__ qlist,
                                             int nq, const float* __restrict__ QX,
                                             const float* __restrict__ QY,
                                             const float* __restrict__ QZ,
                                             int32_t* __restrict__ nn, int32_t* __restrict__ next,
                                             uint32_t* __restrict__ n_next) {
  const int t = blockIdx.x * kBS + threadIdx.x;
  const bool active = t < nq;
  const int qi = active ? (qlist ? qlist[t] : t) : 0;
  const float qx = active ? QX[qi] : 0.0f, qy = active ? QY[qi] : 0.0f,
              qz = active ? QZ[qi] : 0.0f;
  const bool ok = active && finite3(qx, qy, qz);
  if (active && !ok) nn[qi] = -1;
  const GridDesc& G = L.G[l];
  const bool top = l == L.levels - 1;
  const float lim = top ? INFINITY : G.cell * G.cell;
  float bd = INFINITY;
  int bi = INT_MAX;
  const int cx = cell_of(qx, G.lo[0], G.inv_cell, G.g[0]);
  const int cy = cell_of(qy, G.lo[1], G.inv_cell, G.g[1]);
  const int cz = cell_of(qz, G.lo[2], G.inv_cell, G.g[2]);
  if (ok)
  for (int z = max(cz - 1, 0); z <= min(cz + 1, G.g[2] - 1); ++z)
    for (int y = max(cy - 1, 0); y <= min(cy + 1, G.g[1] - 1); ++y)
      for (int x = max(cx - 1, 0); x <= min(cx + 1, G.g[0] - 1); ++x) {
        const int2 rg = cell_range(L.tkeys[l], L.trange[l], L.tmask[l], cell_key(G, x, y, z));
        for (int u = rg.x; u < rg.y; ++u) {
          const float d2 = flann_d2(qx, qy, qz, L.sx[l][u], L.sy[l][u], L.sz[l][u]);
          if (!(d2 < lim) || d2 > bd) continue;
          const int iu = L.idx[l][u];
          if (d2 < bd || iu < bi) { bd = d2; bi = iu; }
        }
      }
  const bool defer = ok && bi == INT_MAX && !top;
  wave_append(defer, qi, next, n_next);
  if (ok && !defer) nn[qi] = bi == INT_MAX ? -1 : bi;
}

// PlaneDetect.h:565-578: Eigen Vector3f dot (not vectorised: (a0 b0 + a1 b1) + a2 b2)
__global__ __launch_bounds__(kBS) void k_flip_to_reference(float* __restrict__ nrm, int64_t stride,
                                                           const float* __restrict__ ref,
                                                           int64_t ref_stride,
                                                           const int32_t* __restrict__ nn, int n) {
  const int i = blockIdx.x * kBS + threadIdx.x;
  if (i >= n) return;
  const int j = nn[i];
  if (j < 0) return;
  float* a = nrm + (int64_t)i * stride;
  const float* b = ref + (int64_t)j * ref_stride;
  const float d = (a[0] * b[0] + a[1] * b[1]) + a[2] * b[2];
  if (d < 0.0f) {
    a[0] *= -1.0f; a[1] *= -1.0f; a[2] *= -1.0f;
  }
}

// ---------------------------------------------------------------------------------------------
// preProcess() (PlaneDetect.h:448-512): NaN removal, translation to the centroid, and the greedy
// redundancy removal -- keep i unless an already kept j < i lies within min_dist -- which is the
// lexicographically-first maximal independent set of the radius graph in index order.

__global__ __launch_bounds__(kBS) void k_finite_flags(const float* __restrict__ X,
                                                      const float* __restrict__ Y,
                                                      const float* __restrict__ Z, int n,
                                                      uint8_t* __restrict__ flags) {
  const int i = blockIdx.x * kBS + threadIdx.x;
  if (i < n) flags[i] = finite3(X[i], Y[i], Z[i]) ? 1 : 0;
}

__global__ __launch_bounds__(kBS) void k_gather3(const int32_t* __restrict__ src, int n,
                                                 const float* __restrict__ X,
                                                 const float* __restrict__ Y,
                                                 const float* __restrict__ Z,
                                                 float* __restrict__ OX, float* __restrict__ OY,
                                                 float* __restrict__ OZ) {
  const int i = blockIdx.x * kBS + threadIdx.x;
  if (i >= n) return;
  const int j = src[i];
  OX[i] = X[j];
  OY[i] = Y[j];
  OZ[i] = Z[j];
}

// the reference's centroid (PlaneDetect.h:463-471): the three sequential float sums (fsum's
// chains 6-8, exact in parallel) divided by float(n), correctly rounded as on the host
__global__ void k_centroid_div(const float* __restrict__ sums3, int n, float* __restrict__ out) {
  const int k = threadIdx.x;
  if (k < 3) out[k] = sums3[k] / (float)n;
}

__global__ __launch_bounds__(kBS) void k_translate(float* __restrict__ X, float* __restrict__ Y,
                                                   float* __restrict__ Z, int n,
                                                   const float* __restrict__ p) {
  const int i = blockIdx.x * kBS + threadIdx.x;
  if (i >= n) return;
  X[i] -= p[0];
  Y[i] -= p[1];
  Z[i] -= p[2];
}

// one round of the index-ordered MIS over the sorted positions still undecided (state 0):
// kept (1) iff every lower-index neighbour is removed, removed (2) as soon as one is kept
__global__ __launch_bounds__(kBS) void k_mis_round(
    const int32_t* __restrict__ qlist, int nq, const float* __restrict__ sx,
    const float* __restrict__ sy, const float* __restrict__ sz, const int32_t* __restrict__ sidx,
    GridDesc G, const uint32_t* __restrict__ tkeys, const int2* __restrict__ trange,
    uint32_t tmask, float r2, uint8_t* state, int32_t* __restrict__ next,
    uint32_t* __restrict__ n_next) {
  const int t = blockIdx.x * kBS + threadIdx.x;
  const bool active = t < nq;
  const int u = active ? (qlist ? qlist[t] : t) : 0;
  const int j = active ? sidx[u] : 0;
  const float qx = active ? sx[u] : 0.0f, qy = active ? sy[u] : 0.0f, qz = active ? sz[u] : 0.0f;
  bool kept_nb = !active, all_removed = true;
  const int cx = cell_of(qx, G.lo[0], G.inv_cell, G.g[0]);
  const int cy = cell_of(qy, G.lo[1], G.inv_cell, G.g[1]);
  const int cz = cell_of(qz, G.lo[2], G.inv_cell, G.g[2]);
  for (int z = max(cz - 1, 0); z <= min(cz + 1, G.g[2] - 1) && !kept_nb; ++z)
    for (int y = max(cy - 1, 0); y <= min(cy + 1, G.g[1] - 1) && !kept_nb; ++y)
      for (int x = max(cx - 1, 0); x <= min(cx + 1, G.g[0] - 1) && !kept_nb; ++x) {
        const int2 rg = cell_range(tkeys, trange, tmask, cell_key(G, x, y, z));
        // four cell points' (immutable) index and coordinates loaded together; the state of a
        // lower-index neighbour is read as before, one candidate at a time
        for (int v0 = rg.x; v0 < rg.y && !kept_nb; v0 += 4) {
          int ci[4];
          float px[4], py[4], pz[4];
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            const int v = min(v0 + k, rg.y - 1);
            ci[k] = sidx[v]; px[k] = sx[v]; py[k] = sy[v]; pz[k] = sz[v];
          }
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            const int v = v0 + k;
            if (kept_nb || v >= rg.y || ci[k] >= j) continue;
            if (!(flann_d2(qx, qy, qz, px[k], py[k], pz[k]) < r2)) continue;
            const uint8_t st = __hip_atomic_load(&state[v], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (st == 1) kept_nb = true;
            else if (st == 0) all_removed = false;
          }
        }
      }
  if (active && kept_nb) {
    __hip_atomic_store(&state[u], (uint8_t)2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  } else if (active && all_removed) {
    __hip_atomic_store(&state[u], (uint8_t)1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  wave_append(active && !kept_nb && !all_removed, u, next, n_next);
}

// kept[point] = state[sorted position] == 1
__global__ __launch_bounds__(kBS) void k_mis_flags(const int32_t* __restrict__ sidx, int n,
                                                   const uint8_t* __restrict__ state,
                                                   uint8_t* __restrict__ kept) {
  const int u = blockIdx.x * kBS + threadIdx.x;
  if (u < n) kept[sidx[u]] = state[u] == 1 ? 1 : 0;
}

// output records: translated xyz (+ pad 1.0 in a 16-byte PointXYZ) and the source index
__global__ __launch_bounds__(kBS) void k_emit_points(const int32_t* __restrict__ sel, int n,
                                                     const float* __restrict__ X,
                                                     const float* __restrict__ Y,
                                                     const float* __restrict__ Z,
                                                     const int32_t* __restrict__ src,
                                                     float* __restrict__ out, int64_t stride,
                                                     int32_t* __restrict__ out_idx) {
  const int i = blockIdx.x * kBS + threadIdx.x;
  if (i >= n) return;
  const int k = sel[i];
  float* o = out + (int64_t)i * stride;
  o[0] = X[k]; o[1] = Y[k]; o[2] = Z[k];
  for (int f = 3; f < stride; ++f) o[f] = f == 3 ? 1.0f : 0.0f;
  out_idx[i] = src[k];
}

// ---------------------------------------------------------------------------------------------
// RegulateNormal BFS, one level per (claim, settle, order)
// The BFS state lives in the grid's sorted order (position u of point sidx[u]): processed[],
// claim[] and the normals are read per cell run, i.e. coalesced, instead of at random point ids.
// The queue holds point ids (PCL's order keys use them); pos_of[] maps id -> u.
__global__ __launch_bounds__(kBS) void k_bfs_prepare(const int32_t* __restrict__ sidx, int n,
                                                     const float4* __restrict__ nrm,
                                                     float4* __restrict__ nrm_s,
                                                     int32_t* __restrict__ pos_of) {
  const int u = blockIdx.x * kBS + threadIdx.x;
  if (u >= n) return;
  const int j = sidx[u];
  pos_of[j] = u;
  nrm_s[u] = nrm[j];
}

// seed (PlaneDetect.h:600-607): flip unless outward, mark processed, queue[0] = seed
__global__ void k_bfs_seed(int32_t seed, int flip, const int32_t* __restrict__ pos_of,
                           float4* __restrict__ nrm_s, uint8_t* __restrict__ processed_s,
                           int32_t* __restrict__ queue) {
  const int u = pos_of[seed];
  if (flip) {
    float4 v = nrm_s[u];
    v.x *= -1.0f; v.y *= -1.0f; v.z *= -1.0f;
    nrm_s[u] = v;
  }
  processed_s[u] = 1;
  queue[0] = seed;
}

// one thread per (frontier node, one of its 27 cells) in the claim pass: short dependent
// chains, 27x the threads
// ---- RegulateNormal without host round trips: every per-level quantity lives on the device.
// st[0] = fbase (queue position of the level's first node), st[1] = nf (level size),
// st[2] = ncand (nodes reached by this level), st[3] = qt (queue length).  Kernels stride over
// device-side counts, so the host enqueues many levels and only checks nf now and then.  The
// next level is ordered by a counting sort on the parent position (children per parent counted,
// scanned, scattered) and a per-parent sort of the few children by (d2, index).
__global__ __launch_bounds__(kBS) void k_bfs2_claim(
    const int32_t* __restrict__ queue, const long long* __restrict__ st,
    const int32_t* __restrict__ pos_of, const float* __restrict__ sx, const float* __restrict__ sy,
    const float* __restrict__ sz, GridDesc G, const uint32_t* __restrict__ tkeys,
    const int2* __restrict__ trange, uint32_t tmask, float r2,
    const uint8_t* __restrict__ processed_s, uint32_t* __restrict__ claim_s,
    int32_t* __restrict__ cand, long long* __restrict__ st_w, uint32_t* __restrict__ child_cnt,
    uint32_t* __restrict__ cursor, const uint32_t* __restrict__ cell_done) {
  (void)cell_done;
  constexpr int kStage = 2048;
  __shared__ uint32_t s_n;
  __shared__ long long s_base;
  __shared__ int32_t s_buf[kStage];
  if (threadIdx.x == 0) s_n = 0;
  __syncthreads();
  const long long fbase = st[0];
  const long long nf = st[1];
  const long long total = nf * 27;
  for (long long t = (long long)blockIdx.x * kBS + threadIdx.x; t < total;
       t += (long long)gridDim.x * kBS) {
    const int f = (int)(t / 27), c = (int)(t % 27);
    if (c == 0) { child_cnt[f] = 0; cursor[f] = 0; }
    const uint32_t mypos = (uint32_t)(fbase + f);
    const int cu = pos_of[queue[mypos]];
    const float qx = sx[cu], qy = sy[cu], qz = sz[cu];
    if (!finite3(qx, qy, qz)) continue;
    const int x = cell_of(qx, G.lo[0], G.inv_cell, G.g[0]) + c % 3 - 1;
    const int y = cell_of(qy, G.lo[1], G.inv_cell, G.g[1]) + (c / 3) % 3 - 1;
    const int z = cell_of(qz, G.lo[2], G.inv_cell, G.g[2]) + c / 9 - 1;
    if (x < 0 || y < 0 || z < 0 || x >= G.g[0] || y >= G.g[1] || z >= G.g[2]) continue;
    const int2 rg = cell_range(tkeys, trange, tmask, cell_key(G, x, y, z));
    // four cell points' state and coordinates loaded together (processed_s is fixed during the
    // claim pass; claims are a min, so the order the candidates are met in does not matter)
    for (int u0 = rg.x; u0 < rg.y; u0 += 4) {
      uint8_t pr[4];
      float px[4], py[4], pz[4];
#pragma unroll
      for (int v = 0; v < 4; ++v) {
        const int u = min(u0 + v, rg.y - 1);
        pr[v] = processed_s[u]; px[v] = sx[u]; py[v] = sy[u]; pz[v] = sz[u];
      }
#pragma unroll
      for (int v = 0; v < 4; ++v) {
        const int u = u0 + v;
        if (u >= rg.y || pr[v]) continue;
        if (!(flann_d2(qx, qy, qz, px[v], py[v], pz[v]) < r2)) continue;
        if (claim_s[u] <= mypos) continue;  // claims only decrease
        if (atomicMin(&claim_s[u], mypos) == 0xffffffffu) {
          const uint32_t p = atomicAdd(&s_n, 1u);
          if (p < (uint32_t)kStage) s_buf[p] = u;
          else cand[atomicAdd((unsigned long long*)&st_w[2], 1ull)] = u;
        }
      }
    }
  }
  __syncthreads();
  const uint32_t m = min(s_n, (uint32_t)kStage);
  if (threadIdx.x == 0 && m)
    s_base = (long long)atomicAdd((unsigned long long*)&st_w[2], (unsigned long long)m);
  __syncthreads();
  for (uint32_t i = threadIdx.x; i < m; i += kBS) cand[s_base + i] = s_buf[i];
}

// The claim pass with one wave per frontier node (default): the node's 27 cells packed into one
// candidate list (nbr_rows), scanned 64 candidates per step with four steps' loads in flight;
// waves take runs of kBqRun consecutive frontier nodes (children of consecutive parents: mostly
// the same cells, looked up once).  Same claims as k_bfs2_claim (a min: the order the candidates
// are met in does not matter), appended through the workgroup's LDS stage.
constexpr int kBqRun = 2;
__global__ __launch_bounds__(kBS) void k_bfs2_claim_w(
    const int32_t* __restrict__ queue, const long long* __restrict__ st,
    const int32_t* __restrict__ pos_of, const float* __restrict__ sx, const float* __restrict__ sy,
    const float* __restrict__ sz, GridDesc G, const uint32_t* __restrict__ tkeys,
    const int2* __restrict__ trange, uint32_t tmask, float r2,
    const uint8_t* __restrict__ processed_s, uint32_t* __restrict__ claim_s,
    int32_t* __restrict__ cand, long long* __restrict__ st_w, uint32_t* __restrict__ child_cnt,
    uint32_t* __restrict__ cursor, const uint32_t* __restrict__ cell_done) {
  constexpr int kStage = 2048;
  constexpr int kW = kBS / 64;
  __shared__ uint32_t s_n;
  __shared__ long long s_base;
  __shared__ int32_t s_buf[kStage];
  __shared__ int32_t s_rows[kW][20];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  int32_t* rows = s_rows[wv];
  if (threadIdx.x == 0) s_n = 0;
  __syncthreads();
  const long long fbase = st[0];
  const int nf = (int)st[1];
  const int nruns = (nf + kBqRun - 1) / kBqRun;
  const int gw = (int)((blockIdx.x * kBS + threadIdx.x) >> 6), nw = (int)((gridDim.x * kBS) >> 6);
  for (int run = gw; run < nruns; run += nw) {
    int pcx = -1, pcy = -1, pcz = -1;
    const int f_end = min(nf, (run + 1) * kBqRun);
    for (int f = run * kBqRun; f < f_end; ++f) {
      if (lane == 0) { child_cnt[f] = 0; cursor[f] = 0; }
      const uint32_t mypos = (uint32_t)(fbase + f);
      const int cu = pos_of[queue[mypos]];
      const float qx = sx[cu], qy = sy[cu], qz = sz[cu];
      if (!finite3(qx, qy, qz)) continue;
      const int cx = cell_of(qx, G.lo[0], G.inv_cell, G.g[0]);
      const int cy = cell_of(qy, G.lo[1], G.inv_cell, G.g[1]);
      const int cz = cell_of(qz, G.lo[2], G.inv_cell, G.g[2]);
      if (cx != pcx || cy != pcy || cz != pcz) {
        pcx = cx; pcy = cy; pcz = cz;
        nbr_rows(G, tkeys, trange, tmask, cx, cy, cz, rows, cell_done);
      }
      int r_start[9], r_off[9];
#pragma unroll
      for (int q = 0; q < 9; ++q) {
        r_start[q] = rows[q];
        r_off[q] = rows[9 + q];
      }
      const int tot = rows[18];
      for (int k0 = 0; k0 < tot; k0 += 64 * kFqB) {
        int uu[kFqB];
        uint8_t pr[kFqB];
        float px[kFqB], py[kFqB], pz[kFqB];
#pragma unroll
        for (int j = 0; j < kFqB; ++j) {
          const int v = k0 + 64 * j + lane;
          const int u = nbr_pos(r_start, r_off, min(v, tot - 1));
          uu[j] = v < tot ? u : -1;
          pr[j] = processed_s[u]; px[j] = sx[u]; py[j] = sy[u]; pz[j] = sz[u];
        }
#pragma unroll
        for (int j = 0; j < kFqB; ++j) {
          const int u = uu[j];
          if (u < 0 || pr[j]) continue;
          if (!(flann_d2(qx, qy, qz, px[j], py[j], pz[j]) < r2)) continue;
          if (claim_s[u] <= mypos) continue;  // claims only decrease
          if (atomicMin(&claim_s[u], mypos) == 0xffffffffu) {
            const uint32_t p = atomicAdd(&s_n, 1u);
            if (p < (uint32_t)kStage) s_buf[p] = u;
            else cand[atomicAdd((unsigned long long*)&st_w[2], 1ull)] = u;
          }
        }
      }
    }
  }
  __syncthreads();
  const uint32_t m = min(s_n, (uint32_t)kStage);
  if (threadIdx.x == 0 && m)
    s_base = (long long)atomicAdd((unsigned long long*)&st_w[2], (unsigned long long)m);
  __syncthreads();
  for (uint32_t i = threadIdx.x; i < m; i += kBS) cand[s_base + i] = s_buf[i];
}

__global__ __launch_bounds__(kBS) void k_bfs2_settle(
    const int32_t* __restrict__ queue, const int32_t* __restrict__ cand,
    const long long* __restrict__ st, const int32_t* __restrict__ pos_of,
    uint8_t* __restrict__ processed_s, const uint32_t* __restrict__ claim_s,
    float4* __restrict__ nrm_s, uint32_t* __restrict__ child_cnt, const float* __restrict__ sx,
    const float* __restrict__ sy, const float* __restrict__ sz, GridDesc G,
    const uint32_t* __restrict__ tkeys, uint32_t tmask, uint32_t* __restrict__ cell_done) {
  const long long fbase = st[0], nc = st[2];
  for (long long t = (long long)blockIdx.x * kBS + threadIdx.x; t < nc;
       t += (long long)gridDim.x * kBS) {
    const int u = cand[t];
    const uint32_t ppos = claim_s[u];
    const int pu = pos_of[queue[ppos]];
    const float4 pn = nrm_s[pu];
    float4 nn = nrm_s[u];
    const float dp = pn.x * nn.x + pn.y * nn.y + pn.z * nn.z;  // PlaneDetect.h:629
    if (dp < 0.0f) {
      nn.x *= -1.0f; nn.y *= -1.0f; nn.z *= -1.0f;
      nrm_s[u] = nn;
    }
    processed_s[u] = 1;
    atomicAdd(&child_cnt[ppos - fbase], 1u);
    // (u is finite: it passed the radius test; its cell is the one the grid binned it in)
    const int h = cell_slot(tkeys, tmask,
                            cell_key(G, cell_of(sx[u], G.lo[0], G.inv_cell, G.g[0]),
                                     cell_of(sy[u], G.lo[1], G.inv_cell, G.g[1]),
                                     cell_of(sz[u], G.lo[2], G.inv_cell, G.g[2])));
    if (h >= 0) atomicAdd(&cell_done[h], 1u);
  }
}

// exclusive scan of child_cnt[0..nf): tiles of 1024 scanned in LDS (offs = in-tile prefix,
// tile_tot = tile sums), then one workgroup scans the tile sums (nf is one BFS level)
__global__ __launch_bounds__(kBS) void k_bfs2_scan_tiles(const long long* __restrict__ st,
                                                         const uint32_t* __restrict__ child_cnt,
                                                         uint32_t* __restrict__ offs,
                                                         uint32_t* __restrict__ tile_tot) {
  __shared__ uint32_t s[1024];
  const long long nf = st[1];
  const long long ntiles = (nf + 1023) / 1024;
  for (long long tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    const long long base = tile * 1024;
    __syncthreads();
    for (int k = threadIdx.x; k < 1024; k += kBS)
      s[k] = base + k < nf ? child_cnt[base + k] : 0u;
    __syncthreads();
    // each thread scans 4 consecutive entries, then a block scan of the 256 partial sums
    uint32_t v[4], sum = 0;
    for (int k = 0; k < 4; ++k) { v[k] = s[threadIdx.x * 4 + k]; sum += v[k]; }
    __syncthreads();
    s[threadIdx.x] = sum;
    __syncthreads();
    for (int o = 1; o < kBS; o <<= 1) {
      const uint32_t add = threadIdx.x >= (unsigned)o ? s[threadIdx.x - o] : 0u;
      __syncthreads();
      s[threadIdx.x] += add;
      __syncthreads();
    }
    uint32_t run = s[threadIdx.x] - sum;
    for (int k = 0; k < 4; ++k) {
      const long long i = base + threadIdx.x * 4 + k;
      if (i < nf) offs[i] = run;
      run += v[k];
    }
    if (threadIdx.x == kBS - 1) tile_tot[tile] = s[kBS - 1];
  }
}

__global__ __launch_bounds__(1024) void k_bfs2_scan_top(const long long* __restrict__ st,
                                                        uint32_t* __restrict__ tile_tot) {
  __shared__ uint32_t s[1024];
  const long long ntiles = (st[1] + 1023) / 1024;
  uint32_t carry = 0;
  for (long long b = 0; b < ntiles; b += 1024) {
    const long long i = b + threadIdx.x;
    const uint32_t v = i < ntiles ? tile_tot[i] : 0u;
    s[threadIdx.x] = v;
    __syncthreads();
    for (int o = 1; o < 1024; o <<= 1) {
      const uint32_t add = threadIdx.x >= (unsigned)o ? s[threadIdx.x - o] : 0u;
      __syncthreads();
      s[threadIdx.x] += add;
      __syncthreads();
    }
    if (i < ntiles) tile_tot[i] = carry + s[threadIdx.x] - v;  // exclusive
    carry += s[1023];
    __syncthreads();
  }
}

__global__ __launch_bounds__(kBS) void k_bfs2_scatter(
    const int32_t* __restrict__ queue, const int32_t* __restrict__ cand,
    const long long* __restrict__ st, const int32_t* __restrict__ pos_of,
    const int32_t* __restrict__ sidx, const float* __restrict__ sx, const float* __restrict__ sy,
    const float* __restrict__ sz, const uint32_t* __restrict__ claim_s,
    const uint32_t* __restrict__ offs, const uint32_t* __restrict__ tile_tot,
    uint32_t* __restrict__ cursor, float* __restrict__ slot_d2, int32_t* __restrict__ slot_id,
    uint32_t* __restrict__ slot_of) {
  const long long fbase = st[0], nc = st[2];
  for (long long t = (long long)blockIdx.x * kBS + threadIdx.x; t < nc;
       t += (long long)gridDim.x * kBS) {
    const int u = cand[t];
    const uint32_t ppos = claim_s[u];
    const long long p = ppos - fbase;
    const int pu = pos_of[queue[ppos]];
    const uint32_t slot = tile_tot[p >> 10] + offs[p] + atomicAdd(&cursor[p], 1u);
    // the parent's neighbour list is sorted by the d2 FLANN computes for query = parent
    slot_d2[slot] = flann_d2(sx[pu], sy[pu], sz[pu], sx[u], sy[u], sz[u]);
    slot_id[slot] = sidx[u];
    slot_of[t] = slot;
  }
}

// each child's rank among its siblings by (d2, index) -> its queue position
__global__ __launch_bounds__(kBS) void k_bfs2_rank(const long long* __restrict__ st,
                                                   const int32_t* __restrict__ cand,
                                                   const uint32_t* __restrict__ claim_s,
                                                   const uint32_t* __restrict__ offs,
                                                   const uint32_t* __restrict__ tile_tot,
                                                   const uint32_t* __restrict__ child_cnt,
                                                   const uint32_t* __restrict__ slot_of,
                                                   const float* __restrict__ slot_d2,
                                                   const int32_t* __restrict__ slot_id,
                                                   int32_t* __restrict__ queue) {
  const long long fbase = st[0], nc = st[2], qt = st[3];
  for (long long t = (long long)blockIdx.x * kBS + threadIdx.x; t < nc;
       t += (long long)gridDim.x * kBS) {
    const long long p = claim_s[cand[t]] - fbase;
    const uint32_t o = tile_tot[p >> 10] + offs[p], m = child_cnt[p], me = slot_of[t];
    const float d = slot_d2[me];
    const int id = slot_id[me];
    uint32_t r = 0;
    for (uint32_t j = 0; j < m; ++j) {
      const float dj = slot_d2[o + j];
      r += (dj < d || (dj == d && slot_id[o + j] < id)) ? 1u : 0u;
    }
    queue[qt + o + r] = id;
  }
}

__global__ void k_bfs2_advance(long long* __restrict__ st) {
  const long long nf = st[1], nc = st[2];
  st[0] += nf;
  st[3] += nc;
  st[1] = nc;
  st[2] = 0;
}

// sorted order -> point order
__global__ __launch_bounds__(kBS) void k_bfs_finish(const int32_t* __restrict__ sidx, int n,
                                                    const float4* __restrict__ nrm_s,
                                                    const uint8_t* __restrict__ processed_s,
                                                    float4* __restrict__ nrm,
                                                    uint8_t* __restrict__ processed) {
  const int u = blockIdx.x * kBS + threadIdx.x;
  if (u >= n) return;
  const int j = sidx[u];
  nrm[j] = nrm_s[u];
  processed[j] = processed_s[u];
}

__global__ __launch_bounds__(kBS) void k_pack_normals(const float4* __restrict__ nrm, int n,
                                                      float* __restrict__ out, int64_t stride,
                                                      int curv_offset) {
  const int i = blockIdx.x * kBS + threadIdx.x;
  if (i >= n) return;
  const float4 v = nrm[i];
  float* o = out + (int64_t)i * stride;
  o[0] = v.x; o[1] = v.y; o[2] = v.z;
  if (curv_offset < 0) return;  // direction only: leave the caller's other fields alone
  for (int f = 3; f < stride; ++f) o[f] = f == curv_offset ? v.w : 0.0f;
}

__global__ __launch_bounds__(kBS) void k_unpack_normals(const float* __restrict__ in, int n,
                                                        int64_t stride, float4* __restrict__ nrm) {
  const int i = blockIdx.x * kBS + threadIdx.x;
  if (i >= n) return;
  const float* p = in + (int64_t)i * stride;
  nrm[i] = make_float4(p[0], p[1], p[2], 0.0f);
}

__global__ __launch_bounds__(kBS) void k_deinterleave(const float* __restrict__ raw, int n,
                                                      int64_t stride, float* __restrict__ X,
                                                      float* __restrict__ Y, float* __restrict__ Z) {
  const int i = blockIdx.x * kBS + threadIdx.x;
  if (i >= n) return;
  const float* p = raw + (int64_t)i * stride;
  X[i] = p[0];
  Y[i] = p[1];
  Z[i] = p[2];
}

inline unsigned cdiv(int64_t a, int64_t b) { return (unsigned)((a + b - 1) / b); }

}  // namespace

// ---------------------------------------------------------------------------------------------
int bbox_blocks(int n) {
  int b = (int)cdiv(n, kBS * 8);
  return b < 1 ? 1 : (b > 1024 ? 1024 : b);
}

void launch_bbox(const float* X, const float* Y, const float* Z, int n, float* partial,
                 hipStream_t s) {
  hipLaunchKernelGGL(k_bbox, dim3(bbox_blocks(n)), dim3(kBS), 0, s, X, Y, Z, n, partial);
}

size_t sort_tmp_bytes(int n, int key_bits) {
  size_t tmp = 0;
  (void)hipcub::DeviceRadixSort::SortPairs(nullptr, tmp, (uint32_t*)nullptr, (uint32_t*)nullptr,
                                           (int32_t*)nullptr, (int32_t*)nullptr, n, 0, key_bits);
  return tmp;
}

hipError_t grid_build(const float* X, const float* Y, const float* Z, int n, const GridDesc& G,
                      GridBufs& B, uint32_t* n_occupied, hipStream_t s, float4* rec) {
  hipError_t e = hipMemsetAsync(B.tkeys, 0xff, (size_t)(B.tmask + 1) * 4, s);
  if (e != hipSuccess) return e;
  e = hipMemsetAsync(n_occupied, 0, 16, s);  // [0] occupied cells, [2..3] sum of occupancy^2
  if (e != hipSuccess || n <= 0) return e;
  hipLaunchKernelGGL(k_cell_keys, dim3(cdiv(n, kBS)), dim3(kBS), 0, s, X, Y, Z, n, G, B.keys_in,
                     B.idx_in, rec);
  size_t tmp = B.sort_tmp_bytes;
  e = hipcub::DeviceRadixSort::SortPairs(B.sort_tmp, tmp, B.keys_in, B.keys_out, B.idx_in,
                                         B.idx_out, n, 0, G.key_bits, s);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(k_cells_build, dim3(cdiv(n, kBS)), dim3(kBS), 0, s, B.keys_out, B.idx_out, n,
                     G.ncells, X, Y, Z, B.tkeys, B.trange, B.tmask, B.sx, B.sy, B.sz, n_occupied,
                     (const float4*)rec);
  hipLaunchKernelGGL(k_cells_end, dim3(cdiv(n, kBS)), dim3(kBS), 0, s, B.keys_out, n, G.ncells,
                     B.tkeys, B.trange, B.tmask,
                     reinterpret_cast<unsigned long long*>(n_occupied + 2));
  return hipGetLastError();
}

void launch_normals_radius(const GridDesc& G, const GridBufs& B, int n, float r2, const float vp[3],
                           float4* normals, hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_normals_radius, dim3(cdiv(n, kBS)), dim3(kBS), 0, s, B.sx, B.sy, B.sz,
                     B.idx_out, n, G, B.tkeys, B.trange, B.tmask, r2, vp[0], vp[1], vp[2],
                     normals);
}

void launch_normals_knn(const KnnLevels& L, int level, const int32_t* qpos, int nq,
                        const float* X, const float* Y, const float* Z, int k, const float vp[3],
                        float4* normals, uint8_t* defer, int64_t defer_stride, int lmax,
                        bool pcl_float, hipStream_t s, int tnext) {
  if (nq <= 0) return;
  const dim3 g(cdiv(nq, kBS)), b(kBS);
  auto go = [&](auto kern) {
    hipLaunchKernelGGL(kern, g, b, 0, s, L, level, qpos, nq, X, Y, Z, k, vp[0], vp[1], vp[2],
                       normals, defer, defer_stride, lmax);
  };
  // (level 0: the histogram-buffered variant; the deferred levels scan and insert directly)
  auto pick = [&](auto l0) {
    constexpr bool Z = decltype(l0)::value;
    if (pcl_float) {
      if (k <= 8) go(k_normals_knn<8, true, Z>);
      else if (k <= 16) go(k_normals_knn<16, true, Z>);
      else if (k <= 24) go(k_normals_knn<24, true, Z>);
      else if (k <= 32) go(k_normals_knn<32, true, Z>);
      else go(k_normals_knn<64, true, Z>);
    } else {
      if (k <= 8) go(k_normals_knn<8, false, Z>);
      else if (k <= 16) go(k_normals_knn<16, false, Z>);
      else if (k <= 24) go(k_normals_knn<24, false, Z>);
      else if (k <= 32) go(k_normals_knn<32, false, Z>);
      else go(k_normals_knn<64, false, Z>);
    }
  };
  if (level == 0 && level != L.levels - 1) {
    pick(std::true_type{});
  } else if (level > 0 && k <= 64) {
    // (the deferred levels: one wave per query, k_normals_knn_wave)
    const dim3 gw((unsigned)cdiv((int64_t)nq * 64, kBS));
    const int tl = std::min(tnext >= 0 ? tnext : level + 1, lmax);
    auto gow = [&](auto kern) {
      hipLaunchKernelGGL(kern, gw, b, 0, s, L, level, qpos, nq, X, Y, Z, k, vp[0], vp[1], vp[2],
                         normals, defer, defer_stride, tl);
    };
    if (pcl_float) {
      if (k <= 24) gow(k_normals_knn_wave<24, true>);
      else gow(k_normals_knn_wave<64, true>);
    } else {
      if (k <= 24) gow(k_normals_knn_wave<24, false>);
      else gow(k_normals_knn_wave<64, false>);
    }
  } else {
    pick(std::false_type{});
  }
}

void launch_nbr_count(const GridDesc& G, const GridBufs& B, int q0, int nq, float r2,
                      int32_t* cnt, hipStream_t s) {
  if (nq <= 0) return;
  hipLaunchKernelGGL(k_nbr_count, dim3(cdiv(nq, kBS)), dim3(kBS), 0, s, B.sx, B.sy, B.sz, q0, nq,
                     G, B.tkeys, B.trange, B.tmask, r2, cnt);
}

size_t nbr_scan_tmp_bytes(int nq) {
  size_t t = 0;
  (void)hipcub::DeviceScan::ExclusiveSum(nullptr, t, (const int32_t*)nullptr, (int64_t*)nullptr, nq);
  return t;
}

hipError_t nbr_scan(void* tmp, size_t tmp_bytes, const int32_t* cnt, int64_t* off, int nq,
                    hipStream_t s) {
  return hipcub::DeviceScan::ExclusiveSum(tmp, tmp_bytes, cnt, off, nq, s);
}

void launch_nbr_fill_sort_normals(const GridDesc& G, const GridBufs& B, int q0, int nq, float r2,
                                  const int32_t* cnt, const int64_t* off, uint64_t* keys,
                                  const float* X, const float* Y, const float* Z, const float vp[3],
                                  float4* normals, int num_cus, hipStream_t s) {
  if (nq <= 0) return;
  hipLaunchKernelGGL(k_nbr_fill, dim3(cdiv(nq, kBS)), dim3(kBS), 0, s, B.sx, B.sy, B.sz,
                     B.idx_out, q0, nq, G, B.tkeys, B.trange, B.tmask, r2, off, keys);
  const unsigned gs = (unsigned)std::max<int64_t>(1, std::min<int64_t>(cdiv(nq, kBS / 64), (int64_t)num_cus * 16));
  hipLaunchKernelGGL(k_nbr_sort, dim3(gs), dim3(kBS), 0, s, nq, cnt, off, keys);
  hipLaunchKernelGGL(k_nbr_normals, dim3(cdiv(nq, kBS)), dim3(kBS), 0, s, B.sx, B.sy, B.sz,
                     B.idx_out, q0, nq, cnt, off, keys, X, Y, Z, vp[0], vp[1], vp[2], normals);
}

void launch_nbr_fused(const GridDesc& G, const GridBufs& B, int n, const int32_t* qlist,
                      const uint32_t* qcount, int wide, float r2, const float vp[3],
                      float4* normals, int32_t* ovf, uint32_t* ovf_count, int num_cus,
                      hipStream_t s) {
  if (n <= 0) return;
  const int64_t waves = qlist ? (int64_t)num_cus * 16 : cdiv(n, kFqRun);
  const unsigned g = (unsigned)std::max<int64_t>(1, std::min<int64_t>(cdiv(waves, kBS / 64),
                                                                      (int64_t)num_cus * 64));
  auto* k = wide ? k_nbr_fused_wide<16> : k_nbr_fused<8>;
  hipLaunchKernelGGL(k, dim3(g), dim3(kBS), 0, s, B.sx, B.sy, B.sz, B.idx_out, n, qlist, qcount, G,
                     B.tkeys, B.trange, B.tmask, r2, vp[0], vp[1], vp[2], normals, ovf, ovf_count);
}

__global__ __launch_bounds__(kBS) void k_gather_flags(const uint8_t* __restrict__ f,
                                                      const int32_t* __restrict__ idx, int n,
                                                      uint8_t* __restrict__ out) {
  const int u = blockIdx.x * kBS + threadIdx.x;
  if (u < n) out[u] = f[idx[u]];
}

void launch_gather_flags(const uint8_t* f, const int32_t* idx, int n, uint8_t* out,
                         hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_gather_flags, dim3(cdiv(n, kBS)), dim3(kBS), 0, s, f, idx, n, out);
}

void launch_inverse_perm(const int32_t* idx, int n, int32_t* pos_of, hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_inverse_perm, dim3(cdiv(n, kBS)), dim3(kBS), 0, s, idx, n, pos_of);
}

void launch_nn1(const KnnLevels& L, int level, const int32_t* qlist, int nq, const float* qx,
                const float* qy, const float* qz, int32_t* nn, int32_t* next, uint32_t* n_next,
                hipStream_t s) {
  if (nq <= 0) return;
  hipLaunchKernelGGL(k_nn1, dim3(cdiv(nq, kBS)), dim3(kBS), 0, s, L, level, qlist, nq, qx, qy, qz,
                     nn, next, n_next);
}

void launch_flip_to_reference(float* nrm, int64_t stride_f, const float* ref, int64_t ref_stride_f,
                              const int32_t* nn, int n, hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_flip_to_reference, dim3(cdiv(n, kBS)), dim3(kBS), 0, s, nrm, stride_f, ref,
                     ref_stride_f, nn, n);
}

void launch_finite_flags(const float* X, const float* Y, const float* Z, int n, uint8_t* flags,
                         hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_finite_flags, dim3(cdiv(n, kBS)), dim3(kBS), 0, s, X, Y, Z, n, flags);
}

size_t select_tmp_bytes(int n) {
  size_t t = 0;
  (void)hipcub::DeviceSelect::Flagged(nullptr, t, hipcub::CountingInputIterator<int32_t>(0),
                                      (const uint8_t*)nullptr, (int32_t*)nullptr,
                                      (uint32_t*)nullptr, (int64_t)n);
  return t;
}

hipError_t select_flagged(void* tmp, size_t tmp_bytes, const uint8_t* flags, int n, int32_t* out,
                          uint32_t* n_out, hipStream_t s) {
  size_t t = tmp_bytes;
  return hipcub::DeviceSelect::Flagged(tmp, t, hipcub::CountingInputIterator<int32_t>(0), flags,
                                       out, n_out, (int64_t)n, s);
}

void launch_gather3(const int32_t* src, int n, const float* X, const float* Y, const float* Z,
                    float* OX, float* OY, float* OZ, hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_gather3, dim3(cdiv(n, kBS)), dim3(kBS), 0, s, src, n, X, Y, Z, OX, OY, OZ);
}

void launch_centroid_div(const float* sums3, int n, float* out, hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_centroid_div, dim3(1), dim3(64), 0, s, sums3, n, out);
}

void launch_translate(float* X, float* Y, float* Z, int n, const float* p, hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_translate, dim3(cdiv(n, kBS)), dim3(kBS), 0, s, X, Y, Z, n, p);
}

void launch_mis_round(const int32_t* qlist, int nq, const GridDesc& G, const GridBufs& B, float r2,
                      uint8_t* state, int32_t* next, uint32_t* n_next, hipStream_t s) {
  if (nq <= 0) return;
  hipLaunchKernelGGL(k_mis_round, dim3(cdiv(nq, kBS)), dim3(kBS), 0, s, qlist, nq, B.sx, B.sy,
                     B.sz, B.idx_out, G, B.tkeys, B.trange, B.tmask, r2, state, next, n_next);
}

void launch_mis_flags(const GridBufs& B, int n, const uint8_t* state, uint8_t* kept,
                      hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_mis_flags, dim3(cdiv(n, kBS)), dim3(kBS), 0, s, B.idx_out, n, state, kept);
}

void launch_emit_points(const int32_t* sel, int n, const float* X, const float* Y, const float* Z,
                        const int32_t* src, float* out, int64_t stride_f, int32_t* out_idx,
                        hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_emit_points, dim3(cdiv(n, kBS)), dim3(kBS), 0, s, sel, n, X, Y, Z, src, out,
                     stride_f, out_idx);
}

void launch_bfs_prepare(const GridBufs& B, int n, const float4* nrm, float4* nrm_s, int32_t* pos_of,
                        hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_bfs_prepare, dim3(cdiv(n, kBS)), dim3(kBS), 0, s, B.idx_out, n, nrm, nrm_s,
                     pos_of);
}

void launch_bfs_seed(int32_t seed, int flip, const int32_t* pos_of, float4* nrm_s,
                     uint8_t* processed_s, int32_t* queue, hipStream_t s) {
  hipLaunchKernelGGL(k_bfs_seed, dim3(1), dim3(1), 0, s, seed, flip, pos_of, nrm_s, processed_s,
                     queue);
}

void launch_bfs2_level(int32_t* queue, long long* st, const int32_t* pos_of, const GridDesc& G,
                       const GridBufs& B, float r2, uint8_t* processed_s, uint32_t* claim_s,
                       float4* nrm_s, int32_t* cand, const Bfs2Bufs& W, int grid, hipStream_t s,
                       bool wave_claim) {
  // (the wave claim: 16x the workgroups, about one run of kBqRun = 2 frontier nodes per wave --
  // more dependent candidate loads in flight per CU: claim 171 -> 118 us per level at C5; runs
  // of 8 / 4 / 1 with 4x / 8x / 32x: 146 / 131 / 139 us)
  hipLaunchKernelGGL(wave_claim ? k_bfs2_claim_w : k_bfs2_claim, dim3(wave_claim ? 16 * grid : grid),
                     dim3(kBS), 0, s,
                     queue, st, pos_of, B.sx, B.sy, B.sz, G, B.tkeys, B.trange, B.tmask, r2,
                     processed_s, claim_s, cand, st, W.child_cnt, W.cursor, W.cell_done);
  hipLaunchKernelGGL(k_bfs2_settle, dim3(grid), dim3(kBS), 0, s, queue, cand, st, pos_of,
                     processed_s, claim_s, nrm_s, W.child_cnt, B.sx, B.sy, B.sz, G, B.tkeys,
                     B.tmask, W.cell_done);
  hipLaunchKernelGGL(k_bfs2_scan_tiles, dim3(grid), dim3(kBS), 0, s, st, W.child_cnt, W.offs,
                     W.tile_tot);
  hipLaunchKernelGGL(k_bfs2_scan_top, dim3(1), dim3(1024), 0, s, st, W.tile_tot);
  hipLaunchKernelGGL(k_bfs2_scatter, dim3(grid), dim3(kBS), 0, s, queue, cand, st, pos_of,
                     B.idx_out, B.sx, B.sy, B.sz, claim_s, W.offs, W.tile_tot, W.cursor,
                     W.slot_d2, W.slot_id, W.slot_of);
  hipLaunchKernelGGL(k_bfs2_rank, dim3(grid), dim3(kBS), 0, s, st, cand, claim_s, W.offs,
                     W.tile_tot, W.child_cnt, W.slot_of, W.slot_d2, W.slot_id, queue);
  hipLaunchKernelGGL(k_bfs2_advance, dim3(1), dim3(1), 0, s, st);
}

void launch_bfs_finish(const GridBufs& B, int n, const float4* nrm_s, const uint8_t* processed_s,
                       float4* nrm, uint8_t* processed, hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_bfs_finish, dim3(cdiv(n, kBS)), dim3(kBS), 0, s, B.idx_out, n, nrm_s,
                     processed_s, nrm, processed);
}


void launch_pack_normals(const float4* nrm, int n, float* out, int64_t stride_floats,
                         int curv_offset, hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_pack_normals, dim3(cdiv(n, kBS)), dim3(kBS), 0, s, nrm, n, out,
                     stride_floats, curv_offset);
}

void launch_deinterleave(const float* raw, int n, int64_t stride_floats, float* X, float* Y,
                         float* Z, hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_deinterleave, dim3(cdiv(n, kBS)), dim3(kBS), 0, s, raw, n, stride_floats, X,
                     Y, Z);
}

void launch_unpack_normals(const float* in, int n, int64_t stride_floats, float4* nrm,
                           hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_unpack_normals, dim3(cdiv(n, kBS)), dim3(kBS), 0, s, in, n, stride_floats,
                     nrm);
}

}  // namespace dlg
