// postprocess.hip -- the data-parallel parts of postProcessPlanes (Dialog/PlaneDetect.h:1454-1579)
// on gfx950.
//
// Leftover absorption (:1530-1556): every unprocessed point is tested against every plane from
// plane_start_index on with isPointInPoly (:1891-1964).  The test is 10 rays (one per random
// border edge, the same ten for every point: srand(time(0)) is reseeded at each call) x every
// border edge, each an isBothLineSegsIntersect (:1966-2015) in float; a point is inside when at
// least 5 rays cross the border an odd number of times.  Work = candidates x 10 x edges, each
// ~150 f32 VALU ops with 4-6 IEEE square roots: VALU-bound.  Points farther than
// T_dist_point_plane from a plane are filtered first (one double-precision projection per
// (point, plane)), the survivors are grouped per plane, and one workgroup takes 256 candidates
// of one plane against a run of that plane's edges: the edge records are wave-uniform (scalar
// loads), the 10 rays live in registers, and the per-ray crossing parities are combined with
// an atomic XOR when a plane's edges are split over several workgroups.
//
// clusterFilt (:1582-1655): connected components of the radius graph of the remaining points
// (union-find, hooking the larger root under the smaller with CAS); a component is dropped when
// its size <= T_cluster_num.  The BFS of the reference finds the same components.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "grid_dev.hpp"
#include "postprocess.hpp"

namespace dlg {

namespace {

using namespace grid;

constexpr int kBS = 256;

__device__ __forceinline__ bool pip_candidate(V3 q, float4 c, float t_dist) {
  const V3 pp = proj_to_plane(q, c);
  // isPointInPoly returns false for dist > T; NaN distances (NaN plane or point) cannot pass
  // the ray test either (every crossing test compares NaN), so they are not candidates
  return dist_p2p(q, pp) <= t_dist;
}

__global__ __launch_bounds__(kBS) void k_pip_candidates(
    const float* __restrict__ X, const float* __restrict__ Y, const float* __restrict__ Z, int n,
    const uint8_t* __restrict__ processed, const float4* __restrict__ planes, float t_dist,
    uint32_t* __restrict__ counts, const uint32_t* __restrict__ offs, uint32_t* __restrict__ cursor,
    int32_t* __restrict__ cand) {
  const int p = blockIdx.y;
  const int i = blockIdx.x * kBS + threadIdx.x;
  bool c = false;
  if (i < n && !processed[i]) c = pip_candidate(V3{X[i], Y[i], Z[i]}, planes[p], t_dist);
  const uint64_t m = __ballot(c);
  if (m == 0) return;
  const int lane = threadIdx.x & 63;
  const int leader = __ffsll((unsigned long long)m) - 1;
  if (!cand) {
    if (lane == leader) atomicAdd(&counts[p], (uint32_t)__popcll(m));
    return;
  }
  uint32_t base = 0;
  if (lane == leader) base = atomicAdd(&cursor[p], (uint32_t)__popcll(m));
  base = __shfl(base, leader, 64);
  const int below = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32),
                                              __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
  if (c) cand[offs[p] + base + below] = i;
}

__global__ __launch_bounds__(kBS) void k_pip_test(
    const PipTask* __restrict__ tasks, const int32_t* __restrict__ cand,
    const float* __restrict__ X, const float* __restrict__ Y, const float* __restrict__ Z,
    const float4* __restrict__ planes, const float4* __restrict__ rays,
    const PipEdge* __restrict__ edges, const int64_t* __restrict__ edge_off,
    uint32_t* __restrict__ mask) {
  const PipTask T = tasks[blockIdx.x];
  const int t = threadIdx.x;
  const bool act = t < T.ccnt;
  const int ci = T.cbeg + (act ? t : 0);
  const int i = cand[ci];
  const V3 pc = proj_to_plane(V3{X[i], Y[i], Z[i]}, planes[T.plane]);
  PipRay R[kPipRays];
#pragma unroll
  for (int k = 0; k < kPipRays; ++k) {
    const float4 d = rays[T.plane * kPipRays + k];
    R[k] = make_ray(pc, V3{d.x, d.y, d.z});
  }
  const PipEdge* __restrict__ E = edges + edge_off[T.plane];
  uint32_t bits = 0;
  for (int e = T.ebeg; e < T.eend; ++e) {
    const PipEdge ed = E[e];
    const V3 pa{ed.a_dab.x, ed.a_dab.y, ed.a_dab.z}, pb{ed.b.x, ed.b.y, ed.b.z};
    const V3 nab{ed.nab.x, ed.nab.y, ed.nab.z};
#pragma unroll
    for (int k = 0; k < kPipRays; ++k)
      if (segs_intersect(pa, pb, nab, ed.a_dab.w, pc, R[k])) bits ^= 1u << k;
  }
  if (act && bits) atomicXor(&mask[ci], bits);
}

__global__ __launch_bounds__(kBS) void k_pip_mark(
    const int32_t* __restrict__ cand, const uint32_t* __restrict__ mask,
    const uint32_t* __restrict__ offs, const uint32_t* __restrict__ counts, int n,
    uint8_t* __restrict__ absorbed, uint8_t* __restrict__ processed,
    uint32_t* __restrict__ abs_cnt) {
  const int p = blockIdx.y;
  const int t = blockIdx.x * kBS + threadIdx.x;
  bool in = false;
  int i = 0;
  if (t < (int)counts[p]) {
    const int ci = (int)offs[p] + t;
    i = cand[ci];
    in = __popc(mask[ci] & ((1u << kPipRays) - 1u)) >= kPipRays / 2;
  }
  if (in) {
    absorbed[(int64_t)p * n + i] = 1;
    processed[i] = 1;
  }
  const uint64_t m = __ballot(in);
  if (m && (threadIdx.x & 63) == __ffsll((unsigned long long)m) - 1)
    atomicAdd(&abs_cnt[p], (uint32_t)__popcll(m));
}

__global__ __launch_bounds__(kBS) void k_mark_nn(const int32_t* __restrict__ nn, int m,
                                                 uint8_t* __restrict__ processed) {
  const int j = blockIdx.x * kBS + threadIdx.x;
  if (j < m && nn[j] >= 0) processed[nn[j]] = 1;
}

__global__ __launch_bounds__(kBS) void k_invert_flags(const uint8_t* __restrict__ processed, int n,
                                                      uint8_t* __restrict__ flags) {
  const int i = blockIdx.x * kBS + threadIdx.x;
  if (i < n) flags[i] = processed[i] ? 0 : 1;
}

__global__ __launch_bounds__(kBS) void k_gather_ids(const int32_t* __restrict__ sel, int n,
                                                    const int32_t* __restrict__ map,
                                                    int32_t* __restrict__ out) {
  const int i = blockIdx.x * kBS + threadIdx.x;
  if (i < n) out[i] = map[sel[i]];
}

// ---- clusterFilt: union-find over sorted positions ----
__device__ __forceinline__ int uf_load(int32_t* parent, int x) {
  return __hip_atomic_load(&parent[x], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// root of x with path halving (benign races: every stored value is an ancestor)
__device__ int uf_find(int32_t* parent, int x) {
  int p = uf_load(parent, x);
  while (p != x) {
    const int g = uf_load(parent, p);
    if (g != p)
      __hip_atomic_store(&parent[x], g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    x = p;
    p = g;
  }
  return x;
}

__device__ void uf_unite(int32_t* parent, int a, int b) {
  while (true) {
    a = uf_find(parent, a);
    b = uf_find(parent, b);
    if (a == b) return;
    if (a < b) { const int t = a; a = b; b = t; }
    // hook the larger root under the smaller; a failed CAS means a was hooked meanwhile
    const int old = atomicCAS(&parent[a], a, b);
    if (old == a) return;
    a = old;
  }
}

__global__ __launch_bounds__(kBS) void k_cc_init(int32_t* __restrict__ parent,
                                                 uint32_t* __restrict__ size, int n) {
  const int u = blockIdx.x * kBS + threadIdx.x;
  if (u < n) {
    parent[u] = u;
    size[u] = 0;
  }
}

__global__ __launch_bounds__(kBS) void k_cc_hook(const float* __restrict__ sx,
                                                 const float* __restrict__ sy,
                                                 const float* __restrict__ sz, int n, GridDesc G,
                                                 const uint32_t* __restrict__ tkeys,
                                                 const int2* __restrict__ trange, uint32_t tmask,
                                                 float r2, int32_t* parent) {
  const int u = blockIdx.x * kBS + threadIdx.x;
  if (u >= n) return;
  const float qx = sx[u], qy = sy[u], qz = sz[u];
  const int cx = cell_of(qx, G.lo[0], G.inv_cell, G.g[0]);
  const int cy = cell_of(qy, G.lo[1], G.inv_cell, G.g[1]);
  const int cz = cell_of(qz, G.lo[2], G.inv_cell, G.g[2]);
  for (int z = max(cz - 1, 0); z <= min(cz + 1, G.g[2] - 1); ++z)
    for (int y = max(cy - 1, 0); y <= min(cy + 1, G.g[1] - 1); ++y)
      for (int x = max(cx - 1, 0); x <= min(cx + 1, G.g[0] - 1); ++x) {
        const int2 rg = cell_range(tkeys, trange, tmask, cell_key(G, x, y, z));
        const int end = min(rg.y, u);  // each undirected edge once: v < u
        for (int v = rg.x; v < end; ++v) {
          if (!(flann_d2(qx, qy, qz, sx[v], sy[v], sz[v]) < r2)) continue;
          uf_unite(parent, u, v);
        }
      }
}

__global__ __launch_bounds__(kBS) void k_cc_count(int32_t* parent, int n,
                                                  uint32_t* __restrict__ size) {
  const int u = blockIdx.x * kBS + threadIdx.x;
  if (u >= n) return;
  atomicAdd(&size[uf_find(parent, u)], 1u);
}

__global__ __launch_bounds__(kBS) void k_cc_keep(const int32_t* __restrict__ sidx,
                                                 const int32_t* parent, int n,
                                                 const uint32_t* __restrict__ size,
                                                 uint64_t t_cluster_num,
                                                 uint8_t* __restrict__ keep) {
  const int u = blockIdx.x * kBS + threadIdx.x;
  if (u >= n) return;
  int r = u;  // read-only walk: every chain ends at its final root once the hooks are done
  while (parent[r] != r) r = parent[r];
  keep[sidx[u]] = (uint64_t)size[r] > t_cluster_num ? 1 : 0;
}

inline unsigned cdiv(int64_t a, int64_t b) { return (unsigned)((a + b - 1) / b); }

}  // namespace

void launch_pip_candidates(const float* X, const float* Y, const float* Z, int n,
                           const uint8_t* processed, const float4* planes, int n_planes,
                           float t_dist, uint32_t* counts, const uint32_t* offs, uint32_t* cursor,
                           int32_t* cand, hipStream_t s) {
  if (n <= 0 || n_planes <= 0) return;
  hipLaunchKernelGGL(k_pip_candidates, dim3(cdiv(n, kBS), n_planes), dim3(kBS), 0, s, X, Y, Z, n,
                     processed, planes, t_dist, counts, offs, cursor, cand);
}

void launch_pip_test(const PipTask* tasks, int n_tasks, const int32_t* cand, const float* X,
                     const float* Y, const float* Z, const float4* planes, const float4* rays,
                     const PipEdge* edges, const int64_t* edge_off, uint32_t* mask,
                     hipStream_t s) {
  if (n_tasks <= 0) return;
  hipLaunchKernelGGL(k_pip_test, dim3(n_tasks), dim3(kBS), 0, s, tasks, cand, X, Y, Z, planes,
                     rays, edges, edge_off, mask);
}

void launch_pip_mark(const int32_t* cand, const uint32_t* mask, const uint32_t* offs,
                     const uint32_t* counts, int n_planes, int max_count, int n,
                     uint8_t* absorbed, uint8_t* processed, uint32_t* abs_cnt, hipStream_t s) {
  if (max_count <= 0 || n_planes <= 0) return;
  hipLaunchKernelGGL(k_pip_mark, dim3(cdiv(max_count, kBS), n_planes), dim3(kBS), 0, s, cand, mask,
                     offs, counts, n, absorbed, processed, abs_cnt);
}

void launch_mark_nn(const int32_t* nn, int m, uint8_t* processed, hipStream_t s) {
  if (m <= 0) return;
  hipLaunchKernelGGL(k_mark_nn, dim3(cdiv(m, kBS)), dim3(kBS), 0, s, nn, m, processed);
}

void launch_invert_flags(const uint8_t* processed, int n, uint8_t* flags, hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_invert_flags, dim3(cdiv(n, kBS)), dim3(kBS), 0, s, processed, n, flags);
}

void launch_gather_ids(const int32_t* sel, int n, const int32_t* map, int32_t* out,
                       hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_gather_ids, dim3(cdiv(n, kBS)), dim3(kBS), 0, s, sel, n, map, out);
}

void launch_cc(const GridDesc& G, const GridBufs& B, int n, float r2, int64_t t_cluster_num,
               int32_t* parent, uint32_t* size, uint8_t* keep, hipStream_t s) {
  if (n <= 0) return;
  const unsigned g = cdiv(n, kBS);
  hipLaunchKernelGGL(k_cc_init, dim3(g), dim3(kBS), 0, s, parent, size, n);
  hipLaunchKernelGGL(k_cc_hook, dim3(g), dim3(kBS), 0, s, B.sx, B.sy, B.sz, n, G, B.tkeys,
                     B.trange, B.tmask, r2, parent);
  hipLaunchKernelGGL(k_cc_count, dim3(g), dim3(kBS), 0, s, parent, n, size);
  hipLaunchKernelGGL(k_cc_keep, dim3(g), dim3(kBS), 0, s, B.idx_out, parent, n, size,
                     (uint64_t)t_cluster_num, keep);
}

}  // namespace dlg
