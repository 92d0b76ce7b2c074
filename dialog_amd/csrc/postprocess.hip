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
#include <hipcub/hipcub.hpp>

#include <cfloat>
#include <cstdint>

#include "grid_dev.hpp"
#include "postprocess.hpp"

namespace dlg {

namespace {

using namespace grid;

constexpr int kBS = 256;

inline unsigned cdiv(int64_t a, int64_t b) { return (unsigned)((a + b - 1) / b); }

__device__ __forceinline__ bool pip_candidate(V3 q, float4 c, float t_dist) {
  const V3 pp = proj_to_plane(q, c);
  // isPointInPoly returns false for dist > T; NaN distances (NaN plane or point) cannot pass
  // the ray test either (every crossing test compares NaN), so they are not candidates
  return dist_p2p(q, pp) <= t_dist;
}

// exclusive prefix of `pred` over the workgroup (ballot + LDS wave totals); returns the total
__device__ __forceinline__ uint32_t block_prefix(bool pred, uint32_t* below) {
  __shared__ uint32_t wtot[kBS / 64];
  const uint64_t m = __ballot(pred);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const uint32_t in_wave = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32),
                                                     __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
  if (lane == 0) wtot[w] = (uint32_t)__popcll(m);
  __syncthreads();
  uint32_t before = 0, tot = 0;
  for (int k = 0; k < kBS / 64; ++k) {
    before += k < w ? wtot[k] : 0u;
    tot += wtot[k];
  }
  *below = before + in_wave;
  return tot;
}

// pass 1: bcnt[p * nblk + block] = candidates of plane p (blockIdx.y) in the block's points
__global__ __launch_bounds__(kBS) void k_pip_count(
    const float* __restrict__ X, const float* __restrict__ Y, const float* __restrict__ Z, int n,
    const uint8_t* __restrict__ processed, const float4* __restrict__ planes, float t_dist,
    uint32_t* __restrict__ bcnt) {
  const int p = blockIdx.y;
  const int i = blockIdx.x * kBS + threadIdx.x;
  bool c = false;
  if (i < n && !processed[i]) c = pip_candidate(V3{X[i], Y[i], Z[i]}, planes[p], t_dist);
  uint32_t below;
  const uint32_t tot = block_prefix(c, &below);
  if (threadIdx.x == 0) bcnt[(size_t)p * gridDim.x + blockIdx.x] = tot;
}

// pass 2: candidates of plane p in ascending point order at boff[p * nblk + block] + rank
__global__ __launch_bounds__(kBS) void k_pip_fill(
    const float* __restrict__ X, const float* __restrict__ Y, const float* __restrict__ Z, int n,
    const uint8_t* __restrict__ processed, const float4* __restrict__ planes, float t_dist,
    const uint32_t* __restrict__ boff, int32_t* __restrict__ cand) {
  const int p = blockIdx.y;
  const int i = blockIdx.x * kBS + threadIdx.x;
  bool c = false;
  if (i < n && !processed[i]) c = pip_candidate(V3{X[i], Y[i], Z[i]}, planes[p], t_dist);
  uint32_t below;
  (void)block_prefix(c, &below);
  if (c) cand[boff[(size_t)p * gridDim.x + blockIdx.x] + below] = i;
}

__device__ __forceinline__ uint64_t spread3_14(uint32_t v) {  // 14 bits -> every third bit
  uint64_t x = v & 0x3fffu;
  x = (x | (x << 16)) & 0x0000ff0000ffull;
  x = (x | (x << 8)) & 0x00f00f00f00full;
  x = (x | (x << 4)) & 0x0c30c30c30c3ull;
  x = (x | (x << 2)) & 0x249249249249ull;
  return x;
}

// sort key of a candidate: plane (major), then the 3-D Morton code of the point, so that the
// lanes of a wave hold nearby points (their parallel rays meet the same few border edges, and
// the early outs of segs_intersect agree across the wave)
__global__ __launch_bounds__(kBS) void k_pip_keys(const int32_t* __restrict__ cand,
                                                  const uint32_t* __restrict__ offs,
                                                  const float* __restrict__ X,
                                                  const float* __restrict__ Y,
                                                  const float* __restrict__ Z, float4 lo_scale,
                                                  uint64_t* __restrict__ keys) {
  const int p = blockIdx.y;
  const int t = blockIdx.x * kBS + threadIdx.x;
  if (t >= (int)(offs[p + 1] - offs[p])) return;
  const int ci = (int)offs[p] + t;
  const int i = cand[ci];
  const float sc = lo_scale.w;
  const uint32_t qx = (uint32_t)fminf(fmaxf((X[i] - lo_scale.x) * sc, 0.0f), 16383.0f);
  const uint32_t qy = (uint32_t)fminf(fmaxf((Y[i] - lo_scale.y) * sc, 0.0f), 16383.0f);
  const uint32_t qz = (uint32_t)fminf(fmaxf((Z[i] - lo_scale.z) * sc, 0.0f), 16383.0f);
  keys[ci] = ((uint64_t)p << 42) | spread3_14(qx) | (spread3_14(qy) << 1) | (spread3_14(qz) << 2);
}

// offs[p] = first candidate of plane p, offs[P] = total
__global__ void k_pip_ranges(const uint32_t* __restrict__ bcnt, const uint32_t* __restrict__ boff,
                             int nblk, int n_planes, uint32_t* __restrict__ offs) {
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p < n_planes) offs[p] = boff[(size_t)p * nblk];
  if (p == n_planes) {
    const size_t last = (size_t)n_planes * nblk - 1;
    offs[p] = boff[last] + bcnt[last];
  }
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
  const float pc_l1 = (fabsf(pc.x) + fabsf(pc.y)) + fabsf(pc.z);
  const PipEdge* __restrict__ E = edges + edge_off[T.plane];
  uint32_t bits = 0;
  // ray-outer, edge-inner: one ray in registers, the (wave-uniform) edge records in SGPRs
#pragma unroll 1
  for (int k = 0; k < kPipRays; ++k) {
    const float4 d = rays[T.plane * kPipRays + k];
    const PipRay R = make_ray(pc, V3{d.x, d.y, d.z});
    uint32_t odd = 0;
    for (int e = T.ebeg; e < T.eend; ++e) {
      const PipEdge ed = E[e];
      const V3 pa{ed.a_dab.x, ed.a_dab.y, ed.a_dab.z}, pb{ed.b.x, ed.b.y, ed.b.z};
      const V3 nab{ed.nab.x, ed.nab.y, ed.nab.z};
      odd ^= segs_intersect(pa, pb, nab, ed.a_dab.w, ed.b.w, pc, pc_l1, R) ? 1u : 0u;
    }
    bits |= odd << k;
  }
  if (act && bits) atomicXor(&mask[ci], bits);
}

__global__ __launch_bounds__(kBS) void k_pip_mark(
    const int32_t* __restrict__ cand, const uint32_t* __restrict__ mask,
    const uint32_t* __restrict__ offs, int n, uint8_t* __restrict__ absorbed,
    uint8_t* __restrict__ processed, uint32_t* __restrict__ abs_cnt) {
  const int p = blockIdx.y;
  const int t = blockIdx.x * kBS + threadIdx.x;
  bool in = false;
  int i = 0;
  if (t < (int)(offs[p + 1] - offs[p])) {
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

// ---- 1-NN shortcut: a plane point equal to a cloud point has that point as nearest neighbour
// (d2 = 0; equal points -> the lowest index).  Valid when every coordinate has |v| >= 2^-50:
// any other float differs by >= 2^-73 there, whose square does not underflow, so d2 > 0 for
// every point not equal to the query.  Other queries take the grid search.
__device__ __forceinline__ uint32_t xyz_hash(uint32_t a, uint32_t b, uint32_t c) {
  uint32_t h = a * 0x9e3779b1u ^ (b + 0x7f4a7c15u) * 0x85ebca77u ^ (c + 0x165667b1u) * 0xc2b2ae3du;
  h ^= h >> 15;
  h *= 0x2c1b3c6du;
  h ^= h >> 12;
  return h;
}

__device__ __forceinline__ bool same_bits(float a, float b) {
  return __float_as_uint(a) == __float_as_uint(b);
}

__global__ __launch_bounds__(kBS) void k_xyz_insert(const float* __restrict__ X,
                                                    const float* __restrict__ Y,
                                                    const float* __restrict__ Z, int n,
                                                    int32_t* table, uint32_t tmask) {
  const int i = blockIdx.x * kBS + threadIdx.x;
  if (i >= n) return;
  const float x = X[i], y = Y[i], z = Z[i];
  if (!(isfinite(x) && isfinite(y) && isfinite(z))) return;
  uint32_t h = xyz_hash(__float_as_uint(x), __float_as_uint(y), __float_as_uint(z)) & tmask;
  while (true) {
    int32_t j = atomicCAS(&table[h], -1, i);
    if (j == -1) return;
    // occupied: every index stored in a slot has the coordinates of the slot's first writer
    if (same_bits(X[j], x) && same_bits(Y[j], y) && same_bits(Z[j], z)) {
      atomicMin(&table[h], i);
      return;
    }
    h = (h + 1) & tmask;
  }
}

__global__ __launch_bounds__(kBS) void k_xyz_lookup(
    const float* __restrict__ qx, const float* __restrict__ qy, const float* __restrict__ qz, int m,
    const int32_t* __restrict__ table, uint32_t tmask, const float* __restrict__ X,
    const float* __restrict__ Y, const float* __restrict__ Z, int32_t* __restrict__ nn,
    int32_t* __restrict__ rest, uint32_t* __restrict__ n_rest) {
  const int q = blockIdx.x * kBS + threadIdx.x;
  bool miss = false;
  if (q < m) {
    const float x = qx[q], y = qy[q], z = qz[q];
    const float lim = 0x1p-50f;
    miss = true;
    if (fabsf(x) >= lim && fabsf(y) >= lim && fabsf(z) >= lim && fabsf(x) <= FLT_MAX &&
        fabsf(y) <= FLT_MAX && fabsf(z) <= FLT_MAX) {
      uint32_t h = xyz_hash(__float_as_uint(x), __float_as_uint(y), __float_as_uint(z)) & tmask;
      while (true) {
        const int32_t j = table[h];
        if (j == -1) break;
        if (same_bits(X[j], x) && same_bits(Y[j], y) && same_bits(Z[j], z)) {
          nn[q] = j;
          miss = false;
          break;
        }
        h = (h + 1) & tmask;
      }
    }
  }
  const uint64_t mk = __ballot(miss);
  if (mk == 0) return;
  const int lane = threadIdx.x & 63;
  const int leader = __ffsll((unsigned long long)mk) - 1;
  uint32_t base = 0;
  if (lane == leader) base = atomicAdd(n_rest, (uint32_t)__popcll(mk));
  base = __shfl(base, leader, 64);
  const int below = __builtin_amdgcn_mbcnt_hi((uint32_t)(mk >> 32),
                                              __builtin_amdgcn_mbcnt_lo((uint32_t)mk, 0u));
  if (miss) rest[base + below] = q;
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

// component sizes: lanes of a wave sharing a root (neighbours in cell order mostly do) add
// with one atomic, so a large component does not serialise on its counter
__global__ __launch_bounds__(kBS) void k_cc_count(int32_t* parent, int n,
                                                  uint32_t* __restrict__ size) {
  const int u = blockIdx.x * kBS + threadIdx.x;
  const int r = u < n ? uf_find(parent, u) : -1;
  bool todo = u < n;
  const int lane = threadIdx.x & 63;
  uint64_t act = __ballot(todo);
  while (act) {
    const int leader = __ffsll((unsigned long long)act) - 1;
    const int rl = __shfl(r, leader, 64);
    const uint64_t same = __ballot(todo && r == rl);
    if (lane == leader) atomicAdd(&size[rl], (uint32_t)__popcll(same));
    if (r == rl) todo = false;
    act = __ballot(todo);
  }
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


}  // namespace

size_t pip_scan_tmp_bytes(size_t count) {
  size_t t = 0;
  (void)hipcub::DeviceScan::ExclusiveSum(nullptr, t, (const uint32_t*)nullptr, (uint32_t*)nullptr,
                                         count);
  return t;
}

int pip_blocks(int n) { return (int)cdiv(n, kBS); }

hipError_t launch_pip_candidates(const float* X, const float* Y, const float* Z, int n,
                                 const uint8_t* processed, const float4* planes, int n_planes,
                                 float t_dist, uint32_t* bcnt, uint32_t* boff, void* tmp,
                                 size_t tmp_bytes, int32_t* cand, uint32_t* offs, hipStream_t s) {
  if (n <= 0 || n_planes <= 0) return hipSuccess;
  const int nblk = pip_blocks(n);
  const dim3 g(nblk, n_planes);
  if (!cand) {
    hipLaunchKernelGGL(k_pip_count, g, dim3(kBS), 0, s, X, Y, Z, n, processed, planes, t_dist,
                       bcnt);
    size_t t = tmp_bytes;
    hipError_t e = hipcub::DeviceScan::ExclusiveSum(tmp, t, bcnt, boff,
                                                    (size_t)n_planes * nblk, s);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_pip_ranges, dim3(cdiv(n_planes + 1, 64)), dim3(64), 0, s, bcnt, boff,
                       nblk, n_planes, offs);
    return hipGetLastError();
  }
  hipLaunchKernelGGL(k_pip_fill, g, dim3(kBS), 0, s, X, Y, Z, n, processed, planes, t_dist, boff,
                     cand);
  return hipGetLastError();
}

size_t pip_sort_tmp_bytes(int count) {
  size_t t = 0;
  (void)hipcub::DeviceRadixSort::SortPairs(nullptr, t, (const uint64_t*)nullptr,
                                           (uint64_t*)nullptr, (const int32_t*)nullptr,
                                           (int32_t*)nullptr, count);
  return t;
}

hipError_t launch_pip_sort(const int32_t* cand, int count, const uint32_t* offs, int n_planes,
                           int max_count, const float* X, const float* Y, const float* Z,
                           float4 lo_scale, uint64_t* keys, uint64_t* keys_alt, int32_t* cand_out,
                           void* tmp, size_t tmp_bytes, hipStream_t s) {
  if (count <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_pip_keys, dim3(cdiv(max_count, kBS), n_planes), dim3(kBS), 0, s, cand, offs,
                     X, Y, Z, lo_scale, keys);
  int end_bit = 42;
  while (end_bit < 64 && ((uint64_t)1 << (end_bit - 42)) < (uint64_t)n_planes) ++end_bit;
  size_t t = tmp_bytes;
  return hipcub::DeviceRadixSort::SortPairs(tmp, t, keys, keys_alt, cand, cand_out, count, 0,
                                            end_bit, s);
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
                     int n_planes, int max_count, int n, uint8_t* absorbed, uint8_t* processed,
                     uint32_t* abs_cnt, hipStream_t s) {
  if (max_count <= 0 || n_planes <= 0) return;
  hipLaunchKernelGGL(k_pip_mark, dim3(cdiv(max_count, kBS), n_planes), dim3(kBS), 0, s, cand, mask,
                     offs, n, absorbed, processed, abs_cnt);
}

void launch_xyz_insert(const float* X, const float* Y, const float* Z, int n, int32_t* table,
                       uint32_t tmask, hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_xyz_insert, dim3(cdiv(n, kBS)), dim3(kBS), 0, s, X, Y, Z, n, table, tmask);
}

void launch_xyz_lookup(const float* qx, const float* qy, const float* qz, int m,
                       const int32_t* table, uint32_t tmask, const float* X, const float* Y,
                       const float* Z, int32_t* nn, int32_t* rest, uint32_t* n_rest,
                       hipStream_t s) {
  if (m <= 0) return;
  hipLaunchKernelGGL(k_xyz_lookup, dim3(cdiv(m, kBS)), dim3(kBS), 0, s, qx, qy, qz, m, table, tmask,
                     X, Y, Z, nn, rest, n_rest);
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
