// spatial.hip -- Morton-ordered copy of the active points, tile / super-tile bounding spheres and
// k_score_pruned, the pruned countWithinDistance (see spatial.hpp for the argument).
#include "spatial.hpp"

#include <hip/hip_ext.h>
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <climits>
#include <cmath>
#include <cstdlib>

#include "dev_common.hpp"
#include "np_dev.hpp"
#include "pick_dev.hpp"

namespace dlg {

namespace {

__device__ __forceinline__ uint32_t spread10(uint32_t v) {  // 10 bits -> every third bit
  v &= 0x3FFu;
  v = (v | (v << 16)) & 0x030000FFu;
  v = (v | (v << 8)) & 0x0300F00Fu;
  v = (v | (v << 4)) & 0x030C30C3u;
  v = (v | (v << 2)) & 0x09249249u;
  return v;
}

__device__ __forceinline__ uint32_t quant10(float v, float a) {
  if (!(a > 0.0f)) return 0u;
  const float t = (v + a) * (1023.99f / (2.0f * a));
  return (uint32_t)fminf(fmaxf(t, 0.0f), 1023.0f);
}

// Hilbert index of the 10-bit cell (x, y, z) (Skilling's transpose form: undo the excess work of
// each bit level's Gray-code reflections, Gray-decode, then interleave the three words as a
// Morton key would).  Consecutive keys are face-adjacent cells, so a run of 32 points -- a tile --
// stays in one connected patch of the curve: no Z-order jump across the cloud inside a tile.
// (tools: the curve's unit steps and the tiles' sphere radii checked by a numpy model.)
__device__ __forceinline__ uint32_t hilbert10(uint32_t x, uint32_t y, uint32_t z) {
  uint32_t X0 = x, X1 = y, X2 = z;
#pragma unroll
  for (uint32_t Q = 1u << 9; Q > 1u; Q >>= 1) {
    const uint32_t P = Q - 1u;
    if (X0 & Q) X0 ^= P;
    if (X1 & Q) X0 ^= P;
    else { const uint32_t t = (X0 ^ X1) & P; X0 ^= t; X1 ^= t; }
    if (X2 & Q) X0 ^= P;
    else { const uint32_t t = (X0 ^ X2) & P; X0 ^= t; X2 ^= t; }
  }
  X1 ^= X0;
  X2 ^= X1;
  uint32_t t = 0u;
#pragma unroll
  for (uint32_t Q = 1u << 9; Q > 1u; Q >>= 1)
    if (X2 & Q) t ^= Q - 1u;
  X0 ^= t; X1 ^= t; X2 ^= t;
  return (spread10(X0) << 2) | (spread10(X1) << 1) | spread10(X2);
}

// (also writes the points as (x, y, z, 0) records: k_gather_order and k_ucompact gather from
// them, one 16-byte record per point instead of three scattered floats)
__global__ void k_morton_keys(PointsView src, float ax, float ay, float az,
                              uint32_t* __restrict__ keys, int32_t* __restrict__ idx,
                              int32_t* __restrict__ n_nonfinite, float4* __restrict__ aos,
                              int hilbert) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  bool nf = false;
  if (i < src.n) {
    const float x = src.x[i], y = src.y[i], z = src.z[i];
    aos[i] = make_float4(x, y, z, 0.0f);
    uint32_t k = 0xFFFFFFFFu;
    if (isfinite(x) && isfinite(y) && isfinite(z))
      k = hilbert ? hilbert10(quant10(x, ax), quant10(y, ay), quant10(z, az))
                  : spread10(quant10(x, ax)) | (spread10(quant10(y, ay)) << 1) | (spread10(quant10(z, az)) << 2);
    else
      nf = true;
    keys[i] = k;
    idx[i] = (int32_t)i;
  }
  const uint64_t m = ballot(nf);
  if (m && (threadIdx.x & (kWave - 1)) == 0) atomicAdd(n_nonfinite, (int32_t)__popcll(m));
}

__global__ void k_gather_order(const float4* __restrict__ src, const int32_t* __restrict__ order,
                               int64_t n, PointsOut dst) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int32_t k = order[i];
  const float4 v = src[k];
  dst.x[i] = v.x;
  dst.y[i] = v.y;
  dst.z[i] = v.z;
  dst.gid[i] = k;  // the Morton copy's "gid" is the pristine index (lean-list rounds stamp it)
}

// Tile sphere: centre = midpoint of the tile's bounding box, radius = max |p - c| (float)
// inflated by 2^-18 (covers the few roundings of the distance evaluation).  Super sphere: centre
// = midpoint of the super box, radius = max over its tiles of |c_t - C| + r_t, inflated the same
// way.
// k_sphere_bounds3: two lanes per tile (lane l: tile l & 31, points 16 (l >> 5) .. + 16), 32
// tiles (two super-tiles) a wave staged in LDS with coalesced loads (padded rows: no bank
// conflicts), the two halves' boxes and radii combined by one shuffle, then the 16 lanes of a
// super-tile combine their spheres.  (Round 5's k_sphere_bounds2 took one lane per tile and 64
// tiles a wave: 25 KB of LDS a workgroup, 6 workgroups per CU, 20.5 us per round at C3 against
// 17.8 here; min / max are exact in any order, so the spheres are the same bit for bit.)
constexpr int kSb3Tiles = 32;
constexpr int kSb3Pts = kSb3Tiles * kTileP;  // points per wave (32 tiles)
__global__ __launch_bounds__(64) void k_sphere_bounds3(const float* __restrict__ X,
                                                       const float* __restrict__ Y,
                                                       const float* __restrict__ Z, int64_t n_arg,
                                                       const int32_t* __restrict__ n_dev,
                                                       float4* __restrict__ tiles,
                                                       float4* __restrict__ supers) {
  __shared__ float s_p[3][kSb3Pts + kSb3Pts / kTileP];  // row t: 33 floats
  const int64_t n = n_dev ? (int64_t)*n_dev : n_arg;
  const int lane = threadIdx.x;
  const int64_t base = (int64_t)blockIdx.x * kSb3Pts;
  if (base >= n) return;
  const int cnt = (int)min<int64_t>(kSb3Pts, n - base);
  constexpr int kPer = kSb3Pts / kWave;
  float vx[kPer], vy[kPer], vz[kPer];
#pragma unroll
  for (int k = 0; k < kPer; ++k) {
    const int64_t e = base + min(k * kWave + lane, cnt - 1);
    vx[k] = X[e]; vy[k] = Y[e]; vz[k] = Z[e];
  }
#pragma unroll
  for (int k = 0; k < kPer; ++k) {
    const int i = k * kWave + lane, r = i + i / kTileP;
    s_p[0][r] = vx[k]; s_p[1][r] = vy[k]; s_p[2][r] = vz[k];
  }
  __syncthreads();
  const int tile = lane & (kSb3Tiles - 1), half = lane >> 5;
  const int np = min(kTileP, cnt - tile * kTileP);  // the tile's size (<= 0: none)
  const int p0 = half * (kTileP / 2), p1 = min(np, p0 + kTileP / 2);  // this lane's points
  const float* px = &s_p[0][tile * (kTileP + 1)];
  const float* py = &s_p[1][tile * (kTileP + 1)];
  const float* pz = &s_p[2][tile * (kTileP + 1)];
  float x0 = INFINITY, y0 = INFINITY, z0 = INFINITY, x1 = -INFINITY, y1 = -INFINITY, z1 = -INFINITY;
  for (int i = p0; i < p1; ++i) {
    const float x = px[i], y = py[i], z = pz[i];
    x0 = fminf(x0, x); y0 = fminf(y0, y); z0 = fminf(z0, z);
    x1 = fmaxf(x1, x); y1 = fmaxf(y1, y); z1 = fmaxf(z1, z);
  }
  x0 = fminf(x0, __shfl_xor(x0, 32)); y0 = fminf(y0, __shfl_xor(y0, 32));
  z0 = fminf(z0, __shfl_xor(z0, 32)); x1 = fmaxf(x1, __shfl_xor(x1, 32));
  y1 = fmaxf(y1, __shfl_xor(y1, 32)); z1 = fmaxf(z1, __shfl_xor(z1, 32));
  const float cx = 0.5f * (x0 + x1), cy = 0.5f * (y0 + y1), cz = 0.5f * (z0 + z1);
  float d = 0.0f;
  for (int i = p0; i < p1; ++i) {
    const float dx = px[i] - cx, dy = py[i] - cy, dz = pz[i] - cz;
    d = fmaxf(d, sqrtf(dx * dx + dy * dy + dz * dz));
  }
  d = fmaxf(d, __shfl_xor(d, 32));
  const float rt = d * (1.0f + 0x1p-18f) + 1e-30f;
  const int64_t t = (int64_t)blockIdx.x * kSb3Tiles + tile;
  if (np > 0 && half == 0) tiles[t] = make_float4(cx, cy, cz, rt);
  // super-tile of each kSuperTiles tiles (both halves hold the same values): box over its tiles,
  // then max |c_t - C| + r_t
  float bx0 = x0, by0 = y0, bz0 = z0, bx1 = x1, by1 = y1, bz1 = z1;
#pragma unroll
  for (int o = 1; o < kSuperTiles; o <<= 1) {
    bx0 = fminf(bx0, __shfl_xor(bx0, o)); by0 = fminf(by0, __shfl_xor(by0, o));
    bz0 = fminf(bz0, __shfl_xor(bz0, o));
    bx1 = fmaxf(bx1, __shfl_xor(bx1, o)); by1 = fmaxf(by1, __shfl_xor(by1, o));
    bz1 = fmaxf(bz1, __shfl_xor(bz1, o));
  }
  const float Cx = 0.5f * (bx0 + bx1), Cy = 0.5f * (by0 + by1), Cz = 0.5f * (bz0 + bz1);
  float R = 0.0f;
  if (np > 0) {
    const float dx = cx - Cx, dy = cy - Cy, dz = cz - Cz;
    R = sqrtf(dx * dx + dy * dy + dz * dz) + rt;
  }
#pragma unroll
  for (int o = 1; o < kSuperTiles; o <<= 1) R = fmaxf(R, __shfl_xor(R, o));
  const int sub = tile / kSuperTiles;
  if (half == 0 && (tile % kSuperTiles) == 0 && sub * kSuperP < cnt)
    supers[(int64_t)blockIdx.x * (kSb3Tiles / kSuperTiles) + sub] =
        make_float4(Cx, Cy, Cz, R * (1.0f + 0x1p-18f) + 1e-30f);
}

// ---------------------------------------------------------------------------------------------
// Pruned countWithinDistance in two launches:
//   k_prune_supers : every plane against every super-tile sphere (planes in LDS, 1024 threads =
//                    4 planes per thread per super-tile); the planes that may hold an inlier go
//                    to the super-tile's list lp[s * D ...], their number to lp_n[s];
//   k_score_tiles_rl : per tile, the planes of its super-tile's list are tested against the tile
//                    sphere, the near ones appended to the wave's ring, and every 32 queued
//                    planes (and the remainder) scored against the tile's 32 points as one
//                    32 x 32 bf16 matrix-core block with exact band re-decision; per-plane
//                    counts in LDS, flushed once per workgroup.
// A (sphere, plane) pair is ruled out only when fl(|h|) > (margin + r)(1 + 2^-20), i.e. the
// exact distance of the plane to the sphere centre exceeds cthr + r + 2 e_max: no point of the
// sphere can then pass PCL's test (spatial.hpp).
//
// Block scoring relative to the tile centre c: A rows hold the split of p - c (|p - c| <= r),
// the B column's d slots the split of h = n.c + d (double, rounded once to float).  The matrix
// cores then add small terms, so |D - pcl_dot| is dominated by PCL's own rounding (4.1 u S)
// and the re-decision band is ~15x narrower than k_score_bf16's 64 u S.
constexpr int kPrBS = 1024;
// XCD x's super-tiles of list-length class b (spatial.hpp: the work area after the lengths)
__device__ __forceinline__ int32_t* ord_of(const int32_t* lp_n, int64_t nsup, int x, int b) {
  const int64_t cap = (nsup + 7) / 8;
  return const_cast<int32_t*>(lp_n) + nsup + ((int64_t)x * kPwBuckets + b) * cap;
}
constexpr int kPrWaves = kPrBS / kWave;

// One workgroup per "hyper" of H consecutive super-tiles (a compact region in Morton order): the
// bounding sphere of their spheres first takes the D planes down to the few near it (LDS list),
// then each super-tile tests only those.  A plane ruled out by the hyper sphere has no PCL
// inlier anywhere in it (the same test on a sphere that bounds every super-tile sphere), so the
// super-tile lists keep every plane that can score.
__global__ __launch_bounds__(kPrBS) void k_prune_supers(const float4* __restrict__ supers,
                                                        int nsup, const HypRec* __restrict__ hyps,
                                                        int D, int ls, float margin, int H,
                                                        uint16_t* __restrict__ lp,
                                                        int32_t* __restrict__ lp_n,
                                                        int32_t* __restrict__ work, int order,
                                                        float4* __restrict__ cn) {
  __shared__ float4 s_cf[kMaxHypPerLaunch];
  __shared__ uint16_t s_hl[kMaxHypPerLaunch];  // the planes near this hyper's sphere
  __shared__ float4 s_sp[kWave];
  __shared__ float4 s_hyp;
  __shared__ int s_nh;
  const int t = threadIdx.x, lane = t & (kWave - 1);
  if (blockIdx.x == 0 && t < 8) work[t * kPruneWorkStride] = 0;  // the scorers' item counters
  if (cn && blockIdx.x == gridDim.x - 1)  // (NORMAL_PLANE: Eigen's normalized() of each plane)
    for (int j = t; j < D; j += kPrBS) {
      const HypRec h = hyps[j];
      cn[j] = eigen_normalized3(h.a, h.b, h.c, 0.0f);
    }
  for (int j = t; j < D; j += kPrBS) {
    const HypRec h = hyps[j];
    s_cf[j] = make_float4(h.a, h.b, h.c, h.d);
  }
  for (int64_t h0 = (int64_t)blockIdx.x * H; h0 < nsup; h0 += (int64_t)gridDim.x * H) {
    const int ns = (int)min<int64_t>(H, nsup - h0);
    __syncthreads();  // (the previous hyper's s_sp / s_hl are no longer read)
    if (t < kWave) {  // wave 0: the hyper sphere (box midpoint, max |c_s - C| + r_s, inflated)
      const bool v = lane < ns;
      const float4 sp = v ? supers[h0 + lane] : make_float4(0.f, 0.f, 0.f, 0.f);
      if (v) s_sp[lane] = sp;
      float x0 = v ? sp.x - sp.w : INFINITY, y0 = v ? sp.y - sp.w : INFINITY;
      float z0 = v ? sp.z - sp.w : INFINITY, x1 = v ? sp.x + sp.w : -INFINITY;
      float y1 = v ? sp.y + sp.w : -INFINITY, z1 = v ? sp.z + sp.w : -INFINITY;
#pragma unroll
      for (int o = 1; o < kWave; o <<= 1) {
        x0 = fminf(x0, __shfl_xor(x0, o)); y0 = fminf(y0, __shfl_xor(y0, o));
        z0 = fminf(z0, __shfl_xor(z0, o)); x1 = fmaxf(x1, __shfl_xor(x1, o));
        y1 = fmaxf(y1, __shfl_xor(y1, o)); z1 = fmaxf(z1, __shfl_xor(z1, o));
      }
      const float Cx = 0.5f * (x0 + x1), Cy = 0.5f * (y0 + y1), Cz = 0.5f * (z0 + z1);
      float R = 0.0f;
      if (v) {
        const float dx = sp.x - Cx, dy = sp.y - Cy, dz = sp.z - Cz;
        R = sqrtf(dx * dx + dy * dy + dz * dz) + sp.w;
      }
#pragma unroll
      for (int o = 1; o < kWave; o <<= 1) R = fmaxf(R, __shfl_xor(R, o));
      if (lane == 0) {
        s_hyp = make_float4(Cx, Cy, Cz, R * (1.0f + 0x1p-18f) + 1e-30f);
        s_nh = 0;
      }
    }
    __syncthreads();
    const float4 hs = s_hyp;
    for (int b = 0; b < D; b += kPrBS) {  // block-uniform trip count
      const int j = b + t;
      const bool near = j < D && sphere_near(s_cf[j], hs, margin);  // NaN planes: never near
      const uint64_t m = ballot(near);
      if (m) {
        int base = 0;
        if (lane == 0) base = atomicAdd(&s_nh, (int)__popcll(m));
        base = __shfl(base, 0);
        if (near) s_hl[base + lanes_below(m)] = (uint16_t)j;
      }
    }
    __syncthreads();
    // the near planes against the super-tiles: one wave per super-tile (no workgroup barrier),
    // list positions from the wave's own running count
    const int nh = s_nh, w = t / kWave;
    for (int k = w; k < ns; k += kPrWaves) {
      const float4 sp = s_sp[k];
      uint16_t* out = lp + (h0 + k) * ls;
      int cnt = 0;
      for (int b = 0; b < nh; b += kWave) {
        const int i = b + lane;
        const int j = i < nh ? (int)s_hl[i] : 0;
        const bool near = i < nh && sphere_near(s_cf[j], sp, margin);
        const uint64_t m = ballot(near);
        if (near) out[cnt + lanes_below(m)] = (uint16_t)j;
        cnt += (int)__popcll(m);
      }
      if (lane == 0) {
        lp_n[h0 + k] = cnt;
        if (order) {  // (k_score_tiles_ex's claim order: the longest lists' class first)
          const int64_t s = h0 + k, cap = ((int64_t)nsup + 7) / 8;
          const int x = (int)(s & 7), b = pw_class(cnt);
          ord_of(lp_n, nsup, x, b)[atomicAdd(&work[kPwBucket + x * kPruneWorkStride + b], 1)] =
              (int32_t)s;
          (void)cap;
        }
      }
    }
  }
}

// ---------------------------------------------------------------------------------------------
// k_score_tiles_rl: no global load on the group path.  A work item (2 consecutive tiles of one
// super-tile) loads its super-tile's plane
// list once into registers (up to kListCap entries, two uint16 per dword, 8 dwords per lane);
// per tile the list is tested against the tile sphere from registers + LDS (packed FMAs, two
// entries per lane), near planes go to the wave's LDS ring, and every 32 queued planes are
// scored with B columns split from the LDS coefficients (exact bf16 split of a, b, c and of the
// double-evaluated h = n.c + d) and a rounding band computed from S = |a| ax + |b| ay + |c| az +
// |d| (4.25 u S >= the 4.21 u S of k_prep_bf16's band x 0.065).  The next tile's header and
// points are loaded after the current tile's A operand is built (vmcnt is in order: the wait
// for this tile's data never waits for the prefetch).  LDS: coefficients 64 KB + counts 8 KB +
// rings 8 KB.  (An 80 KB per-plane LDS record of the B splits, assembled with byte permutes,
// measured no faster.)
constexpr int kListRegs = 8;
constexpr int kListCap = kListRegs * 2 * kWave;  // 1024 entries
constexpr int kRing2 = 512;                       // >= 31 queued + 256 appended per list step

// NPM: SACMODEL_NORMAL_PLANE (PCL's exact prefilter b = (1 - w) d_euclid < thr as the per-point
// float compare d_euclid < lim, k_score_np; passing pairs queued per wave and decided with full
// lanes in double as in k_score_np), the spheres ruled out with the margin of the cloud's
// largest lim; plane model otherwise.
template <int BS, bool NPM>
__global__ __launch_bounds__(BS) void k_score_tiles_rl(
    const float* __restrict__ X, const float* __restrict__ Y, const float* __restrict__ Z,
    int n, const float4* __restrict__ tiles, const uint16_t* __restrict__ lp, int ls,
    const int32_t* __restrict__ lp_n, int32_t* __restrict__ work, int blk_cap, int chunk, int xcd,
    const HypRec* __restrict__ hyps, int D, float cthr, float margin, float ax, float ay,
    float az, int32_t* __restrict__ counts, unsigned long long* __restrict__ stats,
    const float4* __restrict__ NRM, double lambda, double thr, PickArgs pick_args) {
  __shared__ float4 s_cf[kMaxHypPerLaunch];
  __shared__ uint32_t s_cnt[kMaxHypPerLaunch / 2];  // 16-bit halves: <= 65535 points per workgroup
  __shared__ uint16_t s_ring[(BS / kWave)][kRing2];
  __shared__ unsigned long long s_st[6];
  __shared__ int s_taken;  // items this workgroup has claimed (<= blk_cap: 16-bit counters)
  // NPM: the tile's (normalised normal, curvature) per point, and the per-wave queue of
  // prefilter-passing (point slot | plane << 5, b = (1 - w) d_euclid) pairs
  constexpr int kQ = NPM ? 128 : 1;
  __shared__ float4 s_pn[NPM ? BS / kWave : 1][NPM ? kTileP : 1];
  __shared__ uint32_t s_qk[NPM ? BS / kWave : 1][kQ];
  __shared__ double s_qb[NPM ? BS / kWave : 1][kQ];
  const int lane = threadIdx.x & (kWave - 1), wv = threadIdx.x / kWave;
  const int r32 = lane & 31, hh = lane >> 5;
  for (int j = threadIdx.x; j < D; j += BS) {
    const HypRec h = hyps[j];
    s_cf[j] = make_float4(h.a, h.b, h.c, h.d);
  }
  if (threadIdx.x == 0) s_taken = 0;
  for (int j = threadIdx.x; j < kMaxHypPerLaunch / 2; j += BS) s_cnt[j] = 0u;
  if (threadIdx.x < 6) s_st[threadIdx.x] = 0;
  __syncthreads();
  const f32x16 zero = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  const int ntiles = (n + kTileP - 1) / kTileP;
  const int nitems = (ntiles + chunk - 1) / chunk;
  uint16_t* ring = s_ring[wv];
  // a workgroup owns items blockIdx.x + k * gridDim.x (interleaved over the cloud); its waves
  // claim them dynamically through an LDS counter (balances the waves of a CU; a global
  // counter measured 3x slower: one contended L2 atomic per item; dealing super-tiles to the
  // workgroups of one XCD so that a plane list is fetched into one L2 only: no faster), one
  // claim ahead.  The grid keeps each workgroup <= blk_cap items (16-bit LDS counters).
  // xcd (gridDim.x a multiple of 8): the items of a super-tile go to workgroups of one XCD
  // (workgroups are dealt round-robin over the 8 XCDs), so its plane list is fetched into one L2
  // instead of eight: XCD x takes super-tiles x, x + 8, ...; their items are dealt round-robin
  // to its gridDim.x / 8 workgroups.  Either mapping visits every item once, in increasing order
  // per workgroup (the first index past nitems ends the workgroup's loop).
  const int ips = kSuperTiles / chunk;  // items per super-tile
  auto claim = [&]() -> int {
    int v = nitems;
    if (lane == 0) {
      const int k = atomicAdd(&s_taken, 1);
      if (k < blk_cap) {
        if (xcd) {
          const int64_t l = (int64_t)k * (gridDim.x >> 3) + (blockIdx.x >> 3);
          const int64_t s = (int64_t)(blockIdx.x & 7) + 8 * (l / ips);
          v = (int)min((int64_t)nitems, s * ips + l % ips);
        } else {
          v = (int)min((int64_t)nitems, (int64_t)blockIdx.x + (int64_t)k * gridDim.x);
        }
      }
    }
    return __builtin_amdgcn_readfirstlane(__shfl(v, 0));  // (uniform: scalar control flow)
  };
  (void)work;
  int it_next = claim();
  for (;;) {
    const int it = it_next;
    if (it >= nitems) break;
    it_next = claim();
    const int t0 = it * chunk, t_end = min(ntiles, t0 + chunk);
    const int sidx = t0 / kSuperTiles;  // kSuperTiles % chunk == 0: one super-tile per item
    const int nlp = __builtin_amdgcn_readfirstlane(lp_n[sidx]);
    const uint32_t* lw = reinterpret_cast<const uint32_t*>(lp + (int64_t)sidx * ls);
    // the item's tiles take the list kListCap entries at a time (one pass unless it is long)
#pragma unroll 1
    for (int lb = 0; lb < nlp; lb += kListCap) {
    const int le = min(nlp, lb + kListCap);
    uint32_t L[kListRegs];
#pragma unroll
    for (int k = 0; k < kListRegs; ++k) {
      const int e = lb + 2 * (lane + k * kWave);
      L[k] = e < le ? lw[(lb >> 1) + lane + k * kWave] : 0u;
      if (e + 1 >= le) L[k] &= 0xFFFFu;  // (past the end: plane 0, never counted)
    }
    // first tile of the item
    float4 tb = tiles[t0];
    float x = 0.f, y = 0.f, z = 0.f;
    float4 nn = make_float4(0.f, 0.f, 0.f, 0.f);
    {
      const int64_t p = (int64_t)t0 * kTileP + r32;
      if (p < n) {
        x = X[p]; y = Y[p]; z = Z[p];
        if constexpr (NPM) nn = NRM[p];
      }
    }
    for (int t = t0; t < t_end; ++t) {
      const int64_t p0 = (int64_t)t * kTileP;
      const bool valid = p0 + r32 < n;
      const float tlim = prune_lim(margin, tb.w);
      if (stats && lane == 0) { atomicAdd(&s_st[2], 1ull); atomicAdd(&s_st[1], (unsigned long long)nlp); }
      // A operand (the tile's points relative to its centre) before the next tile's loads are
      // issued: waiting for this tile's data then never waits for the prefetch (vmcnt is in order)
      const bool bad = ballot(!valid || !(isfinite(x) && isfinite(y) && isfinite(z))) != 0;
      u32x4 a1 = {0u, 0u, 0u, 0u}, a2 = {0u, 0u, 0u, 0u};
      float plim = -INFINITY;  // NPM: d_euclid < plim passes PCL's prefilter
      double pomw = 0.0;
      if constexpr (NPM) {
        const double w = lambda * (1.0 - (double)nn.w);
        pomw = 1.0 - w;
        // (NaN w: the exact test is NaN < thr, never an inlier)
        plim = valid && w == w ? np_de_limit(w, thr) : -INFINITY;
        if (hh == 0) s_pn[wv][r32] = nn;
      } else {
        const float dx = valid ? x - tb.x : 0.f, dy = valid ? y - tb.y : 0.f;
        const float dz = valid ? z - tb.z : 0.f;
        const Split3 sx = split3(dx), sy = split3(dy), sz = split3(dz);
        if (hh == 0) {
          a1 = u32x4{pk(sx.p1, sx.p1), pk(sx.p2, sx.p1), pk(sx.p3, sx.p2), pk(sy.p1, sy.p1)};
          a2 = u32x4{pk(sz.p3, sz.p2), pk(kBf16One, kBf16One), pk(kBf16One, 0u), 0u};
        } else {
          a1 = u32x4{pk(sy.p2, sy.p1), pk(sy.p3, sy.p2), pk(sz.p1, sz.p1), pk(sz.p2, sz.p1)};
          a2 = u32x4{0u, 0u, 0u, 0u};
        }
      }
      // prefetch the next tile of the item
      float4 tb_n = make_float4(0.f, 0.f, 0.f, 0.f);
      float xn = 0.f, yn = 0.f, zn = 0.f;
      float4 nn_n = make_float4(0.f, 0.f, 0.f, 0.f);
      if (t + 1 < t_end) {
        tb_n = tiles[t + 1];
        const int64_t p = (int64_t)(t + 1) * kTileP + r32;
        if (p < n) {
          xn = X[p]; yn = Y[p]; zn = Z[p];
          if constexpr (NPM) nn_n = NRM[p];
        }
      }
      int nq = 0, head = 0;
      int qn = 0;  // NPM queue length (wave-uniform)
      // NPM: decide the first m queued pairs with full lanes (k_score_np's np_full), keep the rest
      auto drain = [&](int m) {
        __builtin_amdgcn_wave_barrier();
        if (lane < m) {
          const uint32_t e = s_qk[wv][lane];
          const float4 pn = s_pn[wv][e & 31u];
          const int jj = (int)(e >> 5);
          const float4 cf = s_cf[jj];
          const float4 cn = eigen_normalized3(cf.x, cf.y, cf.z, 0.0f);
          const double w = lambda * (1.0 - (double)pn.w);
          if (np_full(cn, pn, w, s_qb[wv][lane], thr))
            atomicAdd(&s_cnt[jj >> 1], 1u << (16 * (jj & 1)));
        }
        const int rest = qn - m;
        uint32_t mk = 0;
        double mb = 0.0;
        if (lane < rest) {
          mk = s_qk[wv][m + lane];
          mb = s_qb[wv][m + lane];
        }
        __builtin_amdgcn_wave_barrier();
        if (lane < rest) {
          s_qk[wv][lane] = mk;
          s_qb[wv][lane] = mb;
        }
        qn = rest;
      };
      auto score = [&](int m) {
        if (stats && lane == 0) { atomicAdd(&s_st[3], 1ull); atomicAdd(&s_st[4], (unsigned long long)m); }
        const bool col = r32 < m;
        const int j = col ? (int)ring[(head + r32) & (kRing2 - 1)] : 0;
        if constexpr (NPM) {
          // lane: point r32 of the tile, planes hh * 16 .. hh * 16 + 15 of the group
          (void)j;
#pragma unroll 1
          for (int q = 0; q < 16; ++q) {
            const int kq = hh * 16 + q;
            const bool cq = kq < m;
            const int jq = cq ? (int)ring[(head + kq) & (kRing2 - 1)] : 0;
            const float4 cq4 = s_cf[jq];
            const float de = np_deuclid(cq4, x, y, z);
            const bool near = cq && de < plim;
            const uint64_t mm = ballot(near);
            if (near) {
              const int pos = qn + lanes_below(mm);
              s_qk[wv][pos] = (uint32_t)r32 | ((uint32_t)jq << 5);
              s_qb[wv][pos] = pomw * (double)de;
            }
            qn += (int)__popcll(mm);
            if (qn >= kWave) drain(kWave);
          }
          head += m;
          return;
        }
        const float4 cf = s_cf[j];
        // B column of plane j (k_prep_bf16's layout, d slots = split of h = n.c + d), assembled
        // from the LDS record with byte permutes
        u32x4 b1 = {0u, 0u, 0u, 0u}, b2 = {0u, 0u, 0u, 0u};
        float w = 0.0f;
        if (col) {
          const double hd = __builtin_fma((double)cf.x, (double)tb.x,
                                          __builtin_fma((double)cf.y, (double)tb.y,
                                                        __builtin_fma((double)cf.z, (double)tb.z, (double)cf.w)));
          const float hf = (float)hd;
          float S;
          {
            const Split3 sa = split3(cf.x), sb = split3(cf.y), sc = split3(cf.z);
            if (hh == 0) {
              const Split3 sh = split3(hf);
              b1 = u32x4{pk(sa.p1, sa.p2), pk(sa.p1, sa.p3), pk(sa.p1, sa.p2), pk(sb.p1, sb.p2)};
              b2 = u32x4{pk(sc.p1, sc.p2), pk(sh.p1, sh.p2), pk(sh.p3, 0u), 0u};
            } else {
              b1 = u32x4{pk(sb.p1, sb.p3), pk(sb.p1, sb.p2), pk(sc.p1, sc.p2), pk(sc.p1, sc.p3)};
            }
            S = __builtin_fmaf(fabsf(cf.x), ax, __builtin_fmaf(fabsf(cf.y), ay,
                               __builtin_fmaf(fabsf(cf.z), az, fabsf(cf.w))));
          }
          // |D - pcl_dot| <= 4.1 u S + 44 u (|n|_1 r + |h|) (PCL rounding + centring); S in float
          // (<= 4 roundings, possibly rounded up to bf16) times 4.25 u covers the 4.21 u S there
          w = __builtin_fmaf(0x1.1p-22f, S, 3.0e-6f * __builtin_fmaf(1.8f, tb.w, fabsf(hf))) + 1e-8f;
          if (!(w <= INFINITY)) w = INFINITY;  // NaN (0 x inf): re-decide everything
        } else if (hh == 0) {
          b2 = u32x4{0u, pk(0x4000u, 0u), 0u, 0u};  // not a plane: D = 2, never counted
        }
        f32x16 Dv = __builtin_amdgcn_mfma_f32_32x32x16_bf16(as_bf16x8(a1), as_bf16x8(b1), zero, 0, 0, 0);
        Dv = __builtin_amdgcn_mfma_f32_32x32x16_bf16(as_bf16x8(a2), as_bf16x8(b2), Dv, 0, 0, 0);
        uint32_t acc = 0;
        float mn = INFINITY;
#pragma unroll
        for (int i = 0; i < 16; i += 4) {
          const float r0 = fabsf(Dv[i]) - cthr, r1 = fabsf(Dv[i + 1]) - cthr;
          const float r2 = fabsf(Dv[i + 2]) - cthr, r3 = fabsf(Dv[i + 3]) - cthr;
          acc = count4(r0, r1, r2, r3, acc);
          mn = min3_abs(mn, r0, r1);
          mn = min3_abs(mn, r2, r3);
        }
        const bool need = bad || mn <= w;
        if (ballot(need)) {  // rare: re-decide the band elements in PCL op order
          if (stats && lane == 0) atomicAdd(&s_st[5], 1ull);
          uint32_t bm = 0u, am = 0u;  // per lane: band elements, and their approximate verdicts
          if (need) {
#pragma unroll
            for (int i = 0; i < 16; ++i) {
              const float ri = fabsf(Dv[i]) - cthr;
              bm |= (uint32_t)(bad || fabsf(ri) <= w) << i;
              am |= (__float_as_uint(ri) >> 31) << i;
            }
          }
          while (ballot(bm != 0u)) {  // one band element per lane per pass
            const int i = bm ? __builtin_ctz(bm) : 0;
            const bool inb = bm != 0u;
            bm &= bm - 1u;
            const int row = (i & 3) + 8 * (i >> 2) + 4 * hh;
            const float px = __shfl(x, row), py = __shfl(y, row), pz = __shfl(z, row);
            const bool ex = p0 + row < n && fabsf(pcl_dot(cf.x, cf.y, cf.z, cf.w, px, py, pz)) < cthr;
            if (inb) acc = acc + (ex ? 255u : 0u) - 255u * ((am >> i) & 1u);
          }
        }
        uint32_t c = acc / 255u;
        c += __shfl_xor(c, 32);
        if (hh == 0 && col && c) atomicAdd(&s_cnt[j >> 1], c << (16 * (j & 1)));
        head += m;
      };
      // tile-sphere test of two list entries per lane (entries e0 = 2 (lane + 64 k), e0 + 1;
      // entries past the list end were zeroed at load: plane 0, masked here), packed FMAs
      const f32x2 tbx = {tb.x, tb.x}, tby = {tb.y, tb.y}, tbz = {tb.z, tb.z};
      // four list entries per lane per step (two list registers): four LDS reads in flight, two
      // packed FMA chains; the ring takes <= 31 queued + 256 appended
      auto test4 = [&](uint32_t wa, uint32_t wb, int ea) {
        const int j0 = (int)(wa & 0xFFFFu), j1 = (int)(wa >> 16);
        const int j2 = (int)(wb & 0xFFFFu), j3 = (int)(wb >> 16);
        const float4 c0 = s_cf[j0], c1 = s_cf[j1], c2 = s_cf[j2], c3 = s_cf[j3];
        const f32x2 ax2 = {c0.x, c1.x}, ay2 = {c0.y, c1.y}, az2 = {c0.z, c1.z}, aw2 = {c0.w, c1.w};
        const f32x2 bx2 = {c2.x, c3.x}, by2 = {c2.y, c3.y}, bz2 = {c2.z, c3.z}, bw2 = {c2.w, c3.w};
        const f32x2 ha = __builtin_elementwise_fma(ax2, tbx, __builtin_elementwise_fma(ay2, tby,
                                                   __builtin_elementwise_fma(az2, tbz, aw2)));
        const f32x2 hb = __builtin_elementwise_fma(bx2, tbx, __builtin_elementwise_fma(by2, tby,
                                                   __builtin_elementwise_fma(bz2, tbz, bw2)));
        const int eb = ea + 2 * kWave;
        const bool n0 = ea < le && fabsf(ha.x) <= tlim;
        const bool n1 = ea + 1 < le && fabsf(ha.y) <= tlim;
        const bool n2 = eb < le && fabsf(hb.x) <= tlim;
        const bool n3 = eb + 1 < le && fabsf(hb.y) <= tlim;
        const uint64_t m0 = ballot(n0), m1 = ballot(n1), m2 = ballot(n2), m3 = ballot(n3);
        const int k0 = (int)__popcll(m0), k1 = k0 + (int)__popcll(m1), k2 = k1 + (int)__popcll(m2);
        if (n0) ring[(nq + lanes_below(m0)) & (kRing2 - 1)] = (uint16_t)j0;
        if (n1) ring[(nq + k0 + lanes_below(m1)) & (kRing2 - 1)] = (uint16_t)j1;
        if (n2) ring[(nq + k1 + lanes_below(m2)) & (kRing2 - 1)] = (uint16_t)j2;
        if (n3) ring[(nq + k2 + lanes_below(m3)) & (kRing2 - 1)] = (uint16_t)j3;
        nq += k2 + (int)__popcll(m3);
        __builtin_amdgcn_wave_barrier();
        while (nq - head >= 32) score(32);
      };
      {  // one copy of the test/score code: the list registers rotate through R[0], R[1]
        uint32_t R[kListRegs];
#pragma unroll
        for (int k = 0; k < kListRegs; ++k) R[k] = L[k];
#pragma unroll 1
        for (int k = 0; lb + k * 2 * kWave < le; k += 2) {
          test4(R[0], R[1], lb + 2 * (lane + k * kWave));
#pragma unroll
          for (int q = 0; q + 2 < kListRegs; ++q) R[q] = R[q + 2];
        }
      }
      if (nq > head) score(nq - head);
      if constexpr (NPM) {
        if (qn > 0) drain(qn);  // the queue refers to this tile's points
        nn = nn_n;
      }
      tb = tb_n; x = xn; y = yn; z = zn;
    }
    }  // list passes
  }
  __syncthreads();
  for (int j = threadIdx.x; j < D; j += BS) {
    const int c = (int)((s_cnt[j >> 1] >> (16 * (j & 1))) & 0xFFFFu);
    if (c) atomicAdd(&counts[j], c);
  }
  if (stats && threadIdx.x < 6) atomicAdd(&stats[threadIdx.x], s_st[threadIdx.x]);
  if (pick_args.done) {
    // the speculative pick in the launch's last workgroup (no k_pick_p1 launch and no gap on the
    // round's critical path): this workgroup's count atomics are acknowledged (vmcnt) before it
    // takes its ticket, and the last one reads the sums with device-coherent loads
    __builtin_amdgcn_s_waitcnt(0);
    __shared__ unsigned s_ticket;
    __syncthreads();
    if (threadIdx.x == 0)
      s_ticket = __hip_atomic_fetch_add(pick_args.done, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __syncthreads();
    if (s_ticket != gridDim.x - 1) return;
    if (threadIdx.x == 0)  // (the next launch on this stream starts from zero)
      __hip_atomic_store(pick_args.done, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    pick_body<BS, true>(pick_args);
  }
}

// ---------------------------------------------------------------------------------------------
// k_score_tiles_ex (default tile scorer, SACMODEL_PLANE): the near (tile, plane) pairs evaluated
// exactly in PCL's op order with lanes as planes.  (Two points per packed f32 operation,
// v_pk_mul_f32 / v_pk_add_f32, measured slower: 0.4485 vs 0.4332 ms per first launch.)  Same items, claims, plane lists and tile-sphere
// tests as k_score_tiles_rl, but a near pair is queued as (plane | tile slot << 12) and every 64
// queued pairs form one pass: lane l takes pair l, reads its plane from LDS and walks the 32
// points of its tile, which every lane reads from the wave's LDS tile slots with uniform (or at
// most four distinct, bank-disjoint) ds_read_b128 addresses.  Per test: PCL's 3 mul + 3 add, the
// |d| < cthr compare and the count add; 32 independent tests per lane per pass, no band, no
// re-decision, no cross-lane traffic.  (k_score_tiles_rl spends ~178 VALU instructions per 32 x 32
// block on the B split, the two MFMAs' post-processing and the band check, along one dependent
// chain per block: VALU active 0.28 at 4 waves/SIMD.)  Points past n are stored as NaN (never an
// inlier: PCL's NaN < thr is false), so the pass has no validity test.
// The wave's four tile slots hold two items (slot pair = item sequence & 1): a pass may mix the
// leftover pairs of the previous item with the current item's, and leftovers whose slots are about
// to be overwritten are flushed first.
constexpr int kExRing = 1024;  // >= 64 K - 1 queued + 256 appended per list step + K - 1 pad
constexpr int kExSlotF = 100;  // floats per tile slot: x[32] y[32] z[32] + pad (slot bases 0,
                               // 100, 200, 300 dwords: banks 0, 36, 8, 44, disjoint for b128)
constexpr uint32_t kExPad = 0x4000u;  // ring entry flag: padding (no plane)
constexpr uint32_t kExNone = kMaxHypPerLaunch;  // list-register filler past a list's end
constexpr int kStaticNum = 7, kStaticDen = 8;  // k_score_tiles_ex: items dealt before the tail
constexpr int64_t kOrderMaxSupers = 65536;      // class-ordered claims up to this many super-tiles
// NORMAL_PLANE slots: x[32] y[32] z[32] lim[32] + pad (bases 0, 132, 264, 396 dwords: banks 0,
// 4, 8, 12, disjoint for b128)
constexpr int kExSlotNp = 132;

// inclusive max over the wave (DPP; lanes a step does not reach keep their own value)
template <int kCtrl, int kRowMask>
__device__ __forceinline__ int dpp_max_step(int v) {
  return max(v, __builtin_amdgcn_update_dpp(INT_MIN, v, kCtrl, kRowMask, 0xF, false));
}
__device__ __forceinline__ int wave_incl_max_i32(int v) {
  v = dpp_max_step<0x111, 0xF>(v);
  v = dpp_max_step<0x112, 0xF>(v);
  v = dpp_max_step<0x114, 0xF>(v);
  v = dpp_max_step<0x118, 0xF>(v);
  v = dpp_max_step<0x142, 0xA>(v);
  v = dpp_max_step<0x143, 0xC>(v);
  return v;
}
__device__ __forceinline__ int wave_incl_sum_i32(int v) {
  v += __builtin_amdgcn_update_dpp(0, v, 0x111, 0xF, 0xF, false);
  v += __builtin_amdgcn_update_dpp(0, v, 0x112, 0xF, 0xF, false);
  v += __builtin_amdgcn_update_dpp(0, v, 0x114, 0xF, 0xF, false);
  v += __builtin_amdgcn_update_dpp(0, v, 0x118, 0xF, 0xF, false);
  v += __builtin_amdgcn_update_dpp(0, v, 0x142, 0xA, 0xF, false);
  v += __builtin_amdgcn_update_dpp(0, v, 0x143, 0xC, 0xF, false);
  return v;
}
// v * 16 + the four bits (m0 first) of this lane in the compare masks m0..m3: four v_addc with
// the masks as carry-ins (the s_nop: two wait states between a VALU's mask write and its use)
__device__ __forceinline__ uint32_t shl4_add(uint32_t v, uint64_t m0, uint64_t m1, uint64_t m2,
                                             uint64_t m3) {
  uint64_t co;
  asm("s_nop 1\n\t"
      "v_addc_co_u32_e64 %0, %1, %0, %0, %2\n\t"
      "v_addc_co_u32_e64 %0, %1, %0, %0, %3\n\t"
      "v_addc_co_u32_e64 %0, %1, %0, %0, %4\n\t"
      "v_addc_co_u32_e64 %0, %1, %0, %0, %5"
      : "+v"(v), "=&s"(co)
      : "s"(m0), "s"(m1), "s"(m2), "s"(m3));
  return v;
}
// np_deuclid's |d_euclid| without its "+ 0 * 0" term: that add changes only the sign of a zero,
// which the final fabsf drops (the same float)
__device__ __forceinline__ float np_de_abs(float4 c, float x, float y, float z) {
  return fabsf(((c.x * x + c.z * z) + c.y * y) + c.w);
}
// position (LSB = 0) of the r-th set bit (r counted from 0) of v; r < popcount(v)
__device__ __forceinline__ int nth_set_bit(uint32_t v, int r) {
  int pos = 0, t = __popc(v & 0xFFFFu);
  if (r >= t) { r -= t; v >>= 16; pos += 16; }
  t = __popc(v & 0xFFu);
  if (r >= t) { r -= t; v >>= 8; pos += 8; }
  t = __popc(v & 0xFu);
  if (r >= t) { r -= t; v >>= 4; pos += 4; }
  t = __popc(v & 0x3u);
  if (r >= t) { r -= t; v >>= 2; pos += 2; }
  return pos + (r >= (int)(v & 1u) ? 1 : 0);
}

// ---------------------------------------------------------------------------------------------
// MFMA tile scorer (DLG_TILE_MFMA): a tile's near planes in groups of 16 (its ring segment padded
// to a multiple of 16 with "far" planes), each group scored against the tile's 32 points by two
// v_mfma_f32_16x16x4_f32 (A = 16 points x (x, y, z, 1), B = (a, b, c, d) x 16 planes; lane l
// supplies A[l & 15][l >> 4] and B[l >> 4][l & 15] and receives D[4 (l >> 4) + r][l & 15], i.e.
// four points of its own plane per MFMA; tools/mfma_f32_probe.hip checks the maps).  The matrix
// core evaluates each dot as an f32 fma chain, not in PCL's order ((a x + c z) + (b y + d), six
// roundings): |D - pcl| <= (4 + 4.25) u S with S = |a| ax + |b| ay + |c| az + |d| (u = 2^-24,
// ax.. the cloud's largest |coordinate|; each order's error <= the sum of its partial sums'
// roundings).  With band = 12 u S (+ 2^-100), |D| < cthr - band is a PCL inlier and |D| >=
// cthr + band is not; the rest (a few in 10^4 tests, and NaN: points past n) are re-decided with
// PCL's own arithmetic from the LDS tile slot, so the counts equal the exact scorer's.  Per
// 256 tests: one MFMA on the matrix pipe and ~3 VALU per result (two compares, one add) instead
// of 8 VALU per test.  (Up to 4 groups per pass, their 8 MFMAs issued before any result is read.)
constexpr int kMfG = 16;
constexpr int kMfPass = 2;  // groups per pass (their MFMAs issued before any result is read)
template <int MODE>  // 0: band 12 u S; A/B checks: 1 every result re-decided, 2 band 64 u S
__device__ __forceinline__ void mf_pass(int m, const uint16_t* ring, int head, const float* spt,
                                        const float4* s_cf, uint32_t* s_cnt, int lane, float cthr,
                                        float ax, float ay, float az) {
  typedef float f32x4v __attribute__((ext_vector_type(4)));
  constexpr int G = kMfPass;
  const int ng = m >> 4;  // groups (m: a multiple of 16, <= 16 G)
  const int k = lane >> 4, c = lane & 15;
  f32x4v d0[G], d1[G];
  float band[G];
  int jj[G], sb[G];  // the lane's plane (pad: bit 12 set) and tile-slot base, per group
  const f32x4v zero = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int g = 0; g < G; ++g) {
    if (g < ng) {
      const uint32_t e = ring[(head + kMfG * g + c) & (kExRing - 1)];
      jj[g] = (int)(e & 0xFFFu) | (e & kExPad ? 0x1000 : 0);
      float4 q = s_cf[e & 0xFFFu];
      // a pad: a plane 2^100 away (never near, never ambiguous, counts nothing)
      if (e & kExPad) q = make_float4(0.f, 0.f, 0.f, 0x1p100f);
      const float S = ((fabsf(q.x) * ax + fabsf(q.y) * ay) + fabsf(q.z) * az) + fabsf(q.w);
      band[g] = S * ((MODE == 2 ? 64.0f : 12.0f) * 0x1p-24f * (1.0f + 0x1p-16f)) + 0x1p-100f;
      const float b = k == 0 ? q.x : k == 1 ? q.y : k == 2 ? q.z : q.w;
      sb[g] = (int)((e >> 12) & 3u) * kExSlotF;
      const float* sl = spt + sb[g];
      const int kk = k < 3 ? k : 2;  // (lanes of k = 3 supply the 1 of (x, y, z, 1))
      const float a0 = k < 3 ? sl[kk * kTileP + c] : 1.0f;
      const float a1 = k < 3 ? sl[kk * kTileP + 16 + c] : 1.0f;
      d0[g] = __builtin_amdgcn_mfma_f32_16x16x4f32(a0, b, zero, 0, 0, 0);
      d1[g] = __builtin_amdgcn_mfma_f32_16x16x4f32(a1, b, zero, 0, 0, 0);
    }
  }
  // per result t = |D| - cthr: a sure inlier when t < -band, a sure outlier when t > band; the
  // group is ambiguous on this lane when the smallest |t| is not above band (NaN results -- points
  // past n -- compare false and are skipped by the min: never counted, as PCL's NaN < thr)
  uint32_t cnt[G];
  bool amb[G];
  bool any = false;
#pragma unroll
  for (int g = 0; g < G; ++g) {
    cnt[g] = 0u;
    amb[g] = false;
    if (g < ng) {
      float mn = INFINITY;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float t0 = fabsf(d0[g][r]) - cthr, t1 = fabsf(d1[g][r]) - cthr;
        cnt[g] += t0 < -band[g] ? 1u : 0u;
        cnt[g] += t1 < -band[g] ? 1u : 0u;
        mn = fminf(mn, fminf(fabsf(t0), fabsf(t1)));
      }
      // (|t| = band exactly is ambiguous: t = -band is an inlier the count above left out)
      amb[g] = (MODE == 1 && !(jj[g] & 0x1000)) || !(mn > band[g]);
      any = any || amb[g];
    }
  }
  if (ballot(any) != 0ull) {
    // re-decide the lane's 8 results of an ambiguous group with PCL's arithmetic (points from
    // the LDS slot, the plane from LDS)
#pragma unroll
    for (int g = 0; g < G; ++g) {
      if (amb[g]) {
        const float4 q = s_cf[jj[g] & 0xFFF];  // (never a pad: a pad is never ambiguous)
        const float* sl = spt + sb[g];
        uint32_t e = 0u;
#pragma unroll
        for (int h = 0; h < 2; ++h)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int pt = 16 * h + 4 * k + r;
            const float dd = pcl_dot(q.x, q.y, q.z, q.w, sl[pt], sl[kTileP + pt], sl[2 * kTileP + pt]);
            e += fabsf(dd) < cthr ? 1u : 0u;
          }
        cnt[g] = e;
      }
    }
  }
#pragma unroll
  for (int g = 0; g < G; ++g)
    if (g < ng && cnt[g]) atomicAdd(&s_cnt[(jj[g] & 0xFFF) >> 1], cnt[g] << (16 * (jj[g] & 1)));
}

// NPM (SACMODEL_NORMAL_PLANE, K = 2): the pass evaluates PCL's prefilter b = (1 - w) d_euclid <
// thr as the float compare d_euclid < lim with the point's lim (np_de_limit, computed once when
// the point is fetched, stored in its slot), each lane collecting its 2 x 32 verdicts as bits;
// the passing (point, plane) pairs of the pass are then dealt 64 at a time to the lanes
// (prefix sum of the lanes' bit counts, owner lane by a DPP max-scan of the chunk's first
// positions) and decided with PCL's double arithmetic (np_full, as k_score_np), the normal read
// from global memory.  Same counts as k_score_tiles_rl<NPM> and k_score_np.
template <int BS, int K, bool PK = false, bool NPM = false, bool MF = false, int MFX = 0>
__global__ __launch_bounds__(BS) void k_score_tiles_ex(
    const float* __restrict__ X, const float* __restrict__ Y, const float* __restrict__ Z, int n,
    const float4* __restrict__ tiles, const uint16_t* __restrict__ lp, int ls,
    const int32_t* __restrict__ lp_n, int32_t* __restrict__ work, int blk_cap, int xcd,
    int order, const HypRec* __restrict__ hyps,
    int D, float cthr, float margin, int32_t* __restrict__ counts,
    unsigned long long* __restrict__ stats, PickArgs pick_args,
    const float4* __restrict__ NRM = nullptr, double lambda = 0.0, double thr = 0.0,
    const float4* __restrict__ CN = nullptr, int tail = 1, float ax = 0.f, float ay = 0.f,
    float az = 0.f) {
  static_assert(K == 1 || K == 2 || K == 4, "planes per lane");
  static_assert(!NPM || (K == 2 && !PK), "NORMAL_PLANE: two planes per lane");
  static_assert(!MF || (K == 2 && !PK && !NPM), "MFMA groups: plane model");
  // ring segment granularity: K entries (lanes as planes), or 16 planes of one tile (MFMA)
  constexpr int kSeg = MF ? kMfG : K;
  constexpr int kPassN = MF ? kMfPass * kMfG : K * kWave;  // queued entries one pass takes
  constexpr int kChunk = 2;  // tiles per item
  constexpr int kSlotF = NPM ? kExSlotNp : kExSlotF;
  // (+1: plane kExNone, a NaN plane the list registers hold past the list's end -- never near)
  __shared__ float4 s_cf[kMaxHypPerLaunch + 1];
  __shared__ uint32_t s_cnt[kMaxHypPerLaunch / 2];  // 16-bit halves: <= 65535 points per workgroup
  __shared__ __attribute__((aligned(8))) uint16_t s_ring[BS / kWave][kExRing];
  __shared__ __attribute__((aligned(16))) float s_pt[BS / kWave][4 * kSlotF];
  __shared__ int s_own[NPM ? BS / kWave : 1][NPM ? kWave : 1];   // NPM: chunk owners
  __shared__ int s_stile[NPM ? BS / kWave : 1][4];                // NPM: each slot's tile
  __shared__ unsigned long long s_st[6];
  __shared__ int s_taken;
  const int lane = threadIdx.x & (kWave - 1), wv = threadIdx.x / kWave;
  const uint64_t wg_t0 = stats ? wall_clock64() : 0;  // (stats: the workgroup's span, RTC ticks)
  for (int j = threadIdx.x; j < D; j += BS) {
    const HypRec h = hyps[j];
    s_cf[j] = make_float4(h.a, h.b, h.c, h.d);
  }
  if (threadIdx.x == 0) {
    s_taken = 0;
    s_cf[kExNone] = make_float4(__builtin_nanf(""), 0.f, 0.f, 0.f);
  }
  for (int j = threadIdx.x; j < kMaxHypPerLaunch / 2; j += BS) s_cnt[j] = 0u;
  if (threadIdx.x < 6) s_st[threadIdx.x] = 0;
  __syncthreads();
  const int ntiles = (n + kTileP - 1) / kTileP;
  const int nitems = (ntiles + kChunk - 1) / kChunk;
  uint16_t* ring = s_ring[wv];
  float* spt = s_pt[wv];
  const int ips = kSuperTiles / kChunk;
  // XCD-aware items (workgroup b takes XCD b & 7's: super-tiles s = b & 7 (mod 8), so the 8 items
  // of a super-tile share its plane list in one L2).  order: the XCD's super-tiles by list-length
  // class (pw_class), the longest lists first.  The first kStaticFrac of an XCD's items are dealt
  // round-robin to its workgroups (claimed through the workgroup's LDS counter: cheap), the rest
  // from one global counter per XCD (a device atomic per claim, ~1 us, worth it only where it
  // evens out the workgroups' ends); each workgroup is capped at blk_cap items, and the caps of
  // an XCD's workgroups cover its items, so every item is claimed.
  const int xw = xcd ? (int)(blockIdx.x & 7) : 0;
  const int64_t nsup = ((int64_t)ntiles + kSuperTiles - 1) / kSuperTiles;
  int o_cnt[kPwBuckets];  // (uniform: this XCD's super-tiles per class)
  int64_t nx_st = 0;      // (uniform: this XCD's super-tiles)
#pragma unroll
  for (int b = 0; b < kPwBuckets; ++b) {
    o_cnt[b] = order ? __builtin_amdgcn_readfirstlane(work[kPwBucket + xw * kPruneWorkStride + b]) : 0;
    nx_st += o_cnt[b];
  }
  if (!order) nx_st = xcd ? (nsup - xw + 7) / 8 : nsup;
  const int64_t gx = xcd ? (int64_t)(gridDim.x >> 3) : (int64_t)gridDim.x;  // this XCD's workgroups
  const int64_t bx = xcd ? (int64_t)(blockIdx.x >> 3) : (int64_t)blockIdx.x;
  // (tail 0: every item dealt round-robin, round 4's claim)
  const int64_t n_static = tail ? (nx_st * ips * kStaticNum / kStaticDen) / gx * gx : nx_st * ips;
  // the XCD's l-th item (-1: the last super-tile's missing items; nitems: past the end)
  auto item_of = [&](int64_t l) -> int64_t {
    int64_t i = l / ips;
    int64_t st;
    if (order) {
      int b = kPwBuckets;
#pragma unroll
      for (int q = 0; q < kPwBuckets; ++q)  // (unrolled: o_cnt stays in registers)
        if (b == kPwBuckets) {
          if (i < o_cnt[q]) b = q;
          else i -= o_cnt[q];
        }
      if (b == kPwBuckets) return nitems;
      st = ord_of(lp_n, nsup, xw, b)[i];
    } else {
      st = xcd ? (int64_t)xw + 8 * i : i;
      if (st >= nsup) return nitems;
    }
    const int64_t itm = st * ips + l % ips;
    return itm < nitems ? itm : -1;
  };
  auto claim = [&]() -> int {
    int v = nitems;
    if (lane == 0) {
      const int k = atomicAdd(&s_taken, 1);
      if (k < blk_cap) {
        const int64_t ls = (int64_t)k * gx + bx;
        int64_t itm = ls < n_static ? item_of(ls) : -1;
        while (itm < 0)  // (the global tail; claim again past a missing item)
          itm = item_of(n_static + atomicAdd(&work[xw * kPruneWorkStride], 1));
        v = (int)itm;
      }
    }
    return __builtin_amdgcn_readfirstlane(__shfl(v, 0));  // (uniform: scalar control flow)
  };
  // lane l holds point l of an item (its two tiles); NaN past n.  NPM: and its prefilter limit
  // (-inf: never passes; a NaN w leaves the exact test NaN < thr, never an inlier)
  auto fetch = [&](int it, float& px, float& py, float& pz, float& pl) {
    const int64_t p = (int64_t)it * (kChunk * kTileP) + lane;
    px = py = pz = __builtin_nanf("");
    pl = -INFINITY;
    if (it < nitems && p < n) {
      px = X[p]; py = Y[p]; pz = Z[p];
      if constexpr (NPM) {
        const double w = lambda * (1.0 - (double)NRM[p].w);
        pl = w == w ? np_de_limit(w, thr) : -INFINITY;
      }
    }
  };
  int nq = 0, head = 0;  // ring positions (multiples of K at every tile segment boundary)
  // the m (<= 64 K, a multiple of K) oldest queued pairs: lane l takes the K consecutive entries
  // K l .. K l + K - 1 (one tile, K planes), so each point read from LDS serves K planes
  auto pass = [&](int m) __attribute__((always_inline)) {
    if (stats && lane == 0) { atomicAdd(&s_st[3], 1ull); atomicAdd(&s_st[4], (unsigned long long)m); }
    if constexpr (MF) {
      mf_pass<MFX>(m, ring, head, spt, s_cf, s_cnt, lane, cthr, ax, ay, az);
      head += m;
      return;
    }
    const bool act = lane * K < m;
    uint32_t e[K];
    if constexpr (K == 1) {
      e[0] = act ? (uint32_t)ring[(head + lane) & (kExRing - 1)] : kExPad;
    } else if constexpr (K == 2) {
      const uint32_t w = act ? *reinterpret_cast<const uint32_t*>(ring + ((head + 2 * lane) & (kExRing - 1)))
                             : (kExPad | kExPad << 16);
      e[0] = w & 0xFFFFu; e[1] = w >> 16;
    } else {
      const uint2 w = act ? *reinterpret_cast<const uint2*>(ring + ((head + 4 * lane) & (kExRing - 1)))
                          : make_uint2(kExPad | kExPad << 16, kExPad | kExPad << 16);
      e[0] = w.x & 0xFFFFu; e[1] = w.x >> 16; e[2] = w.y & 0xFFFFu; e[3] = w.y >> 16;
    }
    float4 cf[K];
#pragma unroll
    for (int k = 0; k < K; ++k) {
      cf[k] = s_cf[e[k] & 0xFFFu];
      if (e[k] & kExPad) cf[k] = make_float4(__builtin_nanf(""), 0.f, 0.f, 0.f);  // never counts
    }
    const float* b = spt + ((e[0] >> 12) & 3u) * kSlotF;
    if constexpr (NPM) {
      // prefilter verdicts: bit 31 - p of nm[k] for point p of the lane's tile, plane k
      uint32_t nm[K];
#pragma unroll
      for (int k = 0; k < K; ++k) nm[k] = 0u;
#pragma unroll 2
      for (int p = 0; p < kTileP; p += 4) {
        const float4 xs = *reinterpret_cast<const float4*>(b + p);
        const float4 ys = *reinterpret_cast<const float4*>(b + kTileP + p);
        const float4 zs = *reinterpret_cast<const float4*>(b + 2 * kTileP + p);
        const float4 lm = *reinterpret_cast<const float4*>(b + 3 * kTileP + p);
#pragma unroll
        for (int k = 0; k < K; ++k) {
          const float4 c = cf[k];
          nm[k] = shl4_add(nm[k], ballot(np_de_abs(c, xs.x, ys.x, zs.x) < lm.x),
                           ballot(np_de_abs(c, xs.y, ys.y, zs.y) < lm.y),
                           ballot(np_de_abs(c, xs.z, ys.z, zs.z) < lm.z),
                           ballot(np_de_abs(c, xs.w, ys.w, zs.w) < lm.w));
        }
      }
      // the passing pairs, 64 per step: pair g belongs to the lane whose [excl, incl) holds it
      const int c0 = __popc(nm[0]), cnt = c0 + __popc(nm[1]);
      const int incl = wave_incl_sum_i32(cnt), excl = incl - cnt;
      const int total = __builtin_amdgcn_readlane(incl, kWave - 1);
      const uint32_t ew = e[0] | e[1] << 16;
      int* own = s_own[wv];
#pragma unroll 1
      for (int base = 0; base < total; base += kWave) {
        const uint64_t om = ballot(cnt > 0 && excl <= base);  // (non-empty: total > base)
        const int own0 = 63 - (int)__builtin_clzll(om);
        own[lane] = -1;
        __builtin_amdgcn_wave_barrier();
        if (cnt > 0 && excl > base && excl < base + kWave) own[excl - base] = lane;
        __builtin_amdgcn_wave_barrier();
        int L = lane == 0 ? own0 : own[lane];
        L = wave_incl_max_i32(L);
        __builtin_amdgcn_wave_barrier();  // (own is rewritten by the next step)
        const int g = base + lane;
        const int exL = __shfl(excl, L), c0L = __shfl(c0, L);
        const uint32_t m0 = (uint32_t)__shfl((int)nm[0], L), m1 = (uint32_t)__shfl((int)nm[1], L);
        const uint32_t eL = (uint32_t)__shfl((int)ew, L);
        if (g < total) {
          int r = g - exL;
          const bool second = r >= c0L;
          if (second) r -= c0L;
          const int pt = 31 - nth_set_bit(second ? m1 : m0, r);
          const int jj = (int)((second ? eL >> 16 : eL) & 0xFFFu);
          const int slot = (int)((eL >> 12) & 3u);
          const float* bs = spt + slot * kSlotF;
          const float4 cq = s_cf[jj];
          const float de = np_deuclid(cq, bs[pt], bs[kTileP + pt], bs[2 * kTileP + pt]);
          const float4 nn = NRM[(int64_t)s_stile[wv][slot] * kTileP + pt];
          const double w = lambda * (1.0 - (double)nn.w);
          if (np_full(CN[jj], nn, w, (1.0 - w) * (double)de, thr))
            atomicAdd(&s_cnt[jj >> 1], 1u << (16 * (jj & 1)));
        }
      }
      head += m;
      return;
    }
    uint32_t acc[K];
#pragma unroll
    for (int k = 0; k < K; ++k) acc[k] = 0u;
    // (partly unrolled: fully unrolled, the compiler hoists all 24 LDS reads, 96 VGPRs, and spills)
#pragma unroll 2
    for (int p = 0; p < kTileP; p += 4) {
      const float4 xs = *reinterpret_cast<const float4*>(b + p);
      const float4 ys = *reinterpret_cast<const float4*>(b + kTileP + p);
      const float4 zs = *reinterpret_cast<const float4*>(b + 2 * kTileP + p);
#pragma unroll
      for (int k = 0; k < K; ++k) {
        const float4 c = cf[k];
        if constexpr (PK) {
          // two points per packed op (v_pk_mul_f32 / v_pk_add_f32, the coefficient broadcast by
          // op_sel): the same IEEE products and sums in PCL's order, 3 instead of 6 per test
          const f32x2 A = {c.x, c.x}, B = {c.y, c.y}, C = {c.z, c.z}, Dd = {c.w, c.w};
          const f32x2 x01 = {xs.x, xs.y}, x23 = {xs.z, xs.w}, y01 = {ys.x, ys.y};
          const f32x2 y23 = {ys.z, ys.w}, z01 = {zs.x, zs.y}, z23 = {zs.z, zs.w};
          const f32x2 d01 = (A * x01 + C * z01) + (B * y01 + Dd);
          const f32x2 d23 = (A * x23 + C * z23) + (B * y23 + Dd);
          acc[k] += fabsf(d01.x) < cthr ? 1u : 0u;
          acc[k] += fabsf(d01.y) < cthr ? 1u : 0u;
          acc[k] += fabsf(d23.x) < cthr ? 1u : 0u;
          acc[k] += fabsf(d23.y) < cthr ? 1u : 0u;
        } else {
          acc[k] += fabsf(pcl_dot(c.x, c.y, c.z, c.w, xs.x, ys.x, zs.x)) < cthr ? 1u : 0u;
          acc[k] += fabsf(pcl_dot(c.x, c.y, c.z, c.w, xs.y, ys.y, zs.y)) < cthr ? 1u : 0u;
          acc[k] += fabsf(pcl_dot(c.x, c.y, c.z, c.w, xs.z, ys.z, zs.z)) < cthr ? 1u : 0u;
          acc[k] += fabsf(pcl_dot(c.x, c.y, c.z, c.w, xs.w, ys.w, zs.w)) < cthr ? 1u : 0u;
        }
      }
    }
#pragma unroll
    for (int k = 0; k < K; ++k) {
      const int j = (int)(e[k] & 0xFFFu);
      if (acc[k]) atomicAdd(&s_cnt[j >> 1], acc[k] << (16 * (j & 1)));  // (pads count 0)
    }
    head += m;
  };
  // close a tile segment: pad it to a multiple of K entries (one tile per lane item)
  auto pad = [&](uint32_t tag) {
    if constexpr (kSeg > 1) {
      const int r = (kSeg - (nq & (kSeg - 1))) & (kSeg - 1);
      if (lane < r) ring[(nq + lane) & (kExRing - 1)] = (uint16_t)(tag | kExPad);
      nq += r;
      __builtin_amdgcn_wave_barrier();
      while (nq - head >= kPassN) pass(kPassN);
    }
  };
  int it_next = claim();
  float px, py, pz, pl;
  fetch(it_next, px, py, pz, pl);
  for (int seq = 0;; ++seq) {
    const int it = it_next;
    if (it >= nitems) break;
    it_next = claim();
    const int t0 = it * kChunk, t_end = min(ntiles, t0 + kChunk);
    const int sidx = t0 / kSuperTiles;  // kSuperTiles % kChunk == 0: one super-tile per item
    const int slot0 = (seq & 1) * 2;
    // queued leftovers of the item two back use the slots about to be overwritten: score them
    // (the tag read is uniform: readfirstlane keeps head, and every pass loop, scalar)
    if (nq > head &&
        ((__builtin_amdgcn_readfirstlane((int)ring[head & (kExRing - 1)]) >> 13) & 1) == (seq & 1))
      pass(nq - head);
    const float4 tb0 = tiles[t0];
    const float4 tb1 = t0 + 1 < t_end ? tiles[t0 + 1] : make_float4(0.f, 0.f, 0.f, 0.f);
    const int nlp = __builtin_amdgcn_readfirstlane(lp_n[sidx]);
    const uint32_t* lw = reinterpret_cast<const uint32_t*>(lp + (int64_t)sidx * ls);
    {
      float* d = spt + (slot0 + (lane >> 5)) * kSlotF + (lane & 31);
      __builtin_amdgcn_wave_barrier();
      d[0] = px; d[kTileP] = py; d[2 * kTileP] = pz;
      if constexpr (NPM) {
        d[3 * kTileP] = pl;
        if (lane < kChunk) s_stile[wv][slot0 + lane] = t0 + lane;
      }
      __builtin_amdgcn_wave_barrier();
    }
    fetch(it_next, px, py, pz, pl);  // the next item's points, in flight during this one
#pragma unroll 1
    for (int lb = 0; lb < nlp; lb += kListCap) {
      const int le = min(nlp, lb + kListCap);
      uint32_t L[kListRegs];
#pragma unroll
      for (int k = 0; k < kListRegs; ++k) {
        const int e = lb + 2 * (lane + k * kWave);
        L[k] = e < le ? lw[(lb >> 1) + lane + k * kWave] : (kExNone | kExNone << 16);
        if (e + 1 >= le) L[k] = (L[k] & 0xFFFFu) | kExNone << 16;
      }
#pragma unroll 1
      for (int t = t0; t < t_end; ++t) {
        const float4 tb = t == t0 ? tb0 : tb1;
        const uint32_t tag = (uint32_t)(slot0 + (t - t0)) << 12;
        const float tlim = prune_lim(margin, tb.w);
        if (stats && lane == 0) { atomicAdd(&s_st[2], 1ull); atomicAdd(&s_st[1], (unsigned long long)(le - lb)); }
        const f32x2 tbx = {tb.x, tb.x}, tby = {tb.y, tb.y}, tbz = {tb.z, tb.z};
        auto test4 = [&](uint32_t wa, uint32_t wb, int ea) {
          const int j0 = (int)(wa & 0xFFFFu), j1 = (int)(wa >> 16);
          const int j2 = (int)(wb & 0xFFFFu), j3 = (int)(wb >> 16);
          const float4 c0 = s_cf[j0], c1 = s_cf[j1], c2 = s_cf[j2], c3 = s_cf[j3];
          const f32x2 ax2 = {c0.x, c1.x}, ay2 = {c0.y, c1.y}, az2 = {c0.z, c1.z}, aw2 = {c0.w, c1.w};
          const f32x2 bx2 = {c2.x, c3.x}, by2 = {c2.y, c3.y}, bz2 = {c2.z, c3.z}, bw2 = {c2.w, c3.w};
          const f32x2 ha = __builtin_elementwise_fma(ax2, tbx, __builtin_elementwise_fma(ay2, tby,
                                                     __builtin_elementwise_fma(az2, tbz, aw2)));
          const f32x2 hb = __builtin_elementwise_fma(bx2, tbx, __builtin_elementwise_fma(by2, tby,
                                                     __builtin_elementwise_fma(bz2, tbz, bw2)));
          // (entries past the list's end are kExNone: a NaN plane, never near)
          const bool n0 = fabsf(ha.x) <= tlim, n1 = fabsf(ha.y) <= tlim;
          const bool n2 = fabsf(hb.x) <= tlim, n3 = fabsf(hb.y) <= tlim;
          const uint64_t m0 = ballot(n0), m1 = ballot(n1), m2 = ballot(n2), m3 = ballot(n3);
          const int k0 = (int)__popcll(m0), k1 = k0 + (int)__popcll(m1), k2 = k1 + (int)__popcll(m2);
          if (n0) ring[(nq + lanes_below(m0)) & (kExRing - 1)] = (uint16_t)(tag | (uint32_t)j0);
          if (n1) ring[(nq + k0 + lanes_below(m1)) & (kExRing - 1)] = (uint16_t)(tag | (uint32_t)j1);
          if (n2) ring[(nq + k1 + lanes_below(m2)) & (kExRing - 1)] = (uint16_t)(tag | (uint32_t)j2);
          if (n3) ring[(nq + k2 + lanes_below(m3)) & (kExRing - 1)] = (uint16_t)(tag | (uint32_t)j3);
          nq += k2 + (int)__popcll(m3);
          __builtin_amdgcn_wave_barrier();
          while (nq - head >= kPassN) pass(kPassN);
        };
        uint32_t R[kListRegs];
#pragma unroll
        for (int k = 0; k < kListRegs; ++k) R[k] = L[k];
#pragma unroll 1
        for (int k = 0; lb + k * 2 * kWave < le; k += 2) {
          test4(R[0], R[1], lb + 2 * (lane + k * kWave));
#pragma unroll
          for (int q = 0; q + 2 < kListRegs; ++q) R[q] = R[q + 2];
        }
        pad(tag);
      }
    }
  }
  if (nq > head) pass(nq - head);
  __syncthreads();
  for (int j = threadIdx.x; j < D; j += BS) {
    const int c = (int)((s_cnt[j >> 1] >> (16 * (j & 1))) & 0xFFFFu);
    if (c) atomicAdd(&counts[j], c);
  }
  if (stats && threadIdx.x < 6) atomicAdd(&stats[threadIdx.x], s_st[threadIdx.x]);
  if (stats && threadIdx.x == 0) {
    const unsigned long long dt = wall_clock64() - wg_t0;
    atomicAdd(&stats[6], dt);
    atomicMax(&stats[7], dt);
    atomicAdd(&stats[0], 1ull);
#ifdef DLG_WG_TRACE  // (A/B build only: every workgroup's span and claims)
    printf("WGT %u %llu %llu %d\n", blockIdx.x, (unsigned long long)wg_t0,
           (unsigned long long)(wg_t0 + dt), s_taken);
#endif
  }
  if (order) {  // the last workgroup leaves the super-tile counts zero for the next launch
    __shared__ int s_last;
    __syncthreads();
    if (threadIdx.x == 0) s_last = atomicAdd(&work[kPwTicket], 1) == (int)gridDim.x - 1;
    __syncthreads();
    if (s_last && threadIdx.x < 8 * kPwBuckets)
      work[kPwBucket + (threadIdx.x / kPwBuckets) * kPruneWorkStride + threadIdx.x % kPwBuckets] = 0;
    if (s_last && threadIdx.x == 0) work[kPwTicket] = 0;
  }
  if (pick_args.done) {  // the fused speculative pick, as in k_score_tiles_rl
    __builtin_amdgcn_s_waitcnt(0);
    __shared__ unsigned s_ticket;
    __syncthreads();
    if (threadIdx.x == 0)
      s_ticket = __hip_atomic_fetch_add(pick_args.done, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __syncthreads();
    if (s_ticket != gridDim.x - 1) return;
    if (threadIdx.x == 0)
      __hip_atomic_store(pick_args.done, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    pick_body<BS, true>(pick_args);
  }
}

__global__ void k_gather_nrm(const float4* __restrict__ src, const int32_t* __restrict__ order,
                             int64_t n, float4* __restrict__ dst) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) dst[i] = src[order[i]];
}

__device__ __forceinline__ uint32_t f2ord(float f) {  // float -> order-preserving uint
  const uint32_t u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}

__global__ void k_curv_range(const float4* __restrict__ nrm, int64_t n, uint32_t* __restrict__ out2) {
  uint32_t lo = 0xFFFFFFFFu, hi = 0u;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    const float c = nrm[i].w;
    if (c == c) {
      const uint32_t o = f2ord(c);
      lo = min(lo, o);
      hi = max(hi, o);
    }
  }
#pragma unroll
  for (int o = 1; o < kWave; o <<= 1) {
    lo = min(lo, (uint32_t)__shfl_xor((int)lo, o));
    hi = max(hi, (uint32_t)__shfl_xor((int)hi, o));
  }
  if ((threadIdx.x & (kWave - 1)) == 0) {
    atomicMin(&out2[0], lo);
    atomicMax(&out2[1], hi);
  }
}
}  // namespace

void launch_morton_keys(PointsView src, float ax, float ay, float az, uint32_t* keys,
                        int32_t* idx, int32_t* n_nonfinite, float4* aos, hipStream_t s,
                        bool hilbert) {
  if (src.n <= 0) return;
  hipLaunchKernelGGL(k_morton_keys, dim3((unsigned)((src.n + 255) / 256)), dim3(256), 0, s, src,
                     ax, ay, az, keys, idx, n_nonfinite, aos, hilbert ? 1 : 0);
}

size_t morton_sort_temp_bytes(int64_t n) {
  size_t t = 0;
  (void)hipcub::DeviceRadixSort::SortPairs(nullptr, t, (uint32_t*)nullptr, (uint32_t*)nullptr,
                                           (int32_t*)nullptr, (int32_t*)nullptr, (int)n, 0, 32);
  return t;
}

hipError_t morton_sort(void* tmp, size_t tmp_bytes, uint32_t* keys_in, uint32_t* keys_out,
                       int32_t* idx_in, int32_t* idx_out, int64_t n, hipStream_t s) {
  return hipcub::DeviceRadixSort::SortPairs(tmp, tmp_bytes, keys_in, keys_out, idx_in, idx_out,
                                            (int)n, 0, 32, s);
}

void launch_gather_order(const float4* src, const int32_t* order, int64_t n, PointsOut dst,
                         hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_gather_order, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, src,
                     order, n, dst);
}

void launch_sphere_bounds(const float* x, const float* y, const float* z, int64_t n,
                          const int32_t* n_dev, float4* tiles, float4* supers, hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_sphere_bounds3, dim3((unsigned)((n + kSb3Pts - 1) / kSb3Pts)), dim3(64), 0, s,
                     x, y, z, n, n_dev, tiles, supers);
}

float prune_margin(float cthr, const float amax[3]) {
  const double smax = 2.0001 * ((double)amax[0] + (double)amax[1] + (double)amax[2]) + 1e-30;
  const double emax = 64.0 * 0x1p-24 * smax;
  const double m = ((double)cthr + 2.0 * emax) * (1.0 + 0x1p-19);
  float f = (float)m;
  if ((double)f < m) f = std::nextafter(f, INFINITY);
  return f;
}

void launch_gather_nrm(const float4* src, const int32_t* order, int64_t n, float4* dst,
                       hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_gather_nrm, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, src, order,
                     n, dst);
}

void launch_curv_range(const float4* nrm, int64_t n, uint32_t* out2, hipStream_t s) {
  const uint32_t init[2] = {0xFFFFFFFFu, 0u};
  (void)hipMemcpyAsync(out2, init, 8, hipMemcpyHostToDevice, s);
  if (n <= 0) return;
  const int64_t blocks = std::min<int64_t>(2048, (n + 255) / 256);
  hipLaunchKernelGGL(k_curv_range, dim3((unsigned)blocks), dim3(256), 0, s, nrm, n, out2);
}

float np_lim_max(double w, double thr) {  // np_de_limit (np_dev.hpp) on the host
  if (!(w >= 0.0)) return INFINITY;
  const double omw = 1.0 - w;
  if (!(omw > 0.0)) return INFINITY;
  if (!(thr > 0.0)) return thr == thr ? 0.0f : NAN;
  float x = (float)(thr / omw);
  if (!(x == x)) return INFINITY;
  while (!(omw * (double)x >= thr) && x < INFINITY) x = std::nextafter(x, INFINITY);
  while (x > 0.0f) {
    const float y = std::nextafter(x, -INFINITY);
    if (omw * (double)y >= thr) x = y;
    else break;
  }
  return x;
}

void launch_score_pruned(const SpatialView& v, const HypRec* hyps, int D, float cthr, float margin,
                         const float amax[3], int32_t* counts, uint16_t* lp, int32_t* lp_n,
                         int num_cus, hipStream_t s, unsigned long long* stats, const PrunedNp* np,
                         const PickArgs* pick, hipEvent_t ev_start, hipEvent_t ev_stop,
                         int tile_scorer) {
  if (D <= 0 || v.n <= 0 || D > kMaxHypPerLaunch) {
    if (ev_start) (void)hipEventRecord(ev_start, s);
    if (pick) launch_pick_p1(*pick, s);  // (nothing to score: the pick still runs)
    if (ev_stop) (void)hipEventRecord(ev_stop, s);
    return;
  }
  const int64_t ns = sp_supers(v.n);
  const int ls = prune_list_stride(D);
  // hypers of H super-tiles (H <= 32, a power of two), as large as keeps >= 2 workgroups per CU
  int H = 1;
  while (H < 32 && ns / (2 * H) >= 2 * (int64_t)num_cus) H *= 2;
  const unsigned ga = (unsigned)std::max<int64_t>(1, (ns + H - 1) / H);
  int32_t* work = lp_n - kPwHeader;  // (the buffer's header: spatial.hpp)
  // one 1024-thread workgroup per CU (LDS + VGPRs); its waves claim 2-tile items dynamically,
  // each workgroup capped at blk_cap items (16-bit LDS counters: <= 65535 points per
  // workgroup), and enough workgroups that the caps cover every item
  constexpr int kBS = 1024, kChunkTiles = 2;
  static_assert(kSuperTiles % kChunkTiles == 0, "an item stays inside one super-tile");
  const int64_t items = (sp_tiles(v.n) + kChunkTiles - 1) / kChunkTiles;
  const int blk_cap = 65535 / (kChunkTiles * kTileP);
  int64_t g = std::max<int64_t>(
      1, std::max<int64_t>(std::min<int64_t>(num_cus, (items + kBS / kWave - 1) / (kBS / kWave)),
                           (items + blk_cap - 1) / blk_cap));
  // the XCD-aware item mapping needs a multiple of 8 workgroups, each within blk_cap items: at
  // most ceil(ceil(ns / 8) * ips / (g / 8)) per workgroup
  const int ips = kSuperTiles / kChunkTiles;
  int xcd = 0;
  if (g >= 8) {
    int64_t gx = (g + 7) / 8 * 8;
    const int64_t per_xcd = (ns + 7) / 8 * ips;
    while ((per_xcd + gx / 8 - 1) / (gx / 8) > blk_cap) gx += 8;
    g = gx;
    xcd = 1;
  }
  // (NORMAL_PLANE: DLG_TILE_BF16 selects round 4's k_score_tiles_rl<NPM>, lanes as points)
  const bool ex = tile_scorer != kTileScorerBf16;
  // (A/B only: 15 = round 4's claim, XCD round-robin without classes or tail; 16 = classes
  // without the tail; 17 = the tail without classes)
  const bool claim_ab = tile_scorer >= kTileScorerClaimR4 && tile_scorer <= kTileScorerClaimTail;
  // the class order only up to kOrderMaxSupers super-tiles: at C3 (19.5k) it takes the first
  // launch 0.418 -> 0.409 ms, at C4's 100M points on one GPU (195k) it costs the prune launch 97
  // -> 187 us (the bucket appends' atomics) and the scoring 1465 -> 1610 us (r05j4-j7)
  const int order = ex && xcd && ns <= kOrderMaxSupers && tile_scorer != kTileScorerClaimR4 &&
                            tile_scorer != kTileScorerClaimTail ? 1 : 0;
  const int tail = claim_ab && tile_scorer != kTileScorerClaimTail ? 0 : 1;
  // (timing events, when given, ride the two dispatches themselves: no marker packets, so no
  // launch gaps around the scoring)
  DLG_LAUNCH_EV(k_prune_supers, dim3(ga), dim3(kPrBS), 0, s, ev_start, nullptr, v.supers,
                        (int)ns, hyps, D, ls, margin, H, lp, lp_n, work, order,
                        np && ex ? np->cn : nullptr);
  if (np && ex) {
    DLG_LAUNCH_EV((k_score_tiles_ex<kBS, 2, false, true>), dim3((unsigned)g), dim3(kBS), 0, s,
                          nullptr, ev_stop, v.x, v.y, v.z, (int)v.n, v.tiles, lp, ls, lp_n, work,
                          blk_cap, xcd, order, hyps, D, cthr, margin, counts, stats,
                          pick ? *pick : PickArgs{}, np->nrm, np->lambda, np->thr, np->cn, tail,
                          0.f, 0.f, 0.f);
    return;
  }
  // (the MFMA scorer's rounding band is S x 12 u with S up to (ax + ay + az) + |d|: clouds whose
  // coordinates would overflow it take the exact scorer)
  if (ex && (tile_scorer == kTileScorerMfma || tile_scorer == kTileScorerMfmaX ||
             tile_scorer == kTileScorerMfmaW) &&
      (double)amax[0] + amax[1] + amax[2] < 1e30) {
    auto* kmf = tile_scorer == kTileScorerMfmaX ? k_score_tiles_ex<kBS, 2, false, false, true, 1>
              : tile_scorer == kTileScorerMfmaW ? k_score_tiles_ex<kBS, 2, false, false, true, 2>
                                                : k_score_tiles_ex<kBS, 2, false, false, true>;
    DLG_LAUNCH_EV(kmf, dim3((unsigned)g),
                          dim3(kBS), 0, s, nullptr, ev_stop, v.x, v.y, v.z, (int)v.n, v.tiles,
                          lp, ls, lp_n, work, blk_cap, xcd, order, hyps, D, cthr, margin, counts,
                          stats, pick ? *pick : PickArgs{}, (const float4*)nullptr, 0.0, 0.0,
                          (const float4*)nullptr, tail, amax[0], amax[1], amax[2]);
    return;
  }
  if (ex) {
    auto* kex = tile_scorer == kTileScorerExK1 ? k_score_tiles_ex<kBS, 1>
              : tile_scorer == kTileScorerExK4 ? k_score_tiles_ex<kBS, 4>
              : tile_scorer == kTileScorerExPk ? k_score_tiles_ex<kBS, 2, true>
                                               : k_score_tiles_ex<kBS, 2>;
    DLG_LAUNCH_EV(kex, dim3((unsigned)g), dim3(kBS), 0, s, nullptr, ev_stop,
                          v.x, v.y, v.z, (int)v.n, v.tiles, lp, ls, lp_n, work, blk_cap, xcd,
                          order, hyps, D, cthr, margin, counts, stats, pick ? *pick : PickArgs{},
                          (const float4*)nullptr, 0.0, 0.0, (const float4*)nullptr, tail, 0.f, 0.f,
                          0.f);
    return;
  }
  auto* kfn = np ? k_score_tiles_rl<kBS, true> : k_score_tiles_rl<kBS, false>;
  DLG_LAUNCH_EV(kfn, dim3((unsigned)g), dim3(kBS), 0, s, nullptr, ev_stop, v.x, v.y,
                        v.z, (int)v.n, v.tiles, lp, ls, lp_n, work, blk_cap, kChunkTiles, xcd, hyps, D,
                        cthr, margin, amax[0], amax[1], amax[2], counts, stats,
                        np ? np->nrm : nullptr, np ? np->lambda : 0.0, np ? np->thr : 0.0,
                        pick ? *pick : PickArgs{});
}
}  // namespace dlg
