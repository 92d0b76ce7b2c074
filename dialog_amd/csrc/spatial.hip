// spatial.hip -- Morton-ordered copy of the active points, tile / super-tile bounding spheres and
// k_score_pruned, the pruned countWithinDistance (see spatial.hpp for the argument).
#include "spatial.hpp"

#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <cmath>

#include "dev_common.hpp"

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

__global__ void k_morton_keys(PointsView src, float ax, float ay, float az,
                              uint32_t* __restrict__ keys, int32_t* __restrict__ idx,
                              int32_t* __restrict__ n_nonfinite) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  bool nf = false;
  if (i < src.n) {
    const float x = src.x[i], y = src.y[i], z = src.z[i];
    uint32_t k = 0xFFFFFFFFu;
    if (isfinite(x) && isfinite(y) && isfinite(z))
      k = spread10(quant10(x, ax)) | (spread10(quant10(y, ay)) << 1) | (spread10(quant10(z, az)) << 2);
    else
      nf = true;
    keys[i] = k;
    idx[i] = (int32_t)i;
  }
  const uint64_t m = ballot(nf);
  if (m && (threadIdx.x & (kWave - 1)) == 0) atomicAdd(n_nonfinite, (int32_t)__popcll(m));
}

__global__ void k_gather_order(PointsView src, const int32_t* __restrict__ order, int64_t n,
                               PointsOut dst) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int32_t k = order[i];
  dst.x[i] = src.x[k];
  dst.y[i] = src.y[k];
  dst.z[i] = src.z[k];
  dst.gid[i] = src.gid[k];
}

// one wave per super-tile: the two half-waves take one tile each per step.  Tile sphere: centre
// = midpoint of the tile's bounding box, radius = max |p - c| (float) inflated by 2^-18 (covers
// the few roundings of the distance evaluation).  Super sphere: centre = midpoint of the super
// box, radius = max over its tiles of |c_t - C| + r_t, inflated the same way.
constexpr int kSbBS = 256;
__global__ __launch_bounds__(kSbBS) void k_sphere_bounds(const float* __restrict__ X,
                                                         const float* __restrict__ Y,
                                                         const float* __restrict__ Z, int64_t n,
                                                         float4* __restrict__ tiles,
                                                         float4* __restrict__ supers) {
  __shared__ float4 s_t[kSbBS / kWave][kSuperTiles];
  const int lane = threadIdx.x & (kWave - 1), wv = threadIdx.x / kWave;
  const int r32 = lane & 31, hh = lane >> 5;
  const int64_t s = (int64_t)blockIdx.x * (kSbBS / kWave) + wv;
  if (s * kSuperP >= n) return;
  const int ntile = (int)std::min<int64_t>(kSuperTiles, (n - s * kSuperP + kTileP - 1) / kTileP);
  float bx0 = INFINITY, by0 = INFINITY, bz0 = INFINITY;
  float bx1 = -INFINITY, by1 = -INFINITY, bz1 = -INFINITY;
  for (int tt = 0; tt < kSuperTiles; tt += 2) {
    const int tl = tt + hh;
    const int64_t t = s * kSuperTiles + tl;
    const int64_t p = t * kTileP + r32;
    const bool ok = tl < ntile && p < n;
    float x = 0.f, y = 0.f, z = 0.f;
    if (ok) { x = X[p]; y = Y[p]; z = Z[p]; }
    float x0 = ok ? x : INFINITY, y0 = ok ? y : INFINITY, z0 = ok ? z : INFINITY;
    float x1 = ok ? x : -INFINITY, y1 = ok ? y : -INFINITY, z1 = ok ? z : -INFINITY;
#pragma unroll
    for (int o = 1; o < 32; o <<= 1) {
      x0 = fminf(x0, __shfl_xor(x0, o)); y0 = fminf(y0, __shfl_xor(y0, o)); z0 = fminf(z0, __shfl_xor(z0, o));
      x1 = fmaxf(x1, __shfl_xor(x1, o)); y1 = fmaxf(y1, __shfl_xor(y1, o)); z1 = fmaxf(z1, __shfl_xor(z1, o));
    }
    const float cx = 0.5f * (x0 + x1), cy = 0.5f * (y0 + y1), cz = 0.5f * (z0 + z1);
    float d = 0.0f;
    if (ok) {
      const float dx = x - cx, dy = y - cy, dz = z - cz;
      d = sqrtf(dx * dx + dy * dy + dz * dz);
    }
#pragma unroll
    for (int o = 1; o < 32; o <<= 1) d = fmaxf(d, __shfl_xor(d, o));
    const float r = d * (1.0f + 0x1p-18f) + 1e-30f;
    if (r32 == 0 && tl < ntile) {
      const float4 ts = make_float4(cx, cy, cz, r);
      tiles[t] = ts;
      s_t[wv][tl] = ts;
    }
    // super box over both halves
    bx0 = fminf(bx0, fminf(x0, __shfl_xor(x0, 32))); by0 = fminf(by0, fminf(y0, __shfl_xor(y0, 32)));
    bz0 = fminf(bz0, fminf(z0, __shfl_xor(z0, 32)));
    bx1 = fmaxf(bx1, fmaxf(x1, __shfl_xor(x1, 32))); by1 = fmaxf(by1, fmaxf(y1, __shfl_xor(y1, 32)));
    bz1 = fmaxf(bz1, fmaxf(z1, __shfl_xor(z1, 32)));
  }
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  const float Cx = 0.5f * (bx0 + bx1), Cy = 0.5f * (by0 + by1), Cz = 0.5f * (bz0 + bz1);
  float R = 0.0f;
  if (lane < ntile) {
    const float4 ts = s_t[wv][lane];
    const float dx = ts.x - Cx, dy = ts.y - Cy, dz = ts.z - Cz;
    R = sqrtf(dx * dx + dy * dy + dz * dz) + ts.w;
  }
#pragma unroll
  for (int o = 1; o < kWave; o <<= 1) R = fmaxf(R, __shfl_xor(R, o));
  if (lane == 0) supers[s] = make_float4(Cx, Cy, Cz, R * (1.0f + 0x1p-18f) + 1e-30f);
}

// ---------------------------------------------------------------------------------------------
// k_score_pruned: one 16-wave workgroup per CU (persistent), all D planes (a, b, c, d) in LDS.
// Super-tiles are taken from a global queue.  Per super-tile:
//   1. every plane is tested against the super sphere (FMA chain, 1 plane per thread per step);
//      planes that may hold an inlier go to the LDS list Lp;
//   2. the waves take the super-tile's tiles from an LDS queue; per tile the planes of Lp are
//      tested against the tile sphere (64 per step, lanes = planes) and the near ones appended to
//      the wave's ring; every 32 queued planes (and the remainder at the end of Lp) are scored
//      against the tile's 32 points exactly as k_score_bf16 scores a 32 x 32 block: two
//      v_mfma_f32_32x32x16_bf16 on the split operands, sign-byte count, min |r| band check and
//      PCL-order re-decision of the band elements;
//   3. per-plane counts accumulate in LDS and go to HBM once per workgroup.
// A (tile, plane) pair is skipped only when fl(|h|) > (margin + r)(1 + 2^-20) (rounded
// evaluation), i.e. the exact distance of the plane to the sphere centre exceeds
// cthr + r + 2 e_max: no point of the sphere can then pass PCL's test (spatial.hpp).
constexpr int kPrBS = 1024;
constexpr int kPrWaves = kPrBS / kWave;
constexpr int kPrRing = 128;

__device__ __forceinline__ float prune_lim(float margin, float r) {
  return (margin + r) * (1.0f + 0x1p-20f);
}

__global__ __launch_bounds__(kPrBS) void k_score_pruned(
    const float* __restrict__ X, const float* __restrict__ Y, const float* __restrict__ Z,
    int n, const float4* __restrict__ tiles, const float4* __restrict__ supers,
    const HypRec* __restrict__ hyps, const uint4* __restrict__ bcol,
    const float* __restrict__ band, int D, float cthr, float margin,
    int32_t* __restrict__ counts, uint32_t* __restrict__ work) {
  __shared__ float4 s_cf[kMaxHypPerLaunch];
  __shared__ int32_t s_cnt[kMaxHypPerLaunch];
  __shared__ uint16_t s_lp[kMaxHypPerLaunch];
  __shared__ uint16_t s_ring[kPrWaves][kPrRing];
  __shared__ float4 s_tile[kSuperTiles];
  __shared__ int s_nlp, s_super, s_next;
  const int lane = threadIdx.x & (kWave - 1), wv = threadIdx.x / kWave;
  const int r32 = lane & 31, hh = lane >> 5;
  for (int j = threadIdx.x; j < D; j += kPrBS) {
    const HypRec h = hyps[j];
    s_cf[j] = make_float4(h.a, h.b, h.c, h.d);
    s_cnt[j] = 0;
  }
  const int nsup = (n + kSuperP - 1) / kSuperP;
  const f32x16 zero = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  for (;;) {
    if (threadIdx.x == 0) {
      s_super = (int)atomicAdd(work, 1u);
      s_nlp = 0;
      s_next = 0;
    }
    __syncthreads();
    const int sidx = s_super;
    if (sidx >= nsup) break;
    const int ntile = min(kSuperTiles, (n - sidx * kSuperP + kTileP - 1) / kTileP);
    if (threadIdx.x < ntile) s_tile[threadIdx.x] = tiles[(int64_t)sidx * kSuperTiles + threadIdx.x];
    {
      const float4 sp = supers[sidx];
      const float slim = prune_lim(margin, sp.w);
      for (int b = 0; b < D; b += kPrBS) {  // block-uniform trip count
        const int j = b + threadIdx.x;
        bool near = false;
        if (j < D) {
          const float4 cf = s_cf[j];
          const float h = __builtin_fmaf(cf.x, sp.x, __builtin_fmaf(cf.y, sp.y, __builtin_fmaf(cf.z, sp.z, cf.w)));
          near = fabsf(h) <= slim;  // NaN planes: never near (PCL counts nothing for them)
        }
        const uint64_t m = ballot(near);
        if (m) {
          int base = 0;
          if (lane == 0) base = atomicAdd(&s_nlp, (int)__popcll(m));
          base = __shfl(base, 0);
          if (near) s_lp[base + lanes_below(m)] = (uint16_t)j;
        }
      }
    }
    __syncthreads();
    const int nlp = s_nlp;
    for (;;) {
      int tl = 0;
      if (lane == 0) tl = atomicAdd(&s_next, 1);
      tl = __shfl(tl, 0);
      if (tl >= ntile) break;
      const float4 tb = s_tile[tl];
      const float tlim = prune_lim(margin, tb.w);
      const int64_t p0 = ((int64_t)sidx * kSuperTiles + tl) * kTileP;
      bool have_a = false;
      bool bad = false;
      float x = 0.f, y = 0.f, z = 0.f;
      u32x4 a1 = {0u, 0u, 0u, 0u}, a2 = {0u, 0u, 0u, 0u};
      int nq = 0, head = 0;
      // score the ring entries [head, head + m) (m <= 32) against this tile
      auto group = [&](int m) {
        if (!have_a) {
          have_a = true;
          const bool valid = p0 + r32 < n;
          if (valid) { x = X[p0 + r32]; y = Y[p0 + r32]; z = Z[p0 + r32]; }
          bad = ballot(!valid || !(isfinite(x) && isfinite(y) && isfinite(z))) != 0;
          const Split3 sx = split3(x), sy = split3(y), sz = split3(z);
          if (hh == 0) {
            a1 = u32x4{pk(sx.p1, sx.p1), pk(sx.p2, sx.p1), pk(sx.p3, sx.p2), pk(sy.p1, sy.p1)};
            a2 = u32x4{pk(sz.p3, sz.p2), pk(kBf16One, kBf16One), pk(kBf16One, 0u), 0u};
          } else {
            a1 = u32x4{pk(sy.p2, sy.p1), pk(sy.p3, sy.p2), pk(sz.p1, sz.p1), pk(sz.p2, sz.p1)};
            a2 = u32x4{0u, 0u, 0u, 0u};
          }
        }
        const bool col = r32 < m;
        const int j = col ? (int)s_ring[wv][(head + r32) & (kPrRing - 1)] : 0;
        u32x4 b1 = {0u, 0u, 0u, 0u}, b2 = {0u, 0u, 0u, 0u};
        float w = 0.0f;
        if (col) {
          const uint4 q = bcol[4 * j + hh], q2 = bcol[4 * j + 2 + hh];
          b1 = u32x4{q.x, q.y, q.z, q.w};
          b2 = u32x4{q2.x, q2.y, q2.z, q2.w};
          w = band[j];
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
          const float4 cf = s_cf[j];
#pragma unroll 1
          for (int i = 0; i < 16; ++i) {
            const float ri = fabsf(Dv[i]) - cthr;
            const bool inb = need && (bad || fabsf(ri) <= w);
            if (ballot(inb)) {
              const int row = (i & 3) + 8 * (i >> 2) + 4 * hh;
              const float px = __shfl(x, row), py = __shfl(y, row), pz = __shfl(z, row);
              const bool ex = p0 + row < n && fabsf(pcl_dot(cf.x, cf.y, cf.z, cf.w, px, py, pz)) < cthr;
              const uint32_t approx = __float_as_uint(ri) >> 31;
              if (inb) acc = acc + (ex ? 255u : 0u) - 255u * approx;
            }
          }
        }
        uint32_t c = acc / 255u;
        c += __shfl_xor(c, 32);
        if (hh == 0 && col && c) atomicAdd(&s_cnt[j], (int32_t)c);
      };
      for (int c0 = 0; c0 < nlp; c0 += kWave) {
        const int k = c0 + lane;
        bool near = false;
        int j = 0;
        if (k < nlp) {
          j = s_lp[k];
          const float4 cf = s_cf[j];
          const float h = __builtin_fmaf(cf.x, tb.x, __builtin_fmaf(cf.y, tb.y, __builtin_fmaf(cf.z, tb.z, cf.w)));
          near = fabsf(h) <= tlim;
        }
        const uint64_t m = ballot(near);
        if (near) s_ring[wv][(nq + lanes_below(m)) & (kPrRing - 1)] = (uint16_t)j;
        nq += (int)__popcll(m);
        __builtin_amdgcn_wave_barrier();
        while (nq - head >= 32) {
          group(32);
          head += 32;
        }
      }
      if (nq > head) group(nq - head);
    }
    __syncthreads();  // the queue / lists of this super-tile are reset at the top
  }
  __syncthreads();
  for (int j = threadIdx.x; j < D; j += kPrBS) {
    const int c = s_cnt[j];
    if (c) atomicAdd(&counts[j], c);
  }
}

}  // namespace

void launch_morton_keys(PointsView src, float ax, float ay, float az, uint32_t* keys,
                        int32_t* idx, int32_t* n_nonfinite, hipStream_t s) {
  if (src.n <= 0) return;
  hipLaunchKernelGGL(k_morton_keys, dim3((unsigned)((src.n + 255) / 256)), dim3(256), 0, s, src,
                     ax, ay, az, keys, idx, n_nonfinite);
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

void launch_gather_order(PointsView src, const int32_t* order, int64_t n, PointsOut dst,
                         hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_gather_order, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, src,
                     order, n, dst);
}

void launch_sphere_bounds(const float* x, const float* y, const float* z, int64_t n,
                          float4* tiles, float4* supers, hipStream_t s) {
  if (n <= 0) return;
  const int64_t ns = sp_supers(n);
  const int wpb = kSbBS / kWave;
  hipLaunchKernelGGL(k_sphere_bounds, dim3((unsigned)((ns + wpb - 1) / wpb)), dim3(kSbBS), 0, s,
                     x, y, z, n, tiles, supers);
}

float prune_margin(float cthr, const float amax[3]) {
  const double smax = 2.0001 * ((double)amax[0] + (double)amax[1] + (double)amax[2]) + 1e-30;
  const double emax = 64.0 * 0x1p-24 * smax;
  const double m = ((double)cthr + 2.0 * emax) * (1.0 + 0x1p-19);
  float f = (float)m;
  if ((double)f < m) f = std::nextafter(f, INFINITY);
  return f;
}

void launch_score_pruned(const SpatialView& v, const HypRec* hyps, const uint4* bcol,
                         const float* band, int D, float cthr, float margin, int32_t* counts,
                         uint32_t* work, int num_cus, hipStream_t s) {
  if (D <= 0 || v.n <= 0 || D > kMaxHypPerLaunch) return;
  const int64_t ns = sp_supers(v.n);
  const unsigned grid = (unsigned)std::max<int64_t>(1, std::min<int64_t>(num_cus, ns));
  hipLaunchKernelGGL(k_score_pruned, dim3(grid), dim3(kPrBS), 0, s, v.x, v.y, v.z, (int)v.n,
                     v.tiles, v.supers, hyps, bcol, band, D, cthr, margin, counts, work);
}

}  // namespace dlg
