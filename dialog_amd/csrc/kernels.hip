// kernels.hip -- hand-written CDNA4 (gfx950) kernels of the RANSAC plane path.
//
// Compiled with -ffp-contract=off and correctly rounded f32 divide/sqrt: every float op below
// rounds exactly where PCL 1.8 / Eigen 3.3 (SSE) rounds, so counts, inlier lists and model
// coefficients are bit-identical to the CPU restatement (oracle/pcl_oracle.c).  The only fused
// multiply-adds are the explicit __builtin_fmaf of the prefilter variant, whose result is never
// used for a decision inside its error band.
//
// Reference semantics (PCL 1.8, not vendored; reference call site
// Dialog/SimplifyVerticesSize.cpp:62-67):
//   SampleConsensusModelPlane::countWithinDistance   -> k_score
//   SampleConsensusModelPlane::selectWithinDistance  -> k_select_count / k_select_scatter
//   SampleConsensusModelPlane::isSampleGood + computeModelCoefficients -> k_build_hyps
//   computeMeanAndCovarianceMatrix (fast mode, double)  -> k_moments
#include "kernels.hpp"

#include <cfloat>
#include <cmath>

namespace dlg {

namespace {

constexpr int kWave = 64;

__device__ __forceinline__ uint64_t ballot(bool p) { return __builtin_amdgcn_ballot_w64(p); }

// v_writelane_b32: lane `sel` of v takes the wave-uniform value s (no VALU compare/select)
__device__ __forceinline__ int writelane(int v, int s, int sel) {
  asm volatile("v_writelane_b32 %0, %1, m0" : "+v"(v) : "s"(s), "{m0}"(sel));
  return v;
}

__device__ __forceinline__ int lanes_below(uint64_t m) {
  return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

// Eigen VectorXf(4).dot(Vector4f(x, y, z, 1)) under SSE: predux((c0x, c1y, c2z, c3*1)) =
// (c0 x + c2 z) + (c1 y + c3).  No contraction (-ffp-contract=off).
__device__ __forceinline__ float pcl_dot(float a, float b, float c, float d, float x, float y,
                                         float z) {
  return (a * x + c * z) + (b * y + d * 1.0f);
}

// ---------------------------------------------------------------------------------------------
__global__ void k_gather_samples(const int32_t* __restrict__ pos, int m, int64_t lo,
                                 PointsView src, SampleRec* __restrict__ out) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= m) return;
  int64_t p = (int64_t)pos[i] - lo;
  SampleRec r;
  r.gid = 0; r.x = 0.0f; r.y = 0.0f; r.z = 0.0f;
  if (p >= 0 && p < src.n) {
    r.gid = src.gid[p]; r.x = src.x[p]; r.y = src.y[p]; r.z = src.z[p];
  }
  out[i] = r;
}

// isSampleGood + computeModelCoefficients (sac_model_plane.hpp), one thread per draw.
__global__ void k_build_hyps(const SampleRec* __restrict__ s, int D, float cthr, float ax,
                             float ay, float az, HypRec* __restrict__ hyps,
                             int32_t* __restrict__ good_out) {
  int d = blockIdx.x * blockDim.x + threadIdx.x;
  if (d >= D) return;
  const SampleRec s0 = s[3 * d], s1 = s[3 * d + 1], s2 = s[3 * d + 2];
  float a0 = s1.x - s0.x, a1 = s1.y - s0.y, a2 = s1.z - s0.z;
  float b0 = s2.x - s0.x, b1 = s2.y - s0.y, b2 = s2.z - s0.z;
  float r0 = a0 / b0, r1 = a1 / b1, r2 = a2 / b2;
  bool good = (r0 != r1) || (r2 != r1);
  HypRec h;
  h.pad = 0;
  h.good = good ? 1 : 0;
  if (good) {
    float c0 = a1 * b2 - a2 * b1;
    float c1 = a2 * b0 - a0 * b2;
    float c2 = a0 * b1 - a1 * b0;
    float c3 = 0.0f;
    // VectorXf::normalize(): Eigen 3.3 guards z > 0; squaredNorm = (c0^2 + c2^2) + (c1^2 + c3^2)
    float z = (c0 * c0 + c2 * c2) + (c1 * c1 + c3 * c3);
    if (z > 0.0f) {
      float sq = sqrtf(z);  // correctly rounded (-fhip-fp32-correctly-rounded-divide-sqrt)
      c0 = c0 / sq; c1 = c1 / sq; c2 = c2 / sq; c3 = c3 / sq;
    }
    float dot = (c0 * s0.x + c2 * s0.z) + (c1 * s0.y + c3 * 1.0f);
    h.a = c0; h.b = c1; h.c = c2; h.d = -1.0f * dot;
    // prefilter band: |pcl_dot - fma_chain| <= 7 u S, S = sum |coef_k * coord_k|, u = 2^-24
    double S = fabs((double)h.a) * ax + fabs((double)h.b) * ay + fabs((double)h.c) * az +
               fabs((double)h.d);
    double E = S * (7.0 * 5.9604644775390625e-08) * (1.0 + 1e-6) + 1e-37;
    h.tlo = __double2float_rd((double)cthr - E);
    h.thi = __double2float_ru((double)cthr + E);
  } else {
    h.a = h.b = h.c = h.d = __builtin_nanf("");
    h.tlo = h.thi = 0.0f;
  }
  hyps[d] = h;
  good_out[d] = h.good;
}

// ---------------------------------------------------------------------------------------------
// k_score: counts[h] = #{active i : |pcl_dot(h, p_i)| < cthr}.
//
// One lane per point slot (kP points per lane, coalesced 4-B SoA loads), the hypothesis tile
// staged in LDS and read with a wave-uniform address (LDS broadcast), the per-hypothesis wave
// count from ballot + popcount on the scalar unit, parked in lane (h mod 64) by v_writelane and
// flushed every 64 hypotheses with one ds_add per lane; the workgroup adds its LDS counts to the
// global counts once (one atomic per hypothesis per workgroup).  Grid-stride over 2048-point
// chunks with the grid sized to the resident capacity.
// VALU cost (exact variant): 3 v_mul + 3 v_add + 1 v_cmp per test -> VALU-bound at large D.
constexpr int kScBS = 256;
constexpr int kP = 8;
constexpr int kChunk = kScBS * kP;
constexpr int kHT = 1024;

template <int VARIANT>
__global__ __launch_bounds__(kScBS) void k_score(const float* __restrict__ X,
                                                 const float* __restrict__ Y,
                                                 const float* __restrict__ Z, int n,
                                                 const HypRec* __restrict__ hyps, int D,
                                                 float cthr, int32_t* __restrict__ counts) {
  __shared__ float4 s_coef[kHT];
  __shared__ float2 s_band[VARIANT == kScoreFmaBand ? kHT : 1];
  __shared__ int s_cnt[kMaxHypPerLaunch];
  const int tid = threadIdx.x;
  const int lane = tid & (kWave - 1);
  for (int i = tid; i < D; i += kScBS) s_cnt[i] = 0;
  const int nchunks = (n + kChunk - 1) / kChunk;
  const float qnan = __builtin_nanf("");
  for (int ch = blockIdx.x; ch < nchunks; ch += gridDim.x) {
    float px[kP], py[kP], pz[kP];
#pragma unroll
    for (int j = 0; j < kP; ++j) {
      int e = ch * kChunk + j * kScBS + tid;
      bool ok = e < n;
      px[j] = ok ? X[e] : qnan;
      py[j] = ok ? Y[e] : qnan;
      pz[j] = ok ? Z[e] : qnan;
    }
    for (int t0 = 0; t0 < D; t0 += kHT) {
      const int nt = min(kHT, D - t0);
      __syncthreads();
      for (int i = tid; i < nt; i += kScBS) {
        const HypRec hr = hyps[t0 + i];
        s_coef[i] = make_float4(hr.a, hr.b, hr.c, hr.d);
        if (VARIANT == kScoreFmaBand) s_band[i] = make_float2(hr.tlo, hr.thi);
      }
      __syncthreads();
      for (int g0 = 0; g0 < nt; g0 += kWave) {
        const int ng = min(kWave, nt - g0);
        int my = 0;
        float4 cn = s_coef[g0];
        for (int k = 0; k < ng; ++k) {
          const int h = g0 + k;
          const float4 c = cn;
          if (k + 1 < ng) cn = s_coef[h + 1];  // prefetch the next hypothesis (LDS broadcast)
          int cnt = 0;
          if (VARIANT == kScoreExact) {
#pragma unroll
            for (int j = 0; j < kP; ++j) {
              float dd = pcl_dot(c.x, c.y, c.z, c.w, px[j], py[j], pz[j]);
              cnt += __popcll(ballot(fabsf(dd) < cthr));
            }
          } else {
            const float2 band = s_band[h];
            uint64_t border = 0;
#pragma unroll
            for (int j = 0; j < kP; ++j) {
              float f = __builtin_fmaf(c.x, px[j], __builtin_fmaf(c.y, py[j], __builtin_fmaf(c.z, pz[j], c.w)));
              uint64_t lo = ballot(fabsf(f) < band.x);
              uint64_t hi = ballot(fabsf(f) < band.y);
              cnt += __popcll(lo);
              border |= lo ^ hi;
            }
            if (border) {  // rare: some lane is inside the rounding band -> exact PCL test there
#pragma unroll
              for (int j = 0; j < kP; ++j) {
                float f = __builtin_fmaf(c.x, px[j], __builtin_fmaf(c.y, py[j], __builtin_fmaf(c.z, pz[j], c.w)));
                bool inb = (fabsf(f) >= band.x) && (fabsf(f) < band.y);
                float dd = pcl_dot(c.x, c.y, c.z, c.w, px[j], py[j], pz[j]);
                cnt += __popcll(ballot(inb && (fabsf(dd) < cthr)));
              }
            }
          }
          my = writelane(my, cnt, k);
        }
        if (lane < ng) atomicAdd(&s_cnt[t0 + g0 + lane], my);
      }
    }
  }
  __syncthreads();
  for (int i = tid; i < D; i += kScBS) {
    int v = s_cnt[i];
    if (v) atomicAdd(&counts[i], v);
  }
}

// ---------------------------------------------------------------------------------------------
// k_moments (fast refit): count + first/second moments of the inliers of coef, in double, on
// coordinates shifted by a point of the plane (limits cancellation in cov = E[pp^T] - E[p]E[p]^T).
constexpr int kMoBS = 256;

__device__ __forceinline__ double wave_sum_d(double v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, kWave);
  return v;
}

__global__ __launch_bounds__(kMoBS) void k_moments(PointsView src, float4 cf, float cthr,
                                                   double3 sh, double* __restrict__ partials) {
  double acc[kMomentK];
#pragma unroll
  for (int k = 0; k < kMomentK; ++k) acc[k] = 0.0;
  const int64_t stride = (int64_t)gridDim.x * kMoBS;
  for (int64_t e = (int64_t)blockIdx.x * kMoBS + threadIdx.x; e < src.n; e += stride) {
    float x = src.x[e], y = src.y[e], z = src.z[e];
    float dd = pcl_dot(cf.x, cf.y, cf.z, cf.w, x, y, z);
    if (fabsf(dd) < cthr) {
      double dx = (double)x - sh.x, dy = (double)y - sh.y, dz = (double)z - sh.z;
      acc[0] += 1.0;
      acc[1] += dx; acc[2] += dy; acc[3] += dz;
      acc[4] += dx * dx; acc[5] += dx * dy; acc[6] += dx * dz;
      acc[7] += dy * dy; acc[8] += dy * dz; acc[9] += dz * dz;
    }
  }
  __shared__ double s_red[kMoBS / kWave][kMomentK];
  const int w = threadIdx.x / kWave, lane = threadIdx.x & (kWave - 1);
#pragma unroll
  for (int k = 0; k < kMomentK; ++k) {
    double v = wave_sum_d(acc[k]);
    if (lane == 0) s_red[w][k] = v;
  }
  __syncthreads();
  if (threadIdx.x < kMomentK) {
    double v = 0.0;
    for (int q = 0; q < kMoBS / kWave; ++q) v += s_red[q][threadIdx.x];
    partials[(int64_t)blockIdx.x * kMomentK + threadIdx.x] = v;
  }
}

__global__ void k_reduce_partials(const double* __restrict__ partials, int nb,
                                  double* __restrict__ out) {
  // fixed order: thread k sums column k over blocks 0..nb-1 in 8 strided lanes, then in order
  __shared__ double s[kMomentK][8];
  const int k = threadIdx.x / 8, r = threadIdx.x % 8;
  if (k < kMomentK) {
    double v = 0.0;
    for (int b = r; b < nb; b += 8) v += partials[(int64_t)b * kMomentK + k];
    s[k][r] = v;
  }
  __syncthreads();
  if (threadIdx.x < kMomentK) {
    double v = 0.0;
    for (int q = 0; q < 8; ++q) v += s[threadIdx.x][q];
    out[threadIdx.x] = v;
  }
}

// ---------------------------------------------------------------------------------------------
// select / compact (selectWithinDistance + removal of the inliers from the active list)
constexpr int kSelBS = 256;
constexpr int kSelIt = kSelTile / kSelBS;

__global__ __launch_bounds__(kSelBS) void k_select_count(PointsView src, float4 cf, float cthr,
                                                         int32_t* __restrict__ tile_in) {
  __shared__ int s_w[kSelBS / kWave];
  const int64_t base = (int64_t)blockIdx.x * kSelTile;
  int cnt = 0;
#pragma unroll 4
  for (int j = 0; j < kSelIt; ++j) {
    int64_t e = base + j * kSelBS + threadIdx.x;
    bool in = false;
    if (e < src.n) in = fabsf(pcl_dot(cf.x, cf.y, cf.z, cf.w, src.x[e], src.y[e], src.z[e])) < cthr;
    cnt += __popcll(ballot(in));
  }
  if ((threadIdx.x & (kWave - 1)) == 0) s_w[threadIdx.x / kWave] = cnt;
  __syncthreads();
  if (threadIdx.x == 0) {
    int t = 0;
    for (int q = 0; q < kSelBS / kWave; ++q) t += s_w[q];
    tile_in[blockIdx.x] = t;
  }
}

constexpr int kScanBS = 1024;
__global__ __launch_bounds__(kScanBS) void k_scan_tiles(const int32_t* __restrict__ tile_in,
                                                        int ntiles, int64_t n,
                                                        int32_t* __restrict__ off_in,
                                                        int32_t* __restrict__ off_out,
                                                        int32_t* __restrict__ totals) {
  __shared__ int s_in[kScanBS], s_out[kScanBS];
  const int t = threadIdx.x;
  const int per = (ntiles + kScanBS - 1) / kScanBS;
  const int b0 = t * per, b1 = min(ntiles, b0 + per);
  int si = 0, so = 0;
  for (int b = b0; b < b1; ++b) {
    int sz = (int)min<int64_t>(kSelTile, n - (int64_t)b * kSelTile);
    si += tile_in[b];
    so += sz - tile_in[b];
  }
  s_in[t] = si;
  s_out[t] = so;
  __syncthreads();
  for (int off = 1; off < kScanBS; off <<= 1) {  // Hillis-Steele inclusive scan
    int vi = t >= off ? s_in[t - off] : 0;
    int vo = t >= off ? s_out[t - off] : 0;
    __syncthreads();
    s_in[t] += vi;
    s_out[t] += vo;
    __syncthreads();
  }
  int ri = s_in[t] - si, ro = s_out[t] - so;  // exclusive
  for (int b = b0; b < b1; ++b) {
    int sz = (int)min<int64_t>(kSelTile, n - (int64_t)b * kSelTile);
    off_in[b] = ri;
    off_out[b] = ro;
    ri += tile_in[b];
    ro += sz - tile_in[b];
  }
  if (t == kScanBS - 1) {
    totals[0] = s_in[t];
    totals[1] = s_out[t];
  }
}

__global__ __launch_bounds__(kSelBS) void k_select_scatter(PointsView src, float4 cf, float cthr,
                                                           const int32_t* __restrict__ off_in,
                                                           const int32_t* __restrict__ off_out,
                                                           int32_t* __restrict__ inl_gid,
                                                           float* __restrict__ inl_xyz,
                                                           PointsOut dst, int compact) {
  __shared__ int s_w[2][2][kSelBS / kWave];  // [buffer][in/out][wave]
  const int64_t base = (int64_t)blockIdx.x * kSelTile;
  const int w = threadIdx.x / kWave, lane = threadIdx.x & (kWave - 1);
  int run_in = off_in[blockIdx.x], run_out = off_out[blockIdx.x];
  for (int j = 0; j < kSelIt; ++j) {
    const int buf = j & 1;
    int64_t e = base + j * kSelBS + threadIdx.x;
    bool valid = e < src.n;
    float x = 0.f, y = 0.f, z = 0.f;
    int32_t g = 0;
    bool in = false;
    if (valid) {
      x = src.x[e]; y = src.y[e]; z = src.z[e]; g = src.gid[e];
      in = fabsf(pcl_dot(cf.x, cf.y, cf.z, cf.w, x, y, z)) < cthr;
    }
    uint64_t mi = ballot(in), mo = ballot(valid && !in);
    if (lane == 0) {
      s_w[buf][0][w] = __popcll(mi);
      s_w[buf][1][w] = __popcll(mo);
    }
    __syncthreads();
    int wi = 0, wo = 0, ti = 0, to = 0;
#pragma unroll
    for (int q = 0; q < kSelBS / kWave; ++q) {
      int a = s_w[buf][0][q], b = s_w[buf][1][q];
      wi += q < w ? a : 0;
      wo += q < w ? b : 0;
      ti += a;
      to += b;
    }
    if (in) {
      int p = run_in + wi + lanes_below(mi);
      inl_gid[p] = g;
      if (inl_xyz) {
        inl_xyz[3 * (int64_t)p] = x; inl_xyz[3 * (int64_t)p + 1] = y; inl_xyz[3 * (int64_t)p + 2] = z;
      }
    } else if (valid && compact) {
      int p = run_out + wo + lanes_below(mo);
      dst.x[p] = x; dst.y[p] = y; dst.z[p] = z; dst.gid[p] = g;
    }
    run_in += ti;
    run_out += to;
  }
}

__global__ void k_absmax(PointsView src, uint32_t* __restrict__ out3) {
  float m[3] = {0.f, 0.f, 0.f};
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < src.n; e += stride) {
    m[0] = fmaxf(m[0], fabsf(src.x[e]));
    m[1] = fmaxf(m[1], fabsf(src.y[e]));
    m[2] = fmaxf(m[2], fabsf(src.z[e]));
  }
  for (int k = 0; k < 3; ++k) {
    float v = m[k];
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v = fmaxf(v, __shfl_xor(v, off, kWave));
    // non-negative floats order like their bit patterns; NaN/inf -> +inf bits dominate
    if ((threadIdx.x & (kWave - 1)) == 0) atomicMax(&out3[k], __float_as_uint(v));
  }
}

}  // namespace

// ---------------------------------------------------------------------------------------------
static inline unsigned cdiv(int64_t a, int64_t b) { return (unsigned)((a + b - 1) / b); }

void launch_gather_samples(const int32_t* pos, int m, int64_t lo, PointsView src, SampleRec* out,
                           hipStream_t s) {
  if (m <= 0) return;
  hipLaunchKernelGGL(k_gather_samples, dim3(cdiv(m, 256)), dim3(256), 0, s, pos, m, lo, src, out);
}

void launch_build_hyps(const SampleRec* samples, int D, float cthr, float ax, float ay, float az,
                       HypRec* hyps, int32_t* good, hipStream_t s) {
  if (D <= 0) return;
  hipLaunchKernelGGL(k_build_hyps, dim3(cdiv(D, 256)), dim3(256), 0, s, samples, D, cthr, ax, ay,
                     az, hyps, good);
}

void launch_score(PointsView src, const HypRec* hyps, int D, float cthr, int32_t* counts,
                  int variant, int num_cus, hipStream_t s) {
  if (D <= 0 || src.n <= 0) return;
  const int64_t nchunks = (src.n + kChunk - 1) / kChunk;
  // resident capacity: LDS ~ 16 KB coef + 8 KB band + 16 KB counts -> 4 workgroups / CU
  const int64_t cap = (int64_t)num_cus * 4;
  const int64_t per = (nchunks + cap - 1) / cap;       // chunks per workgroup
  const unsigned grid = (unsigned)((nchunks + per - 1) / per);
  if (variant == kScoreFmaBand)
    hipLaunchKernelGGL(k_score<kScoreFmaBand>, dim3(grid), dim3(kScBS), 0, s, src.x, src.y, src.z,
                       (int)src.n, hyps, D, cthr, counts);
  else
    hipLaunchKernelGGL(k_score<kScoreExact>, dim3(grid), dim3(kScBS), 0, s, src.x, src.y, src.z,
                       (int)src.n, hyps, D, cthr, counts);
}

int moments_blocks(int64_t n) {
  int64_t b = (n + kMoBS * 8 - 1) / (kMoBS * 8);
  if (b < 1) b = 1;
  if (b > 2048) b = 2048;
  return (int)b;
}

void launch_moments(PointsView src, float4 coef, float cthr, double3 shift, double* partials,
                    int nblocks, double* out, hipStream_t s) {
  hipLaunchKernelGGL(k_moments, dim3(nblocks), dim3(kMoBS), 0, s, src, coef, cthr, shift, partials);
  hipLaunchKernelGGL(k_reduce_partials, dim3(1), dim3(kMomentK * 8), 0, s, partials, nblocks, out);
}

int select_tiles(int64_t n) { return (int)((n + kSelTile - 1) / kSelTile); }

void launch_select(PointsView src, float4 coef, float cthr, int32_t* tile_in, int32_t* tile_off_in,
                   int32_t* tile_off_out, int32_t* totals, int32_t* inl_gid, float* inl_xyz,
                   const PointsOut* dst, hipStream_t s) {
  const int nt = select_tiles(src.n);
  if (nt == 0) {
    (void)hipMemsetAsync(totals, 0, 2 * sizeof(int32_t), s);
    return;
  }
  hipLaunchKernelGGL(k_select_count, dim3(nt), dim3(kSelBS), 0, s, src, coef, cthr, tile_in);
  hipLaunchKernelGGL(k_scan_tiles, dim3(1), dim3(kScanBS), 0, s, tile_in, nt, src.n, tile_off_in,
                     tile_off_out, totals);
  PointsOut d = dst ? *dst : PointsOut{nullptr, nullptr, nullptr, nullptr};
  hipLaunchKernelGGL(k_select_scatter, dim3(nt), dim3(kSelBS), 0, s, src, coef, cthr, tile_off_in,
                     tile_off_out, inl_gid, inl_xyz, d, dst ? 1 : 0);
}

void launch_absmax(PointsView src, uint32_t* out3, hipStream_t s) {
  (void)hipMemsetAsync(out3, 0, 3 * sizeof(uint32_t), s);
  if (src.n <= 0) return;
  unsigned g = cdiv(src.n, 256);
  if (g > 1024) g = 1024;
  hipLaunchKernelGGL(k_absmax, dim3(g), dim3(256), 0, s, src, out3);
}

}  // namespace dlg
