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
#include "spatial.hpp"
#include "dev_common.hpp"
#include "np_dev.hpp"
#include "pick_dev.hpp"
#include "host_math.hpp"
#include "exact_refit.hpp"

#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstdlib>

namespace dlg {

namespace {

template <bool NP>
__device__ __forceinline__ bool model_in(const PointsView& src, int64_t e, float4 cf, float4 cn,
                                         const ModelTest& mt, float x, float y, float z) {
  if (NP) return np_test(cf, cn, x, y, z, src.nrm[e], mt.lambda, mt.thr);
  return fabsf(pcl_dot(cf.x, cf.y, cf.z, cf.w, x, y, z)) < mt.cthr;
}

// ---------------------------------------------------------------------------------------------
// lidx (lean lists): the list holds pristine indices only; src = the pristine copy, n_list the
// list length
__global__ void k_gather_samples(const int32_t* __restrict__ pos, int m, int64_t lo,
                                 PointsView src, const int32_t* __restrict__ lidx, int64_t n_list,
                                 SampleRec* __restrict__ out) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= m) return;
  int64_t p = (int64_t)pos[i] - lo;
  SampleRec r;
  r.gid = 0; r.x = 0.0f; r.y = 0.0f; r.z = 0.0f;
  if (p >= 0 && p < n_list) {
    const int64_t q = lidx ? lidx[p] : p;
    r.gid = src.gid[q]; r.x = src.x[q]; r.y = src.y[q]; r.z = src.z[q];
  }
  out[i] = r;
}

// isSampleGood + computeModelCoefficients (sac_model_plane.hpp), one thread per draw.
// isSampleGood + computeModelCoefficients of one draw, in PCL's op order
__device__ __forceinline__ HypRec build_hyp(const SampleRec s0, const SampleRec s1,
                                            const SampleRec s2, float cthr, float ax, float ay,
                                            float az) {
  float a0 = s1.x - s0.x, a1 = s1.y - s0.y, a2 = s1.z - s0.z;
  float b0 = s2.x - s0.x, b1 = s2.y - s0.y, b2 = s2.z - s0.z;
  float r0 = a0 / b0, r1 = a1 / b1, r2 = a2 / b2;
  bool good = (r0 != r1) || (r2 != r1);
  HypRec h;
  h.w = 0.0f;
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
    // min3 variant: r = fl(|f| - cthr) carries <= 2^-24 |r| relative error on top of E
    h.w = __double2float_ru(E * (1.0 + 1e-4));
  } else {
    h.a = h.b = h.c = h.d = __builtin_nanf("");
    h.tlo = h.thi = h.w = 0.0f;
  }
  return h;
}

__device__ __forceinline__ HypRec nan_hyp() {  // padding / not a plane: counts nothing
  HypRec h;
  h.a = h.b = h.c = h.d = __builtin_nanf("");
  h.tlo = h.thi = h.w = 0.0f;
  h.good = 0;
  return h;
}

__global__ void k_build_hyps(const SampleRec* __restrict__ s, int D, int Dp, float cthr, float ax,
                             float ay, float az, HypRec* __restrict__ hyps,
                             int32_t* __restrict__ good_out) {
  int d = blockIdx.x * blockDim.x + threadIdx.x;
  if (d >= Dp) return;
  if (d >= D) {  // padding up to the 64-plane groups of k_score: NaN planes count nothing
    hyps[d] = nan_hyp();
    return;
  }
  const HypRec h = build_hyp(s[3 * d], s[3 * d + 1], s[3 * d + 2], cthr, ax, ay, az);
  hyps[d] = h;
  good_out[d] = h.good;
}

// one rank: gather the three samples of each draw (positions read from the pinned host buffer),
// build the hypothesis, zero its count -- one launch instead of copy + gather + build + memset
__global__ void k_gather_build(const int32_t* pos, int D, int Dp, PointsView src,
                               const int32_t* __restrict__ lidx, int64_t n_list,
                               SampleRec* __restrict__ samples, float cthr, float ax, float ay,
                               float az, HypRec* __restrict__ hyps, int32_t* __restrict__ res) {
  const int d = blockIdx.x * blockDim.x + threadIdx.x;
  if (d >= Dp) return;
  res[d] = 0;  // counts[Dp]
  if (d >= D) {
    hyps[d] = nan_hyp();
    return;
  }
  // three dependent hops (positions over PCIe, list index, point): each hop's three loads are
  // issued together, and no store sits between the hops
  int64_t q[3];
  bool ok[3];
#pragma unroll
  for (int i = 0; i < 3; ++i) q[i] = pos[3 * d + i];
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    ok[i] = q[i] >= 0 && q[i] < n_list;
    q[i] = ok[i] ? q[i] : 0;
  }
  if (lidx) {  // lean list: pristine index -> pristine copy
#pragma unroll
    for (int i = 0; i < 3; ++i)
      if (ok[i]) q[i] = lidx[q[i]];
  }
  SampleRec r[3];
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    r[i].gid = 0; r[i].x = 0.0f; r[i].y = 0.0f; r[i].z = 0.0f;
    if (ok[i]) {
      r[i].gid = src.gid[q[i]]; r[i].x = src.x[q[i]]; r[i].y = src.y[q[i]]; r[i].z = src.z[q[i]];
    }
  }
#pragma unroll
  for (int i = 0; i < 3; ++i) samples[3 * d + i] = r[i];
  const HypRec h = build_hyp(r[0], r[1], r[2], cthr, ax, ay, az);
  hyps[d] = h;
  res[Dp + d] = h.good;  // good[D]
}

// ---------------------------------------------------------------------------------------------
// k_score: counts[h] = #{active i : |pcl_dot(h, p_i)| < cthr}.
//
// One lane per point slot (P points per lane, coalesced 4-B SoA loads), the hypothesis tile
// staged in LDS and read with a wave-uniform address (LDS broadcast), the per-hypothesis wave
// count from ballot + popcount on the scalar unit, parked in lane (h mod 64) by v_writelane and
// flushed every 64 hypotheses with one ds_add per lane; the workgroup adds its LDS counts to the
// global counts once (one atomic per hypothesis per workgroup).  Grid-stride over chunks of
// 256 * P points with the grid sized to the resident capacity.
//
constexpr int kScBS = 512;  // 8 waves share one LDS copy of the hypotheses
constexpr int kHT = 1024;

// the exact VALU kernel (PCL op order for every test): the reference the matrix-core and pruned
// kernels are checked against (tests/test_score_variants.py), and the scorer of contexts with
// DLG_OPT_SCORE_KERNEL = DLG_SCORE_EXACT
template <int P>
__global__ __launch_bounds__(kScBS) void k_score(const float* __restrict__ X,
                                                 const float* __restrict__ Y,
                                                 const float* __restrict__ Z, int n,
                                                 const HypRec* __restrict__ hyps, int D,
                                                 int slice_w, float cthr,
                                                 int32_t* __restrict__ counts) {
  constexpr int kChunk = kScBS * P;
  __shared__ float4 s_coef[kHT + 1];  // +1: the prefetch of the group's last plane reads past
  __shared__ int s_cnt[kHT];
  const int tid = threadIdx.x;
  const int lane = tid & (kWave - 1);
  // this workgroup's hypothesis slice [h0, h0 + nt): loaded once, kept in LDS for all chunks
  const int h0 = blockIdx.y * slice_w;
  const int nt = min(slice_w, D - h0);
  for (int i = tid; i < nt; i += kScBS) {
    s_cnt[i] = 0;
    const HypRec hr = hyps[h0 + i];
    s_coef[i] = make_float4(hr.a, hr.b, hr.c, hr.d);
  }
  __syncthreads();
  const int nchunks = (n + kChunk - 1) / kChunk;
  const float qnan = __builtin_nanf("");
  for (int ch = blockIdx.x; ch < nchunks; ch += gridDim.x) {
    float px[P], py[P], pz[P];
#pragma unroll
    for (int j = 0; j < P; ++j) {
      int e = ch * kChunk + j * kScBS + tid;
      bool ok = e < n;
      px[j] = ok ? X[e] : qnan;
      py[j] = ok ? Y[e] : qnan;
      pz[j] = ok ? Z[e] : qnan;
    }
    for (int g0 = 0; g0 < nt; g0 += kWave) {  // nt is a multiple of 64 (D padded with NaN planes)
      int my = 0;
      // software pipeline: the next hypothesis' LDS broadcast read is in flight while the
      // current one is evaluated (the wait lands at the loop back-edge, not at first use)
      float4 cnext = s_coef[g0];
#pragma unroll 8
      for (int k = 0; k < kWave; ++k) {
        const float4 c = cnext;
        cnext = s_coef[g0 + k + 1];
        int cnt = 0;
#pragma unroll
        for (int j = 0; j < P; ++j) {
          float dd = pcl_dot(c.x, c.y, c.z, c.w, px[j], py[j], pz[j]);
          cnt += __popcll(ballot(fabsf(dd) < cthr));
        }
        my = writelane(my, cnt, k);
      }
      atomicAdd(&s_cnt[g0 + lane], my);
    }
  }
  __syncthreads();
  for (int i = tid; i < nt; i += kScBS) {
    int v = s_cnt[i];
    if (v) atomicAdd(&counts[h0 + i], v);
  }
}

// ---------------------------------------------------------------------------------------------
// k_score_bf16: the plane distance D = a x + b y + c z + d on the bf16 matrix cores.
//
// Every float is split exactly into three bf16 pieces v = v1 + v2 + v3 (truncations: v1 = top 8
// significand bits, v2 = the next 8 of the remainder, v3 = the rest, <= 8 bits), so bf16 x bf16
// products are exact in f32.  One 32-element dot product per (point, plane) keeps the products
// v1 c1, v1 c2, v2 c1, v1 c3, v3 c1, v2 c2 of each coordinate (dropped: <= 2.1 u |v c|, u = 2^-24)
// and d1 + d2 + d3 (point side 1, 1, 1):
//   A row  (point):  x1 x1 x2 x1 x3 x2 | y1 y1 y2 y1 y3 y2 | z1 z1 z2 z1 z3 z2 | 1  1  1 | 0 x 11
//   B col  (plane):  a1 a2 a1 a3 a1 a2 | b1 b2 b1 b3 b1 b2 | c1 c2 c1 c3 c1 c2 | d1 d2 d3 | 0 x 11
// two v_mfma_f32_32x32x16_bf16 (K = 32) per 32 x 32 tile of (points, planes).
// Error: the 21 exact products are summed with <= 20 f32 roundings (<= 40 u sum|p| even if the
// hardware truncated), + dropped products 2.1 u S, + PCL's own rounding of pcl_dot <= 4 u S, so
// |D - pcl_dot| <= e = 64 u S (S = |a| ax + |b| ay + |c| az + |d|, 1.4x margin), floored at 1e-7.
// With r = |D| - cthr: |r| > w = 1.002 e decides exactly (r < 0: inlier).  The VALU per element:
// r (1 op), the sign bits of four r gathered by two v_perm_b32 into bytes 0x00 / 0xFF and summed
// by one v_sad_u8 (0.75 op), min |r| by v_min3 (0.5 op).  When some lane's min |r| <= w (an
// element inside the rounding band, ~1e-5 of the elements) or the tile holds a missing /
// non-finite point, the wave re-decides exactly those elements in PCL op order: the point comes
// from its owner lane by ds_bpermute, the plane from LDS.
//
// C/D layout (32x32x16): lane l holds column (plane) l & 31, rows (reg & 3) + 8 (reg >> 2) +
// 4 (l >> 5); A/B: lane l holds row/col l & 31, k = 8 (l >> 5) + j of each 16-wide K half.
constexpr int kBfBS = 256;  // 4 independent waves

// per plane: B column (4 x uint4 = k 0-7, 8-15, 16-23, 24-31) and band half-width w
__global__ void k_prep_bf16(const HypRec* __restrict__ hyps, int D, int Dp,
                            uint4* __restrict__ bcol, float* __restrict__ band) {
  const int h = blockIdx.x * blockDim.x + threadIdx.x;
  if (h >= Dp) return;
  HypRec hr;
  hr.good = 0;
  if (h < D) hr = hyps[h];
  const bool ok = hr.good && isfinite(hr.a) && isfinite(hr.b) && isfinite(hr.c) && isfinite(hr.d);
  uint4 q0 = make_uint4(0, 0, 0, 0), q1 = q0, q2 = q0, q3 = q0;
  // not a plane (bad sample, NaN coefficients: PCL counts nothing): B = 0 and d = 2 so D = 2,
  // |r| >= 1.9 > w = 0 -- counts nothing, never re-decided
  float w = 0.0f;
  if (ok) {
    const Split3 a = split3(hr.a), b = split3(hr.b), c = split3(hr.c), d = split3(hr.d);
    q0 = make_uint4(pk(a.p1, a.p2), pk(a.p1, a.p3), pk(a.p1, a.p2), pk(b.p1, b.p2));
    q1 = make_uint4(pk(b.p1, b.p3), pk(b.p1, b.p2), pk(c.p1, c.p2), pk(c.p1, c.p3));
    q2 = make_uint4(pk(c.p1, c.p2), pk(d.p1, d.p2), pk(d.p3, 0u), 0u);
    // hr.w >= 7 u S (k_build_hyps), so e = 64 u S <= hr.w * 64 / 7 (1% slack)
    const double e = fmax((double)hr.w * (64.0 / 7.0) * 1.01, 1e-7);
    // no finite bound (an infinite coordinate in the cloud): every element is re-decided
    w = isfinite(hr.w) ? __double2float_ru(1.002 * e) : INFINITY;
  } else {
    q2 = make_uint4(0u, pk(0x4000u, 0u), 0u, 0u);  // d1 = 2.0
  }
  bcol[4 * h] = q0; bcol[4 * h + 1] = q1; bcol[4 * h + 2] = q2; bcol[4 * h + 3] = q3;
  band[h] = w;
}

template <int TH>
__global__ __launch_bounds__(kBfBS) void k_score_bf16(const float* __restrict__ X,
                                                      const float* __restrict__ Y,
                                                      const float* __restrict__ Z, int n,
                                                      const HypRec* __restrict__ hyps,
                                                      const uint4* __restrict__ bcol,
                                                      const float* __restrict__ band, int D,
                                                      int ngroups, int part, float cthr,
                                                      int32_t* __restrict__ counts) {
  __shared__ float4 s_coef[kBfBS / kWave][TH * 32];
  const int lane = threadIdx.x & (kWave - 1);
  const int wv = threadIdx.x / kWave;
  const int wid = blockIdx.x * (kBfBS / kWave) + wv;
  const int g = wid % ngroups;  // this wave's planes: [g * 32 TH, (g + 1) * 32 TH)
  const int pi = wid / ngroups;  // this wave's points: [pi * part, min(n, (pi + 1) * part))
  const int p_beg = pi * part;
  const int p_end = min(n, p_beg + part);
  const int r32 = lane & 31, hh = lane >> 5;
  for (int k = lane; k < TH * 32; k += kWave) {
    const int h = g * TH * 32 + k;
    const HypRec hr = hyps[min(h, max(D - 1, 0))];
    s_coef[wv][k] = make_float4(hr.a, hr.b, hr.c, hr.d);
  }
  if (p_beg >= n) return;  // wave-uniform; no block-wide barrier below
  u32x4 b1[TH], b2[TH];
  float wb[TH];
  uint32_t cnt[TH];
#pragma unroll
  for (int t = 0; t < TH; ++t) {
    const int h = (g * TH + t) * 32 + r32;
    const uint4 q = bcol[4 * h + hh], q2 = bcol[4 * h + 2 + hh];
    b1[t] = u32x4{q.x, q.y, q.z, q.w};
    b2[t] = u32x4{q2.x, q2.y, q2.z, q2.w};
    wb[t] = band[h];
    cnt[t] = 0;
  }
  const f32x16 zero = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  // point loads run two tiles ahead of their use
  float x1 = 0.f, y1 = 0.f, z1 = 0.f, x2 = 0.f, y2 = 0.f, z2 = 0.f;
  {
    const int q1 = p_beg + r32, q2 = p_beg + 32 + r32;
    if (q1 < p_end) { x1 = X[q1]; y1 = Y[q1]; z1 = Z[q1]; }
    if (q2 < p_end) { x2 = X[q2]; y2 = Y[q2]; z2 = Z[q2]; }
  }
  for (int p0 = p_beg; p0 < p_end; p0 += 32) {
    const bool valid = p0 + r32 < p_end;
    const float x = x1, y = y1, z = z1;
    x1 = x2; y1 = y2; z1 = z2;
    {
      const int q = p0 + 64 + r32;
      x2 = 0.f; y2 = 0.f; z2 = 0.f;
      if (q < p_end) { x2 = X[q]; y2 = Y[q]; z2 = Z[q]; }
    }
    // a tile with a missing or non-finite point is re-decided element by element
    const bool bad = __builtin_amdgcn_ballot_w64(!valid || !(isfinite(x) && isfinite(y) && isfinite(z))) != 0;
    const Split3 sx = split3(x), sy = split3(y), sz = split3(z);
    u32x4 a1, a2;
    if (hh == 0) {
      a1 = u32x4{pk(sx.p1, sx.p1), pk(sx.p2, sx.p1), pk(sx.p3, sx.p2), pk(sy.p1, sy.p1)};
      a2 = u32x4{pk(sz.p3, sz.p2), pk(kBf16One, kBf16One), pk(kBf16One, 0u), 0u};
    } else {
      a1 = u32x4{pk(sy.p2, sy.p1), pk(sy.p3, sy.p2), pk(sz.p1, sz.p1), pk(sz.p2, sz.p1)};
      a2 = u32x4{0u, 0u, 0u, 0u};
    }
    const bf16x8 A1 = as_bf16x8(a1), A2 = as_bf16x8(a2);
    uint32_t amask = 0;  // bit t: some element of plane tile t lies within its band
#pragma unroll
    for (int t = 0; t < TH; ++t) {
      f32x16 Dv = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A1, as_bf16x8(b1[t]), zero, 0, 0, 0);
      Dv = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A2, as_bf16x8(b2[t]), Dv, 0, 0, 0);
      uint32_t acc = cnt[t];
      float m = INFINITY;
#pragma unroll
      for (int i = 0; i < 16; i += 4) {
        const float r0 = fabsf(Dv[i]) - cthr, r1 = fabsf(Dv[i + 1]) - cthr;
        const float r2 = fabsf(Dv[i + 2]) - cthr, r3 = fabsf(Dv[i + 3]) - cthr;
        acc = count4(r0, r1, r2, r3, acc);
        m = min3_abs(m, r0, r1);
        m = min3_abs(m, r2, r3);
      }
      cnt[t] = acc;
      amask |= m <= wb[t] ? (1u << t) : 0u;
    }
    // rare: re-decide the band elements in PCL op order (D recomputed on the matrix cores)
    if (__builtin_amdgcn_ballot_w64(bad || amask != 0)) {
#ifdef DLG_BF16_STATS
      if (lane == 0) atomicAdd(&counts[0], 1);
#endif
#pragma unroll 1
      for (int t = 0; t < TH; ++t) {
        const bool need = bad || ((amask >> t) & 1u);
        if (!__builtin_amdgcn_ballot_w64(need)) continue;
        f32x16 Dv = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A1, as_bf16x8(b1[t]), zero, 0, 0, 0);
        Dv = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A2, as_bf16x8(b2[t]), Dv, 0, 0, 0);
        const float4 cf = s_coef[wv][t * 32 + r32];
        const float w = wb[t];
        uint32_t acc = cnt[t];
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const float ri = fabsf(Dv[i]) - cthr;
          const bool inb = need && (bad || fabsf(ri) <= w);
          if (__builtin_amdgcn_ballot_w64(inb)) {
#ifdef DLG_BF16_STATS
            if (lane == 0) atomicAdd(&counts[1], 1);
#endif
            const int row = (i & 3) + 8 * (i >> 2) + 4 * hh;
            const float px = __shfl(x, row, kWave), py = __shfl(y, row, kWave);
            const float pz = __shfl(z, row, kWave);
            const bool ex = p0 + row < p_end &&
                            fabsf(pcl_dot(cf.x, cf.y, cf.z, cf.w, px, py, pz)) < cthr;
            const uint32_t approx = __float_as_uint(ri) >> 31;  // what count4 counted
            if (inb) acc = acc + (ex ? 255u : 0u) - 255u * approx;
          }
        }
        cnt[t] = acc;
      }
    }
  }
#pragma unroll
  for (int t = 0; t < TH; ++t) {
    uint32_t c = cnt[t] / 255u;
    c += __shfl_xor(c, 32);  // lanes l and l + 32 hold the two row halves of column l & 31
    const int h = (g * TH + t) * 32 + r32;
    if (hh == 0 && c && h < D) atomicAdd(&counts[h], (int32_t)c);
  }
}

// ---------------------------------------------------------------------------------------------
// k_moments (fast refit): the exact integer moments of the inliers of coef (exact_refit.hpp):
// per lane kMomDigits int64 digit sums, then wave / workgroup / grid sums of the digits -- integer
// adds, so the result is independent of the visiting order, the grid and the rank count.
constexpr int kMoBS = 256;

__device__ __forceinline__ int64_t wave_sum_i64(int64_t v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, kWave);
  return v;
}

// the fast refit from summed digits s_m (LDS) by the first wave: lanes 0..8 evaluate the nine
// correctly rounded entries (refit_entry) in parallel, lane 0 finishes (Jacobi, orientation,
// centre); bit-identical to refit_exact.  < 4 inliers or optimize off keep the unrefined plane.
__device__ __forceinline__ void refit_wave0(const int64_t* s_m, int qexp,
                                            const float4* __restrict__ cin, int optimize,
                                            float4* __restrict__ cout) {
  __shared__ double s_e[9];
  const int t = threadIdx.x;
  const bool go = optimize && s_m[0] >= 4;
  if (go && t < 9) s_e[t] = refit_entry(s_m, t);
  __syncthreads();
  if (t != 0) return;
  const float4 c = *cin;
  const float ci[4] = {c.x, c.y, c.z, c.w};
  float co[4] = {c.x, c.y, c.z, c.w};
  if (go) {
    double e[9];
    for (int k = 0; k < 9; ++k) e[k] = s_e[k];
    refit_finish(e, s_m[0], qexp, ci, co);
  }
  *cout = make_float4(co[0], co[1], co[2], co[3]);
}

// the grid's digit sums: partials [kMomDigits][nb] (digit-major) -> s_m.  Thread t < 31 * 8
// sums every eighth block sum of digit t / 8 (independent loads, all in flight), then LDS.
constexpr int kMoParts = 8;  // (kMomDigits x kMoParts <= 256 threads)
__device__ __forceinline__ void reduce_digits(const int64_t* __restrict__ partials, int nb,
                                              int64_t* s_m) {
  __shared__ int64_t s_p[kMomDigits * kMoParts];
  const int t = threadIdx.x;
  if (t < kMomDigits * kMoParts) {
    const int k = t / kMoParts, part = t % kMoParts;
    const int64_t* p = partials + (int64_t)k * nb;
    int64_t v = 0;
    int b = part;
    for (; b + 31 * kMoParts < nb; b += 32 * kMoParts) {  // (nb <= 512: at most 2 batches)
      int64_t u[32];
#pragma unroll
      for (int j = 0; j < 32; ++j)
        u[j] = __hip_atomic_load(p + b + j * kMoParts, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#pragma unroll
      for (int j = 0; j < 32; ++j) v += u[j];
    }
    for (; b < nb; b += kMoParts)
      v += __hip_atomic_load(p + b, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    s_p[t] = v;
  }
  __syncthreads();
  if (t < kMomDigits) {
    int64_t v = 0;
#pragma unroll
    for (int q = 0; q < kMoParts; ++q) v += s_p[t * kMoParts + q];
    s_m[t] = v;
  }
  __syncthreads();
}

// the block's digit sums -> partials [kMomDigits][nb]; the last workgroup to finish (device-scope
// counter, reset by it for the next launch) reduces them -> out (MODE 1: and refits -> cout)
template <int MODE>
__device__ __forceinline__ void moments_tail(const int64_t* acc, int64_t* __restrict__ partials,
                                             unsigned* __restrict__ done,
                                             int64_t* __restrict__ out, int qexp,
                                             const float4* __restrict__ cfp,
                                             float4* __restrict__ cout) {
  // (most waves of a filtered pass saw no inlier -- each inlier counts into acc[0] -- and skip
  // the reduction; the others add their wave sums into LDS)
  __shared__ unsigned long long s_sum[kMomDigits];
  const int lane = threadIdx.x & (kWave - 1);
  if (threadIdx.x < kMomDigits) s_sum[threadIdx.x] = 0ull;
  __syncthreads();
  if (ballot(acc[0] != 0)) {
#pragma unroll
    for (int k = 0; k < kMomDigits; ++k) {
      const int64_t v = wave_sum_i64(acc[k]);
      if (lane == 0 && v != 0) atomicAdd(&s_sum[k], (unsigned long long)v);
    }
  }
  __syncthreads();
  const int nb = (int)gridDim.x;
  // last workgroup: the partials go out as device-coherent (agent-scope atomic) stores, complete
  // (vmcnt) before this block takes its ticket; the last one reads them with coherent loads.  (An
  // agent-scope release / acquire fence instead writes back / invalidates the whole L2 of the XCD
  // in every workgroup: ~30 us per launch.)
  if (threadIdx.x < kMomDigits)
    __hip_atomic_store(partials + (int64_t)threadIdx.x * nb + blockIdx.x, (int64_t)s_sum[threadIdx.x],
                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __builtin_amdgcn_s_waitcnt(0);  // (the stores are acknowledged before the barrier)
  __shared__ unsigned s_ticket;
  __syncthreads();
  if (threadIdx.x == 0)
    s_ticket = __hip_atomic_fetch_add(done, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __syncthreads();
  if (s_ticket != (unsigned)nb - 1) return;
  __shared__ int64_t s_m[kMomDigits];
  reduce_digits(partials, nb, s_m);
  if (threadIdx.x == 0) *done = 0u;  // (the next launch on this stream starts from zero)
  if (threadIdx.x < kMomDigits) out[threadIdx.x] = s_m[threadIdx.x];
  if (MODE == 1) refit_wave0(s_m, qexp, cfp, 1, cout);
}

// MODE 0: the grid's digit sums -> out; MODE 1: also the refit -> cout (one rank)
template <bool NP, int MODE>
__global__ __launch_bounds__(kMoBS) void k_moments(PointsView src, const float4* __restrict__ cfp,
                                                   ModelTest mt, double qscale,
                                                   int64_t* __restrict__ partials,
                                                   unsigned* __restrict__ done,
                                                   int64_t* __restrict__ out, int qexp,
                                                   float4* __restrict__ cout) {
  const float4 cf = *cfp;
  const float4 cn = eigen_normalized3(cf.x, cf.y, cf.z, 0.0f);
  int64_t acc[kMomDigits];
#pragma unroll
  for (int k = 0; k < kMomDigits; ++k) acc[k] = 0;
  MomAcc m;
  mom_zero(m);
  // kMoIt points per lane per pass, their loads all in flight before the tests (clamped,
  // unconditional: one guarded load per iteration would wait out each load in turn)
  constexpr int kMoIt = 8;
  static_assert(kMoIt <= kMomFlush, "one flush per pass");
  const int64_t stride = (int64_t)gridDim.x * kMoBS * kMoIt;
  for (int64_t b0 = (int64_t)blockIdx.x * kMoBS * kMoIt; b0 < src.n; b0 += stride) {
    float x[kMoIt], y[kMoIt], z[kMoIt];
#pragma unroll
    for (int j = 0; j < kMoIt; ++j) {
      const int64_t e = min<int64_t>(b0 + j * kMoBS + threadIdx.x, src.n - 1);
      x[j] = src.x[e]; y[j] = src.y[e]; z[j] = src.z[e];
    }
#pragma unroll
    for (int j = 0; j < kMoIt; ++j) {
      const int64_t e = b0 + j * kMoBS + threadIdx.x;
      if (e < src.n && model_in<NP>(src, e, cf, cn, mt, x[j], y[j], z[j]))
        mom_point(m, fast_q(x[j], qscale), fast_q(y[j], qscale), fast_q(z[j], qscale));
    }
    if (m.n != 0.0) mom_flush(acc, m);  // (kMoIt <= kMomFlush points since the last flush)
  }
  moments_tail<MODE>(acc, partials, done, out, qexp, cfp, cout);
}

// lean rounds (plane model over the Morton copy): only the tiles whose bounding sphere may hold an
// inlier of cf are read -- k_prune_supers' test (a ruled-out sphere holds no point that passes
// PCL's test), first per super-tile, then per tile.  The same digits as k_moments (integer sums).
template <int MODE, bool NP = false>
__global__ __launch_bounds__(kMoBS) void k_moments_sp(PointsView src,
                                                      const float4* __restrict__ tiles,
                                                      const float4* __restrict__ supers,
                                                      float margin, const float4* __restrict__ cfp,
                                                      ModelTest mt, double qscale,
                                                      int64_t* __restrict__ partials,
                                                      unsigned* __restrict__ done,
                                                      int64_t* __restrict__ out, int qexp,
                                                      float4* __restrict__ cout) {
  const float4 cf = *cfp;
  const float4 cn = eigen_normalized3(cf.x, cf.y, cf.z, 0.0f);
  int64_t acc[kMomDigits];
#pragma unroll
  for (int k = 0; k < kMomDigits; ++k) acc[k] = 0;
  MomAcc m;
  mom_zero(m);
  // every wave tests 64 super-tiles at a time (lane l: super s0 + l W, W = waves in the grid, so
  // a run of near super-tiles spreads over consecutive waves), then walks its near ones: the 32
  // tile spheres in lanes 0..31, then the points of the near tiles, 16 per lane, all in flight
  const int64_t nsup = (src.n + kSuperP - 1) / kSuperP, ntile = (src.n + kTileP - 1) / kTileP;
  const int lane = threadIdx.x & (kWave - 1);
  const int64_t W = (int64_t)gridDim.x * (kMoBS / kWave);
  const int64_t wid = (int64_t)blockIdx.x * (kMoBS / kWave) + threadIdx.x / kWave;
  constexpr int kIt = kSuperP / kWave;
  static_assert(kIt <= kMomFlush, "one flush per super-tile");
  for (int64_t s0 = wid; s0 < nsup; s0 += kWave * W) {
    const int64_t sl = s0 + lane * W;
    uint64_t near = ballot(sl < nsup && sphere_near(cf, supers[sl], margin));
    while (near) {
      const int64_t s = s0 + (int64_t)(__ffsll((unsigned long long)near) - 1) * W;
      near &= near - 1;
      const int64_t tl = s * kSuperTiles + (lane & (kSuperTiles - 1));
      const uint32_t tm = (uint32_t)ballot(lane < kSuperTiles && tl < ntile &&
                                           sphere_near(cf, tiles[tl], margin));
      const int64_t base = s * kSuperP;
      float x[kIt], y[kIt], z[kIt];
#pragma unroll
      for (int j = 0; j < kIt; ++j) {
        const int64_t e = base + j * kWave + lane;
        if (((tm >> (2 * j + (lane >> 5))) & 1u) && e < src.n) {
          x[j] = src.x[e]; y[j] = src.y[e]; z[j] = src.z[e];
        }
      }
#pragma unroll
      for (int j = 0; j < kIt; ++j) {
        const int64_t e = base + j * kWave + lane;
        if (((tm >> (2 * j + (lane >> 5))) & 1u) && e < src.n &&
            model_in<NP>(src, e, cf, cn, mt, x[j], y[j], z[j]))
          mom_point(m, fast_q(x[j], qscale), fast_q(y[j], qscale), fast_q(z[j], qscale));
      }
      if (m.n != 0.0) mom_flush(acc, m);  // (kIt = kMomFlush points per lane per super-tile)
    }
  }
  moments_tail<MODE>(acc, partials, done, out, qexp, cfp, cout);
}

// fast refit on the device from the (rank-summed) digits: < 4 inliers or optimize off keep the
// unrefined plane.  Keeps the refined plane on the device for the final select (no host round
// trip between them).
__global__ __launch_bounds__(kWave) void k_refit_moments(const int64_t* __restrict__ mom, int qexp,
                                                         const float4* __restrict__ cin,
                                                         int optimize, float4* __restrict__ cout) {
  __shared__ int64_t s_m[kMomDigits];
  if (threadIdx.x < kMomDigits) s_m[threadIdx.x] = optimize ? mom[threadIdx.x] : 0;
  __syncthreads();
  refit_wave0(s_m, qexp, cin, optimize, cout);
}

// ---------------------------------------------------------------------------------------------
// k_pick_p1: RandomSampleConsensus::computeModel's decision over one batch of draws when the
// probability is 1 (log(1 - p) = -inf, so k = +inf and only the iteration cap ends the loop):
// the loop ends at the need_good-th good draw (need_good = max_iterations + 1) and keeps the
// first good draw with the largest count (strict '>').  A bad draw only consumes a getSamples
// try; with fewer than 1000 bad draws in the batch no run of 1000 can end the loop early.
// out[0] = batch index of the best draw (-1: none), out[1] = 1 if the loop ended inside the
// batch.  The winner's HypRec and samples are copied to best / best_smp.  Speculative: the host
// replays the same counts (RansacControl::consume) after the round's sync and redoes the round
// on any disagreement.  One workgroup.
constexpr int kPickBS = 1024;
__global__ __launch_bounds__(kPickBS) void k_pick_p1(PickArgs a) { pick_body<kPickBS, false>(a); }

// ---------------------------------------------------------------------------------------------
// k_publish: the round's small results (select totals, winner + refined plane, every rank's
// totals, the speculative pick and counts) written straight into a coherent pinned host buffer,
// then a system-scope release of the sequence number in pub[0]: the host spins on that word
// instead of waiting on a HIP event (whose wake-up costs ~50 us per round).  One workgroup.
// the publish by the nthr threads of one workgroup (k_publish, or the last tile of a fused
// select); tot01: the select's own totals[0..1] when the caller has just computed them (the
// global words may not be visible yet), else null
// (own01: totals[0..1] from t0 / t1 instead of a.totals -- two scalars, not an array: a
// dynamically indexed local array would put the whole kernel on scratch)
__device__ __forceinline__ void publish_body(const PubArgs& a, bool own01, int32_t t0, int32_t t1,
                                             int t, int nthr) {
  // (the sticky look-back error word, read coherently at agent scope.  A predecessor tile whose
  // aggregate the last tile already summed can still give up after this publish: that failure
  // then surfaces at the next publish or at the extraction's end check, and the extraction throws
  // -- a round is never consumed silently from a failed compaction.  The relaxed agent-scope
  // atomics + s_waitcnt(0) handoffs here and in moments_tail / the fused pick rely on gfx9's
  // in-order L2 write-back at agent scope.)
  if (t == 0)
    a.pub[kPubErr] = a.err ? __hip_atomic_load(a.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0;
  for (int i = t; i < a.ntot; i += nthr)
    a.pub[kPubTot + i] = own01 && i < 2 ? (i == 0 ? t0 : t1) : a.totals[i];
  for (int i = t; i < 4 * a.nsmall; i += nthr)
    a.pub[kPubSmall + i] = __float_as_int(reinterpret_cast<const float*>(a.small)[i]);
  for (int i = t; i < a.npick; i += nthr) a.pub[kPubPick + i] = a.pick[i];
  for (int i = t; i < a.nrk; i += nthr) a.pub[kPubRk + i] = a.rk[i];
  for (int i = t; i < a.nres; i += nthr) a.pub[kPubRk + a.nrk + i] = a.res[i];
  __threadfence_system();
  __syncthreads();
  if (t == 0) __hip_atomic_store(a.pub, a.seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

__global__ __launch_bounds__(256) void k_publish(PubArgs a) {
  publish_body(a, false, 0, 0, threadIdx.x, 256);
}

// ---------------------------------------------------------------------------------------------
// select / compact (selectWithinDistance + removal of the inliers from the active list)
constexpr int kSelBS = 256;
constexpr int kSelIt = kSelTile / kSelBS;

template <bool NP>
__global__ __launch_bounds__(kSelBS) void k_select_count(PointsView src,
                                                         const float4* __restrict__ cfp,
                                                         ModelTest mt,
                                                         int32_t* __restrict__ tile_in) {
  const float4 cf = *cfp;
  const float4 cn = eigen_normalized3(cf.x, cf.y, cf.z, 0.0f);
  __shared__ int s_w[kSelBS / kWave];
  const int64_t base = (int64_t)blockIdx.x * kSelTile;
  int cnt = 0;
#pragma unroll 4
  for (int j = 0; j < kSelIt; ++j) {
    int64_t e = base + j * kSelBS + threadIdx.x;
    bool in = false;
    if (e < src.n) in = model_in<NP>(src, e, cf, cn, mt, src.x[e], src.y[e], src.z[e]);
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

template <bool NP>
__global__ __launch_bounds__(kSelBS) void k_select_scatter(PointsView src,
                                                           const float4* __restrict__ cfp,
                                                           ModelTest mt,
                                                           const int32_t* __restrict__ off_in,
                                                           const int32_t* __restrict__ off_out,
                                                           int32_t* __restrict__ inl_gid,
                                                           float* __restrict__ inl_xyz,
                                                           PointsOut dst, int compact) {
  __shared__ int s_w[2][2][kSelBS / kWave];  // [buffer][in/out][wave]
  const float4 cf = *cfp;
  const float4 cn = eigen_normalized3(cf.x, cf.y, cf.z, 0.0f);
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
      in = model_in<NP>(src, e, cf, cn, mt, x, y, z);
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
      if (inl_gid) inl_gid[p] = g;
      if (inl_xyz) {
        inl_xyz[3 * (int64_t)p] = x; inl_xyz[3 * (int64_t)p + 1] = y; inl_xyz[3 * (int64_t)p + 2] = z;
      }
    } else if (valid && compact) {
      int p = run_out + wo + lanes_below(mo);
      dst.x[p] = x; dst.y[p] = y; dst.z[p] = z; dst.gid[p] = g;
      if (dst.nrm) dst.nrm[p] = src.nrm[e];
    }
    run_in += ti;
    run_out += to;
  }
}

// ---------------------------------------------------------------------------------------------
// Single-pass select / compaction (the "lean list" rounds).  The plane's inliers are decided
// once, on the Morton copy: k_sel1_morton compacts the survivors of the Morton copy and stamps
// each inlier's pristine index in a byte array with the select's tag; the active list, which
// then only holds pristine indices (ascending: list order is pristine order minus the removed
// points), is compacted by k_sel1_list from the stamps alone, emitting the inlier ids in list
// order (PCL's order) -- 9 B per list point instead of the 44 B of count + scatter over the
// list-ordered xyz.
//
// Both are one pass: workgroup t takes tile t (BS threads x 16 points, BS = 256 / 512 / 1024:
// 4096 / 8192 / 16384-point tiles, kSel1Points), counts its inliers, and takes its exclusive
// prefix by decoupled look-back over the tile status words (epoch << 32 | flag << 30 | value;
// flag 1 = tile aggregate, 2 = inclusive prefix).  Survivor positions need no second scan: every
// tile but the last is full, so the survivors before element e of tile t are t * tile + local(e)
// - (inliers before e).  Large tiles keep the look-back short (each window of 64 tiles costs one
// uncached round trip); small ones let several workgroups share a CU, so one tile's loads
// overlap another's scan and scatter (one 1024-thread workgroup of 128 VGPRs fills a CU alone).
constexpr int kS1It = 16;  // points per lane, lane-strided
template <int BS>
struct S1 {
  static constexpr int kTile = BS * kS1It;
  static constexpr int kSlots = kS1It * (BS / kWave);  // (j, wave) counts of a tile
  static_assert(kSlots % kWave == 0 && kSlots <= BS, "slot scan layout");
};

// Tile numbering (sel1_tile_of).  With L.ticket (the default) a workgroup's tile is the ticket
// it takes when it starts, so a tile's predecessors have all started -- they are resident or done
// -- and the lowest unfinished tile of the launch can always finish, whatever else occupies the
// device.  Numbering by workgroup index is only safe while the launch has the device to itself:
// workgroups are dispatched in index order per XCD, not across XCDs, so beside another spinning
// kernel (another context's select on the same device: the loopback groups of the tests) tile t
// can spin on tile t - 1 whose XCD is full of the other kernel's spinning tiles, which wait in
// turn on theirs -- a circular wait that only the spin limit below ends (measured: the round-5
// 8-context hang).  The look-back still carries that exit: after kS1Spin empty
// polls the tile gives up, scatters nothing, publishes flag 3 (failed) and sets the sticky error
// word *L.err, which the last tile never writes; a tile whose look-back meets a failed tile fails
// the same way.  (A successor may already have summed a failed tile's aggregate and completed:
// only the sticky word is reliable, so the host checks it -- in the round's publish for
// k_sel1_morton, at the next publish / the end of the extraction for k_sel1_list.)
constexpr int kS1Spin = 1 << 20;

__device__ __forceinline__ int sel1_tile_of(const Sel1State& L, int* s_tile) {
  if (!L.ticket) return blockIdx.x;
  if (threadIdx.x == 0)
    *s_tile = (int)(__hip_atomic_fetch_add(L.ticket, 1ull, __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_AGENT) - L.base);
  __syncthreads();
  return __builtin_amdgcn_readfirstlane(*s_tile);
}

// in-tile exclusive ranks from the (j, wave) counts in s_cnt, the tile's exclusive prefix by
// look-back; returns the prefix (workgroup-uniform), s_pre[] = in-tile exclusive offsets
template <int BS>
__device__ __forceinline__ int sel1_scan(const Sel1State& L, int tile, int* s_cnt, int* s_pre,
                                         int* s_base) {
  constexpr int kS1Slots = S1<BS>::kSlots;
  __shared__ int s_wt[kS1Slots / kWave];
  __syncthreads();
  const int t = threadIdx.x, lane = t & (kWave - 1);
  int v = 0, inc = 0;
  if (t < kS1Slots) {
    v = s_cnt[t];
    inc = v;
#pragma unroll
    for (int off = 1; off < kWave; off <<= 1) {
      const int u = __shfl_up(inc, off, kWave);
      if (lane >= off) inc += u;
    }
    if (lane == kWave - 1) s_wt[t / kWave] = inc;
  }
  __syncthreads();
  int agg = 0;
#pragma unroll
  for (int q = 0; q < kS1Slots / kWave; ++q) {
    if (t < kS1Slots && q < t / kWave) inc += s_wt[q];
    agg += s_wt[q];
  }
  if (t < kS1Slots) s_pre[t] = inc - v;
  if (t < kWave) {
    const uint64_t ep = (uint64_t)L.epoch << 32;
    int excl = 0;
    if (tile == 0) {
      if (lane == 0)
        __hip_atomic_store(L.status, ep | (2ull << 30) | (uint32_t)agg, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
    } else {
      if (lane == 0)
        __hip_atomic_store(L.status + tile, ep | (1ull << 30) | (uint32_t)agg, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
      // K windows of 64 tiles per round trip: with every tile of a round resident at once,
      // a tile's nearest published prefix can be hundreds of tiles back
      constexpr int K = 1;
      int look = tile - 1, spins = 0;
      for (;;) {
        uint32_t f[K], val[K];
#pragma unroll
        for (int k = 0; k < K; ++k) {
          const int idx = look - lane - k * kWave;
          f[k] = 2u;
          val[k] = 0u;
          if (idx >= 0) {
            const uint64_t w = __hip_atomic_load(L.status + idx, __ATOMIC_RELAXED,
                                                 __HIP_MEMORY_SCOPE_AGENT);
            f[k] = (uint32_t)(w >> 32) == L.epoch ? (uint32_t)(w >> 30) & 3u : 0u;
            val[k] = (uint32_t)w & 0x3FFFFFFFu;
          }
        }
        // the nearest window holding a prefix, and the lanes of it that are needed
        int kp = K, fp = kWave;
        bool missing = false, failed = false;
#pragma unroll
        for (int k = 0; k < K; ++k) {
          if (kp == K && !missing && !failed) {
            const uint64_t pm = ballot(f[k] == 2u), zm = ballot(f[k] == 0u);
            const uint64_t fm = ballot(f[k] == 3u);
            const int q = pm ? __builtin_ctzll(pm) : kWave;
            const uint64_t need = q >= kWave - 1 ? ~0ull : ((2ull << q) - 1ull);
            if (fm & need) failed = true;
            else if (zm & need) missing = true;
            else if (q < kWave) { kp = k; fp = q; }
          }
        }
        if (failed) {
          excl = -1;
          break;
        }
        if (missing) {
          if (++spins > kS1Spin) {
            excl = -1;
            break;
          }
          __builtin_amdgcn_s_sleep(1);
          continue;  // a tile in range has not published yet
        }
        int c = 0;
#pragma unroll
        for (int k = 0; k < K; ++k)
          c += (k < kp || (k == kp && lane <= fp)) ? (int)val[k] : 0;
#pragma unroll
        for (int off = kWave / 2; off > 0; off >>= 1) c += __shfl_xor(c, off, kWave);
        excl += c;
        if (kp < K) break;
        look -= K * kWave;
      }
      if (lane == 0) {
        if (excl >= 0) {
          __hip_atomic_store(L.status + tile, ep | (2ull << 30) | (uint32_t)(excl + agg),
                             __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        } else {  // failed: successors fail too; the sticky word tells the host
          __hip_atomic_store(L.status + tile, ep | (3ull << 30), __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_AGENT);
          atomicOr(L.err, 1);
        }
      }
    }
    if (lane == 0) {
      s_base[0] = excl;
      s_base[1] = agg;
    }
  }
  __syncthreads();
  return s_base[0];
}

// the Morton copy's select: survivors compacted into dst (Morton order kept), inliers stamped
// in tag[] by pristine index (the Morton copy's gid field holds it); the last tile writes
// totals[0] = inliers, totals[1] = list survivors (n_list - inliers), totals[4] = Morton survivors
// pa.pub non-null: the last tile also publishes the round (publish_body) once its totals are
// final, without waiting for the other tiles' scatters (nothing published depends on them)
template <bool NP, int kS1BS>
__global__ __launch_bounds__(kS1BS) void k_sel1_morton(PointsView src, const float4* __restrict__ cfp,
                                                       ModelTest mt, Sel1State L,
                                                       uint8_t* __restrict__ tag, uint8_t tagv,
                                                       PointsOut dst, int64_t n_list, int ntiles,
                                                       int32_t* __restrict__ totals, PubArgs pa) {
  constexpr int kS1Slots = S1<kS1BS>::kSlots, kS1Tile = S1<kS1BS>::kTile;
  __shared__ int s_cnt[kS1Slots], s_pre[kS1Slots], s_base[2];
  const int tile = sel1_tile_of(L, s_base);
  const float4 cf = *cfp;
  const float4 cn = eigen_normalized3(cf.x, cf.y, cf.z, 0.0f);
  const int w = threadIdx.x / kWave;
  const int64_t base = (int64_t)tile * kS1Tile;
  float x[kS1It], y[kS1It], z[kS1It];
  int32_t g[kS1It];
  uint64_t m[kS1It];
  // (clamped, unconditional loads: all 64 in flight at once; a guarded load per element would
  // be a branch, and the compiler waits for each before the next)
#pragma unroll
  for (int j = 0; j < kS1It; ++j) {
    const int64_t e = min<int64_t>(base + j * kS1BS + threadIdx.x, src.n - 1);
    x[j] = src.x[e]; y[j] = src.y[e]; z[j] = src.z[e]; g[j] = src.gid[e];
  }
#pragma unroll
  for (int j = 0; j < kS1It; ++j) {
    const int64_t e = base + j * kS1BS + threadIdx.x;
    const bool in = e < src.n && model_in<NP>(src, e, cf, cn, mt, x[j], y[j], z[j]);
    m[j] = ballot(in);
    if ((threadIdx.x & (kWave - 1)) == 0) s_cnt[j * (kS1BS / kWave) + w] = __popcll(m[j]);
  }
  const int excl = sel1_scan<kS1BS>(L, tile, s_cnt, s_pre, s_base);
  if (excl < 0) return;  // (look-back failed: *L.err is set)
#pragma unroll
  for (int j = 0; j < kS1It; ++j) {
    const int64_t e = base + j * kS1BS + threadIdx.x;
    if (e >= src.n) break;
    const int r = s_pre[j * (kS1BS / kWave) + w] + lanes_below(m[j]);  // inliers before e in tile
    if ((m[j] >> (threadIdx.x & (kWave - 1))) & 1ull) {
      tag[g[j]] = tagv;
    } else {
      const int64_t q = base + j * kS1BS + threadIdx.x - (excl + r);
      dst.x[q] = x[j]; dst.y[q] = y[j]; dst.z[q] = z[j]; dst.gid[q] = g[j];
      if (dst.nrm) dst.nrm[q] = src.nrm[e];  // (normals travel when the copy has them)
    }
  }
  if (tile == ntiles - 1) {
    const int in = excl + s_base[1];
    if (threadIdx.x == 0) {
      totals[0] = in;
      totals[1] = (int32_t)(n_list - in);
      totals[4] = (int32_t)(src.n - in);
    }
    if (pa.pub) {
      publish_body(pa, true, in, (int32_t)(n_list - in), threadIdx.x, kS1BS);
    }
  }
}

// the active list's compaction from the stamps: lidx = pristine index per list point (null: the
// pristine list, lidx[e] = e); inliers -> inl_gid (their ids, list order), survivors' pristine
// indices -> out_lidx; the last tile writes totals[0..1] = (inliers, survivors)
template <bool IDENT, bool GID_IDENT, int kS1BS>
__global__ __launch_bounds__(kS1BS) void k_sel1_list(const int32_t* __restrict__ lidx, int64_t n,
                                                     const uint8_t* __restrict__ tag, uint8_t tagv,
                                                     const int32_t* __restrict__ pgid, int32_t gid_base,
                                                     Sel1State L,
                                                     int32_t* __restrict__ inl_gid,
                                                     int32_t* __restrict__ out_lidx, int ntiles,
                                                     int32_t* __restrict__ totals) {
  constexpr int kS1Slots = S1<kS1BS>::kSlots, kS1Tile = S1<kS1BS>::kTile;
  __shared__ int s_cnt[kS1Slots], s_pre[kS1Slots], s_base[2];
  const int tile = sel1_tile_of(L, s_base);
  const int w = threadIdx.x / kWave;
  const int64_t base = (int64_t)tile * kS1Tile;
  int32_t p[kS1It];
  uint8_t tv[kS1It];
  uint64_t m[kS1It];
#pragma unroll
  for (int j = 0; j < kS1It; ++j) {
    const int64_t e = min<int64_t>(base + j * kS1BS + threadIdx.x, n - 1);
    p[j] = IDENT ? (int32_t)e : lidx[e];
  }
#pragma unroll
  for (int j = 0; j < kS1It; ++j) tv[j] = tag[p[j]];
#pragma unroll
  for (int j = 0; j < kS1It; ++j) {
    const int64_t e = base + j * kS1BS + threadIdx.x;
    const bool in = e < n && tv[j] == tagv;
    m[j] = ballot(in);
    if ((threadIdx.x & (kWave - 1)) == 0) s_cnt[j * (kS1BS / kWave) + w] = __popcll(m[j]);
  }
  // the inliers' ids, loaded before the scan so the loads overlap it (every lane loads: the
  // others re-read their first point's id, so no lane waits on a branch)
  int32_t gi[kS1It];
#pragma unroll
  for (int j = 0; j < kS1It; ++j)
    gi[j] = GID_IDENT ? gid_base + p[j] : pgid[((m[j] >> (threadIdx.x & (kWave - 1))) & 1ull) ? p[j] : p[0]];
  const int excl = sel1_scan<kS1BS>(L, tile, s_cnt, s_pre, s_base);
  if (excl < 0) return;  // (look-back failed: *L.err is set)
#pragma unroll
  for (int j = 0; j < kS1It; ++j) {
    const int64_t e = base + j * kS1BS + threadIdx.x;
    if (e >= n) break;
    const int r = s_pre[j * (kS1BS / kWave) + w] + lanes_below(m[j]);
    if ((m[j] >> (threadIdx.x & (kWave - 1))) & 1ull)
      inl_gid[excl + r] = gi[j];
    else
      out_lidx[base + j * kS1BS + threadIdx.x - (excl + r)] = p[j];
  }
  if (tile == ntiles - 1 && threadIdx.x == 0) {
    const int in = excl + s_base[1];
    totals[0] = in;
    totals[1] = (int32_t)(n - in);
  }
}

// k_ulist (PCL refit in lean rounds, DLG_OPT_UNREFINED_PASS 1): the unrefined plane's inliers in
// list order straight from the list -- lane-strided list entries (16 a lane), their pristine
// coordinates gathered by index (ascending: coalesced while the list is dense), the model test,
// and the single-pass look-back compaction of the inliers' x, y, z (as k_sel1_list / k_ucompact);
// the last tile writes the count to *n_out.  The same inliers, in the same order, as k_ustamp +
// k_ucompact (the Morton copy holds the same coordinates and runs the same test; the list is the
// active points' pristine indices ascending), in one pass instead of two and without the
// bitmap's scattered gather.
template <bool IDENT, bool NP, int kS1BS>
__global__ __launch_bounds__(kS1BS) void k_ulist(const int32_t* __restrict__ lidx, int64_t n,
                                                 PointsView pristine,
                                                 const float4* __restrict__ cfp, ModelTest mt,
                                                 Sel1State L, int ntiles, float* __restrict__ ox,
                                                 float* __restrict__ oy, float* __restrict__ oz,
                                                 int32_t* __restrict__ n_out) {
  constexpr int kS1Slots = S1<kS1BS>::kSlots, kS1Tile = S1<kS1BS>::kTile;
  __shared__ int s_cnt[kS1Slots], s_pre[kS1Slots], s_base[2];
  const int tile = sel1_tile_of(L, s_base);
  const float4 cf = *cfp;
  const float4 cn = eigen_normalized3(cf.x, cf.y, cf.z, 0.0f);
  const int w = threadIdx.x / kWave;
  const int64_t base = (int64_t)tile * kS1Tile;
  int32_t p[kS1It];
  float x[kS1It], y[kS1It], z[kS1It];
  uint64_t m[kS1It];
#pragma unroll
  for (int j = 0; j < kS1It; ++j) {
    const int64_t e = min<int64_t>(base + j * kS1BS + threadIdx.x, n - 1);
    p[j] = IDENT ? (int32_t)e : lidx[e];
  }
#pragma unroll
  for (int j = 0; j < kS1It; ++j) {
    x[j] = pristine.x[p[j]]; y[j] = pristine.y[p[j]]; z[j] = pristine.z[p[j]];
  }
#pragma unroll
  for (int j = 0; j < kS1It; ++j) {
    const int64_t e = base + j * kS1BS + threadIdx.x;
    const bool in = e < n && model_in<NP>(pristine, p[j], cf, cn, mt, x[j], y[j], z[j]);
    m[j] = ballot(in);
    if ((threadIdx.x & (kWave - 1)) == 0) s_cnt[j * (kS1BS / kWave) + w] = __popcll(m[j]);
  }
  const int excl = sel1_scan<kS1BS>(L, tile, s_cnt, s_pre, s_base);
  if (excl < 0) return;  // (look-back failed: *L.err is set)
#pragma unroll
  for (int j = 0; j < kS1It; ++j) {
    const int64_t e = base + j * kS1BS + threadIdx.x;
    if (e >= n) break;
    if ((m[j] >> (threadIdx.x & (kWave - 1))) & 1ull) {
      const int o = excl + s_pre[j * (kS1BS / kWave) + w] + lanes_below(m[j]);
      ox[o] = x[j]; oy[o] = y[j]; oz[o] = z[j];
    }
  }
  if (tile == ntiles - 1 && threadIdx.x == 0) *n_out = excl + s_base[1];
}

__global__ void k_sel1_empty(int64_t n_list, int32_t* totals) {
  totals[0] = 0;
  totals[1] = (int32_t)n_list;
  totals[4] = 0;
}

// the list's x, y, z, gid (+ normals) from the pristine copy by pristine index, in place (a
// lean list is materialised before any path that reads its coordinates)
__global__ void k_list_materialize(PointsView pristine, int64_t n, PointsOut io) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= n) return;
  const int32_t p = io.gid[e];
  io.x[e] = pristine.x[p];
  io.y[e] = pristine.y[p];
  io.z[e] = pristine.z[p];
  io.gid[e] = pristine.gid[p];
  if (io.nrm) io.nrm[e] = pristine.nrm[p];
}

// ---------------------------------------------------------------------------------------------
// PCL refit in lean rounds: the unrefined plane's inliers in list order, without list
// coordinates.  A lean list is the ascending pristine indices of the active points, so "inliers
// in list order" = the set bits of a bitmap over pristine indices, ascending.
// k_ustamp: the Morton copy's tiles whose sphere may hold an inlier (k_moments_sp's walk) set the
// bit of each inlier's pristine index (the copy's gid field).  The bitmap is all-zero on entry
// (k_ucompact clears every word it reads).
template <bool NP>
__global__ __launch_bounds__(kMoBS) void k_ustamp(PointsView src, const float4* __restrict__ tiles,
                                                  const float4* __restrict__ supers, float margin,
                                                  const float4* __restrict__ cfp, ModelTest mt,
                                                  uint32_t* __restrict__ bits) {
  const float4 cf = *cfp;
  const float4 cn = eigen_normalized3(cf.x, cf.y, cf.z, 0.0f);
  const int64_t nsup = (src.n + kSuperP - 1) / kSuperP, ntile = (src.n + kTileP - 1) / kTileP;
  const int lane = threadIdx.x & (kWave - 1);
  const int64_t W = (int64_t)gridDim.x * (kMoBS / kWave);
  const int64_t wid = (int64_t)blockIdx.x * (kMoBS / kWave) + threadIdx.x / kWave;
  constexpr int kIt = kSuperP / kWave;
  for (int64_t s0 = wid; s0 < nsup; s0 += kWave * W) {
    const int64_t sl = s0 + lane * W;
    uint64_t near = ballot(sl < nsup && sphere_near(cf, supers[sl], margin));
    while (near) {
      const int64_t s = s0 + (int64_t)(__ffsll((unsigned long long)near) - 1) * W;
      near &= near - 1;
      const int64_t tl = s * kSuperTiles + (lane & (kSuperTiles - 1));
      const uint32_t tm = (uint32_t)ballot(lane < kSuperTiles && tl < ntile &&
                                           sphere_near(cf, tiles[tl], margin));
      const int64_t base = s * kSuperP;
      float x[kIt], y[kIt], z[kIt];
      int32_t g[kIt];
#pragma unroll
      for (int j = 0; j < kIt; ++j) {
        const int64_t e = base + j * kWave + lane;
        if (((tm >> (2 * j + (lane >> 5))) & 1u) && e < src.n) {
          x[j] = src.x[e]; y[j] = src.y[e]; z[j] = src.z[e]; g[j] = src.gid[e];
        }
      }
#pragma unroll
      for (int j = 0; j < kIt; ++j) {
        const int64_t e = base + j * kWave + lane;
        if (((tm >> (2 * j + (lane >> 5))) & 1u) && e < src.n &&
            model_in<NP>(src, e, cf, cn, mt, x[j], y[j], z[j]))
          atomicOr(bits + (g[j] >> 5), 1u << (g[j] & 31));
      }
    }
  }
}

// k_ucompact: bitmap -> the inliers' x, y, z in ascending pristine order (= list order), a
// single pass with decoupled look-back (sel1_scan); each lane owns one word (32 points), clears
// it and ranks its inliers.  The gather is cooperative: the wave walks its lanes' words two at a
// time (64 consecutive points), lane i taking point i of each pair (coalesced, masked 4-byte
// loads and stores; four pairs in flight), so dense runs and sparse scatter cost the same.  (One
// word per lane: twice the workgroups of round 4's two, 35.4 -> 31.5 us per round at C3.)  The
// last tile writes the count to *n_out.
constexpr int kUcBS = 256;
constexpr int kUcWords = 1;  // words per lane (two lanes' words form one 64-point gather step)
__global__ __launch_bounds__(kUcBS) void k_ucompact(uint32_t* __restrict__ bits, int64_t nwords,
                                                    PointsView pristine, Sel1State L, int ntiles,
                                                    float* __restrict__ ox, float* __restrict__ oy,
                                                    float* __restrict__ oz,
                                                    int32_t* __restrict__ n_out) {
  constexpr int kSlots = S1<kUcBS>::kSlots;
  __shared__ int s_cnt[kSlots], s_pre[kSlots], s_base[2];
  const int tile = sel1_tile_of(L, s_base);
  const int lane = threadIdx.x & (kWave - 1), w = threadIdx.x / kWave;
  const int64_t w0 = ((int64_t)tile * kUcBS + threadIdx.x) * kUcWords;
  uint32_t m = 0;
  if (w0 < nwords) {
    m = bits[w0];
    bits[w0] = 0u;
  }
  const int cnt = __popc(m);
  int incl = cnt;
#pragma unroll
  for (int off = 1; off < kWave; off <<= 1) {
    const int u = __shfl_up(incl, off, kWave);
    if (lane >= off) incl += u;
  }
  // slot (j = 0, wave w) carries the wave's total: in-tile order is lane-major within a wave
  for (int t = threadIdx.x; t < kSlots; t += kUcBS) s_cnt[t] = 0;
  __syncthreads();
  if (lane == kWave - 1) s_cnt[w] = incl;
  const int excl = sel1_scan<kUcBS>(L, tile, s_cnt, s_pre, s_base);
  if (excl < 0) return;  // (look-back failed: *L.err is set; the words are cleared already)
  const int pos = excl + s_pre[w] + (incl - cnt);  // this lane's first output slot
  const int64_t wbase = ((int64_t)tile * kUcBS + w * kWave) * kUcWords * 32;  // the wave's point 0
  const uint32_t below_lo = lane < 32 ? (1u << lane) - 1u : 0xFFFFFFFFu;
  const uint32_t below_hi = lane < 32 ? 0u : (lane == 32 ? 0u : (1u << (lane - 32)) - 1u);
  // step k: the words of lanes s0 + 2k and s0 + 2k + 1 (64 consecutive points, the first
  // lane's output position)
  for (int s0 = 0; s0 < kWave; s0 += 8) {
    uint64_t mk[4];
    int ps[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      mk[k] = (uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)m, s0 + 2 * k) |
              ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)m, s0 + 2 * k + 1) << 32);
      ps[k] = __builtin_amdgcn_readlane(pos, s0 + 2 * k);
    }
    if ((mk[0] | mk[1] | mk[2] | mk[3]) == 0) continue;  // (wave-uniform)
    float x[4], y[4], z[4];
    bool on[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      on[k] = ((mk[k] >> lane) & 1u) != 0;
      if (on[k]) {
        const int64_t pi = wbase + (int64_t)(s0 + 2 * k) * 32 + lane;
        x[k] = pristine.x[pi]; y[k] = pristine.y[pi]; z[k] = pristine.z[pi];
      }
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      if (on[k]) {
        const int o = ps[k] + __popc((uint32_t)mk[k] & below_lo) +
                      __popc((uint32_t)(mk[k] >> 32) & below_hi);
        ox[o] = x[k]; oy[o] = y[k]; oz[o] = z[k];
      }
    }
  }
  if (tile == ntiles - 1 && threadIdx.x == 0) *n_out = excl + s_base[1];
}

// k_score_np: counts[h] for SACMODEL_NORMAL_PLANE.
//
// Per point the exact prefilter b = (1 - w) d_euclid < thr becomes one float compare: b is
// fl(omw * de) with omw fixed per point, monotone in de, so b < thr <=> de < lim where lim is the
// smallest float with fl(omw * lim) >= thr (found once per point per launch; lim = +inf when the
// prefilter does not apply: w < 0 or NaN, or omw <= 0).  The per-test cost is then the plane
// model's: 3 mul + 3 add + compare.  Points that pass go, with their b and the hypothesis, into a
// per-wave LDS queue; every 64 queued pairs are evaluated with full lanes (normalised-normal dot,
// clamp, acos, min(a, pi - a), weighted sum -- all in PCL's order) and counted with LDS atomics,
// so the double-precision acos path never runs in a mostly idle wavefront.
constexpr int kNpBS = 256;
constexpr int kNpWaves = kNpBS / kWave;
constexpr int kNpQ = 128;

template <int kNpP, int kNpHT>
__global__ __launch_bounds__(kNpBS) void k_score_np(PointsView src, const HypRec* __restrict__ hyps,
                                                    int D, double lambda, double thr,
                                                    int32_t* __restrict__ counts) {
  constexpr int kChunk = kNpBS * kNpP;
  __shared__ float4 s_coef[kNpHT + 1];
  __shared__ float4 s_cn[kNpHT];
  __shared__ int s_cnt[kMaxHypPerLaunch];
  __shared__ float4 s_pts[kNpWaves][kNpP * kWave];  // (n.normalized(), curvature) of the chunk
  __shared__ uint32_t s_qk[kNpWaves][kNpQ];         // point slot | tile-local hypothesis << 8
  __shared__ double s_qb[kNpWaves][kNpQ];           // b = (1 - w) d_euclid
  const int tid = threadIdx.x;
  const int lane = tid & (kWave - 1);
  const int wv = tid / kWave;
  for (int i = tid; i < D; i += kNpBS) s_cnt[i] = 0;
  const int64_t n = src.n;
  const int64_t nchunks = (n + kChunk - 1) / kChunk;
  const float qnan = __builtin_nanf("");
  for (int64_t ch = blockIdx.x; ch < nchunks; ch += gridDim.x) {
    float px[kNpP], py[kNpP], pz[kNpP], lim[kNpP];
    double omw[kNpP];
#pragma unroll
    for (int j = 0; j < kNpP; ++j) {
      const int64_t e = ch * kChunk + (int64_t)wv * (kNpP * kWave) + j * kWave + lane;
      const bool ok = e < n;
      px[j] = ok ? src.x[e] : qnan;
      py[j] = ok ? src.y[e] : qnan;
      pz[j] = ok ? src.z[e] : qnan;
      const float4 nn = ok ? src.nrm[e] : make_float4(0.f, 0.f, 0.f, 0.f);
      const double w = lambda * (1.0 - (double)nn.w);
      omw[j] = 1.0 - w;
      lim[j] = ok ? np_de_limit(w, thr) : 0.0f;
      s_pts[wv][j * kWave + lane] = nn;
    }
    for (int t0 = 0; t0 < D; t0 += kNpHT) {
      const int nt = min(kNpHT, D - t0);
      __syncthreads();
      for (int i = tid; i < nt; i += kNpBS) {
        const HypRec hr = hyps[t0 + i];
        s_coef[i] = make_float4(hr.a, hr.b, hr.c, hr.d);
        s_cn[i] = eigen_normalized3(hr.a, hr.b, hr.c, 0.0f);
      }
      __syncthreads();
      int qn = 0;  // wave-uniform queue length
      auto drain = [&](int m) {  // evaluate the first m queued pairs, keep the rest
        __builtin_amdgcn_wave_barrier();  // queue writes of other lanes precede these reads
        if (lane < m) {
          const uint32_t e = s_qk[wv][lane];
          const float4 nn = s_pts[wv][e & 255u];
          const int kk = (int)(e >> 8);
          const double w = lambda * (1.0 - (double)nn.w);
          if (np_full(s_cn[kk], nn, w, s_qb[wv][lane], thr)) atomicAdd(&s_cnt[t0 + kk], 1);
        }
        const int rest = qn - m;
        uint32_t mk = 0;
        double mb = 0.0;
        if (lane < rest) {
          mk = s_qk[wv][m + lane];
          mb = s_qb[wv][m + lane];
        }
        if (lane < rest) {
          s_qk[wv][lane] = mk;
          s_qb[wv][lane] = mb;
        }
        qn = rest;
      };
      float4 cnext = s_coef[0];  // software pipeline: next plane's LDS read in flight
      for (int k = 0; k < nt; ++k) {
        const float4 c = cnext;
        cnext = s_coef[k + 1];
#pragma unroll
        for (int j = 0; j < kNpP; ++j) {
          const float de = np_deuclid(c, px[j], py[j], pz[j]);
          const bool near = de < lim[j];
          const uint64_t m = ballot(near);
          if (near) {
            const int pos = qn + lanes_below(m);
            s_qk[wv][pos] = (uint32_t)(j * kWave + lane) | ((uint32_t)k << 8);
            s_qb[wv][pos] = omw[j] * (double)de;
          }
          qn += __popcll(m);
          if (qn >= kWave) drain(kWave);
        }
      }
      if (qn > 0) drain(qn);  // the tile's coefficients are replaced next
    }
  }
  __syncthreads();
  for (int i = tid; i < D; i += kNpBS) {
    const int v = s_cnt[i];
    if (v) atomicAdd(&counts[i], v);
  }
}

__global__ void k_pack_point_normals(const float* __restrict__ raw, int64_t stride_f, int curv_off,
                                     PointsView src, int32_t id_base, float4* __restrict__ out,
                                     int normalize) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= src.n) return;
  // (gid null: the records follow the list's positions)
  const float* r = raw + (src.gid ? (int64_t)(src.gid[e] - id_base) : e) * stride_f;
  out[e] = normalize ? eigen_normalized3(r[0], r[1], r[2], r[curv_off])
                     : make_float4(r[0], r[1], r[2], r[curv_off]);
}

// dlg_cloud_upload: caller records (stride_f floats, xyz first) -> SoA + global ids
__global__ void k_upload_gather(const float* __restrict__ raw, int64_t stride_f,
                                const int32_t* __restrict__ idx, int64_t n, int32_t id_base,
                                PointsOut out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int64_t k = idx ? idx[i] : i;
  const float* p = raw + k * stride_f;
  out.x[i] = p[0];
  out.y[i] = p[1];
  out.z[i] = p[2];
  out.gid[i] = (int32_t)(id_base + k);
}

__global__ void k_absmax(PointsView src, uint32_t* __restrict__ out4) {
  float m[4] = {0.f, 0.f, 0.f, 0.f};
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < src.n; e += stride) {
    const float ax = fabsf(src.x[e]), ay = fabsf(src.y[e]), az = fabsf(src.z[e]);
    m[0] = fmaxf(m[0], ax);
    m[1] = fmaxf(m[1], ay);
    m[2] = fmaxf(m[2], az);
    // the largest finite |coordinate| of the finite points (fast refit quantum)
    if (ax < INFINITY && ay < INFINITY && az < INFINITY) m[3] = fmaxf(m[3], fmaxf(ax, fmaxf(ay, az)));
  }
  for (int k = 0; k < 4; ++k) {
    float v = m[k];
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v = fmaxf(v, __shfl_xor(v, off, kWave));
    // non-negative floats order like their bit patterns; NaN/inf -> +inf bits dominate
    if ((threadIdx.x & (kWave - 1)) == 0) atomicMax(&out4[k], __float_as_uint(v));
  }
}

}  // namespace

// ---------------------------------------------------------------------------------------------
static inline unsigned cdiv(int64_t a, int64_t b) { return (unsigned)((a + b - 1) / b); }

void launch_gather_samples(const int32_t* pos, int m, int64_t lo, PointsView src, SampleRec* out,
                           hipStream_t s, const int32_t* lidx, int64_t n_list) {
  if (m <= 0) return;
  hipLaunchKernelGGL(k_gather_samples, dim3(cdiv(m, 256)), dim3(256), 0, s, pos, m, lo, src, lidx,
                     lidx || n_list ? n_list : src.n, out);
}

void launch_gather_build(const int32_t* pos_host, int D, PointsView src, SampleRec* samples,
                         float cthr, float ax, float ay, float az, HypRec* hyps, int32_t* res,
                         hipStream_t s, const int32_t* lidx, int64_t n_list) {
  if (D <= 0) return;
  const int Dp = (D + 63) / 64 * 64;
  hipLaunchKernelGGL(k_gather_build, dim3(cdiv(Dp, 256)), dim3(256), 0, s, pos_host, D, Dp, src,
                     lidx, lidx ? n_list : src.n, samples, cthr, ax, ay, az, hyps, res);
}

int sel1_tiles(int64_t n) { return (int)((n + kSel1Points[0] - 1) / kSel1Points[0]); }

// single-pass selects (lean-list rounds): every launch stamps its status words with a fresh epoch
// and (tickets) the first ticket of the launch
static void sel1_next(Sel1State& L, int nt) {
  ++L.epoch;
  if (L.ticket) {
    L.base = L.issued;
    L.issued += (uint64_t)nt;
  }
}

template <bool NP, int BS>
static void sel1_morton_bs(PointsView sp, const float4* coef, const ModelTest& mt, Sel1State& L,
                           uint8_t* tag, uint8_t tagv, const PointsOut& dst, int64_t n_list,
                           int nt, int32_t* totals, hipStream_t s, const PubArgs& pa) {
  hipLaunchKernelGGL((k_sel1_morton<NP, BS>), dim3(nt), dim3(BS), 0, s, sp, coef, mt, L, tag, tagv,
                     dst, n_list, nt, totals, pa);
}

template <bool NP>
static void sel1_morton_np(PointsView sp, const float4* coef, const ModelTest& mt, Sel1State& L,
                           uint8_t* tag, uint8_t tagv, const PointsOut& dst, int64_t n_list,
                           int nt, int32_t* totals, hipStream_t s, const PubArgs& pa, int bs) {
  if (bs == 256) sel1_morton_bs<NP, 256>(sp, coef, mt, L, tag, tagv, dst, n_list, nt, totals, s, pa);
  else if (bs == 512) sel1_morton_bs<NP, 512>(sp, coef, mt, L, tag, tagv, dst, n_list, nt, totals, s, pa);
  else sel1_morton_bs<NP, 1024>(sp, coef, mt, L, tag, tagv, dst, n_list, nt, totals, s, pa);
}

static int sel1_bs(int tile_pts) {
  return tile_pts == kSel1Points[0] ? 256 : tile_pts == kSel1Points[1] ? 512 : 1024;
}

void launch_sel1_morton(PointsView sp, const float4* coef, const ModelTest& mt, Sel1State& L,
                        uint8_t* tag, uint8_t tagv, const PointsOut& dst, int64_t n_list,
                        int32_t* totals, hipStream_t s, const PubArgs* pub, int tile_pts) {
  const int bs = sel1_bs(tile_pts);
  const int nt = (int)((sp.n + bs * kS1It - 1) / (bs * kS1It));
  if (nt == 0) {
    hipLaunchKernelGGL(k_sel1_empty, dim3(1), dim3(1), 0, s, n_list, totals);
    if (pub) hipLaunchKernelGGL(k_publish, dim3(1), dim3(256), 0, s, *pub);
    return;
  }
  sel1_next(L, nt);
  PubArgs pa{};
  if (pub) pa = *pub;
  if (mt.normal_plane)
    sel1_morton_np<true>(sp, coef, mt, L, tag, tagv, dst, n_list, nt, totals, s, pa, bs);
  else
    sel1_morton_np<false>(sp, coef, mt, L, tag, tagv, dst, n_list, nt, totals, s, pa, bs);
}

template <bool IDENT, bool GID_IDENT>
static void sel1_list_k(const int32_t* lidx, int64_t n, const uint8_t* tag, uint8_t tagv,
                        const int32_t* pgid, int32_t gid_base, Sel1State& L, int32_t* inl_gid,
                        int32_t* out_lidx, int nt, int32_t* totals, hipStream_t s, int bs) {
  if (bs == 256)
    hipLaunchKernelGGL((k_sel1_list<IDENT, GID_IDENT, 256>), dim3(nt), dim3(256), 0, s, lidx, n, tag,
                       tagv, pgid, gid_base, L, inl_gid, out_lidx, nt, totals);
  else if (bs == 512)
    hipLaunchKernelGGL((k_sel1_list<IDENT, GID_IDENT, 512>), dim3(nt), dim3(512), 0, s, lidx, n, tag,
                       tagv, pgid, gid_base, L, inl_gid, out_lidx, nt, totals);
  else
    hipLaunchKernelGGL((k_sel1_list<IDENT, GID_IDENT, 1024>), dim3(nt), dim3(1024), 0, s, lidx, n,
                       tag, tagv, pgid, gid_base, L, inl_gid, out_lidx, nt, totals);
}

void launch_sel1_list(const int32_t* lidx, int64_t n, const uint8_t* tag, uint8_t tagv,
                      const int32_t* pgid, int32_t gid_base, Sel1State& L, int32_t* inl_gid,
                      int32_t* out_lidx, int32_t* totals, hipStream_t s, int tile_pts) {
  const int bs = sel1_bs(tile_pts);
  const int nt = (int)((n + bs * kS1It - 1) / (bs * kS1It));
  if (nt == 0) {
    (void)hipMemsetAsync(totals, 0, 2 * sizeof(int32_t), s);
    return;
  }
  sel1_next(L, nt);
  if (lidx) {
    if (pgid)
      sel1_list_k<false, false>(lidx, n, tag, tagv, pgid, gid_base, L, inl_gid, out_lidx, nt, totals, s, bs);
    else
      sel1_list_k<false, true>(lidx, n, tag, tagv, pgid, gid_base, L, inl_gid, out_lidx, nt, totals, s, bs);
  } else {
    if (pgid)
      sel1_list_k<true, false>(lidx, n, tag, tagv, pgid, gid_base, L, inl_gid, out_lidx, nt, totals, s, bs);
    else
      sel1_list_k<true, true>(lidx, n, tag, tagv, pgid, gid_base, L, inl_gid, out_lidx, nt, totals, s, bs);
  }
}

void launch_list_materialize(PointsView pristine, int64_t n, const PointsOut& io, hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_list_materialize, dim3(cdiv(n, 256)), dim3(256), 0, s, pristine, n, io);
}

void launch_ustamp(PointsView sp, const float4* tiles, const float4* supers, float margin,
                   const float4* coef, const ModelTest& mt, uint32_t* bits, hipStream_t s) {
  if (sp.n <= 0) return;
  const int g = (int)std::max<int64_t>(1, std::min<int64_t>(4 * 256, sp_supers(sp.n)));
  // (NORMAL_PLANE: the model test reads the copy's normals, sp.nrm; margin = the NP prune margin)
  hipLaunchKernelGGL(mt.normal_plane ? k_ustamp<true> : k_ustamp<false>, dim3(g), dim3(kMoBS), 0, s,
                     sp, tiles, supers, margin, coef, mt, bits);
}

void launch_ulist(const int32_t* lidx, int64_t n, PointsView pristine, const float4* coef,
                  const ModelTest& mt, Sel1State& L, float* ox, float* oy, float* oz,
                  int32_t* n_out, hipStream_t s) {
  constexpr int kBS = 1024;
  const int nt = (int)((n + kBS * kS1It - 1) / (kBS * kS1It));
  if (nt == 0) {
    (void)hipMemsetAsync(n_out, 0, sizeof(int32_t), s);
    return;
  }
  sel1_next(L, nt);
  auto* k = lidx ? (mt.normal_plane ? k_ulist<false, true, kBS> : k_ulist<false, false, kBS>)
                 : (mt.normal_plane ? k_ulist<true, true, kBS> : k_ulist<true, false, kBS>);
  hipLaunchKernelGGL(k, dim3(nt), dim3(kBS), 0, s, lidx, n, pristine, coef, mt, L, nt, ox, oy, oz,
                     n_out);
}

int ucompact_tiles(int64_t nwords) { return (int)((nwords + kUcBS * kUcWords - 1) / (kUcBS * kUcWords)); }

void launch_ucompact(uint32_t* bits, int64_t nwords, PointsView pristine, Sel1State& L, float* ox,
                     float* oy, float* oz, int32_t* n_out, hipStream_t s) {
  const int nt = ucompact_tiles(nwords);
  if (nt == 0) {
    (void)hipMemsetAsync(n_out, 0, sizeof(int32_t), s);
    return;
  }
  sel1_next(L, nt);
  hipLaunchKernelGGL(k_ucompact, dim3(nt), dim3(kUcBS), 0, s, bits, nwords, pristine, L, nt, ox,
                     oy, oz, n_out);
}

void launch_build_hyps(const SampleRec* samples, int D, float cthr, float ax, float ay, float az,
                       HypRec* hyps, int32_t* good, hipStream_t s) {
  if (D <= 0) return;
  const int Dp = (D + 63) / 64 * 64;
  hipLaunchKernelGGL(k_build_hyps, dim3(cdiv(Dp, 256)), dim3(256), 0, s, samples, D, Dp, cthr, ax,
                     ay, az, hyps, good);
}

template <int P>
static void launch_score_t(PointsView src, const HypRec* hyps, int D, float cthr, int32_t* counts,
                           int num_cus, hipStream_t s) {
  constexpr int kChunk = kScBS * P;
  D = (D + kWave - 1) / kWave * kWave;  // hyps[D..Dp) are NaN planes; counts has room
  const int64_t nchunks = (src.n + kChunk - 1) / kChunk;
  // resident capacity: 4 workgroups (32 waves) per CU.  Work units = (point chunk, hypothesis
  // slice): slices of <= 1024 planes (one LDS load per workgroup), narrowed while there are too
  // few units to fill the chip several times over (small active lists in late extract rounds),
  // and the workgroups of a slice stride over the chunks -- the tail of a launch is at most one
  // chunk of one slice.
  const int64_t cap = (int64_t)num_cus * 4;
  int w = std::min(D, kHT);
  while (w > kWave && nchunks * ((D + w - 1) / w) < 4 * cap) w = std::max(kWave, (w / 2) / kWave * kWave);
  const int slices = (D + w - 1) / w;
  int64_t bx = std::max<int64_t>(1, cap / slices);
  bx = std::min<int64_t>(bx, nchunks);
  const int64_t per = (nchunks + bx - 1) / bx;  // chunks per workgroup, balanced
  bx = (nchunks + per - 1) / per;
  // XCD-aware: workgroups are dealt round-robin to the 8 XCDs by linear id bx + by * gridDim.x,
  // so with gridDim.x a multiple of 8 the slices of one chunk run on the same XCD at the same
  // time and share its L2 (the chunk is fetched from HBM once, not once per slice)
  if (slices > 1 && bx >= 8) bx = std::min<int64_t>((bx + 7) / 8 * 8, std::max<int64_t>(8, cap / slices / 8 * 8));
  hipLaunchKernelGGL((k_score<P>), dim3((unsigned)bx, (unsigned)slices), dim3(kScBS), 0, s,
                     src.x, src.y, src.z, (int)src.n, hyps, D, w, cthr, counts);
}

template <int TH>
static void launch_score_bf16(PointsView src, const HypRec* hyps, int D, float cthr,
                              int32_t* counts, int num_cus, hipStream_t s) {
  constexpr int kGroup = 32 * TH;
  const int Dp = (D + kGroup - 1) / kGroup * kGroup;  // hyps[D..Dp): bad planes (count nothing)
  if (Dp > kMaxHypPerLaunch) return;
  uint4* bcol = reinterpret_cast<uint4*>(reinterpret_cast<float*>(
      reinterpret_cast<float4*>(const_cast<HypRec*>(hyps) + kMaxHypPerLaunch) + kMaxHypPerLaunch) +
      kMaxHypPerLaunch);
  float* band = reinterpret_cast<float*>(bcol + 4 * kMaxHypPerLaunch);
  hipLaunchKernelGGL(k_prep_bf16, dim3((Dp + 255) / 256), dim3(256), 0, s, hyps, D, Dp, bcol, band);
  const int ngroups = Dp / kGroup;
  // ~8 resident waves per SIMD; partitions a multiple of 32 points
  const int64_t want_waves = (int64_t)num_cus * 4 * 8;
  int64_t nparts = std::max<int64_t>(1, (want_waves + ngroups - 1) / ngroups);
  int64_t part = (src.n + nparts - 1) / nparts;
  part = std::max<int64_t>(32, (part + 31) / 32 * 32);
  nparts = (src.n + part - 1) / part;
  const int64_t waves = nparts * ngroups;
  const unsigned grid = (unsigned)((waves + (kBfBS / kWave) - 1) / (kBfBS / kWave));
  hipLaunchKernelGGL((k_score_bf16<TH>), dim3(grid), dim3(kBfBS), 0, s, src.x, src.y, src.z,
                     (int)src.n, hyps, bcol, band, D, ngroups, (int)part, cthr, counts);
}

void launch_prep_bf16(const HypRec* hyps, int D, const uint4** bcol_out, const float** band_out,
                      hipStream_t s) {
  const int Dp = (D + 31) / 32 * 32;
  uint4* bcol = reinterpret_cast<uint4*>(reinterpret_cast<float*>(
      reinterpret_cast<float4*>(const_cast<HypRec*>(hyps) + kMaxHypPerLaunch) + kMaxHypPerLaunch) +
      kMaxHypPerLaunch);
  float* band = reinterpret_cast<float*>(bcol + 4 * kMaxHypPerLaunch);
  if (D > 0) hipLaunchKernelGGL(k_prep_bf16, dim3((Dp + 255) / 256), dim3(256), 0, s, hyps, D, Dp, bcol, band);
  *bcol_out = bcol;
  *band_out = band;
}

void launch_score(PointsView src, const HypRec* hyps, int D, float cthr, int32_t* counts,
                  int kernel, int num_cus, hipStream_t s) {
  if (D <= 0 || src.n <= 0) return;
  switch (kernel) {
    case kScoreExact: launch_score_t<4>(src, hyps, D, cthr, counts, num_cus, s); break;
    case kScoreBf16: launch_score_bf16<8>(src, hyps, D, cthr, counts, num_cus, s); break;
    default: break;
  }
}

int moments_blocks(int64_t n) {
  // (<= 512: the last workgroup reduces 25 x nb block sums)
  int64_t b = (n + kMoBS * 8 - 1) / (kMoBS * 8);
  if (b < 1) b = 1;
  if (b > 512) b = 512;
  return (int)b;
}

void launch_refit_moments(const int64_t* moments, int qexp, const float4* cin, int optimize,
                          float4* cout, hipStream_t s) {
  hipLaunchKernelGGL(k_refit_moments, dim3(1), dim3(kWave), 0, s, moments, qexp, cin, optimize, cout);
}

// done: a device counter that is zero between launches (the last workgroup resets it)
void launch_moments_refit(PointsView src, const float4* coef, const ModelTest& mt, int qexp,
                          int64_t* partials, unsigned* done, int nblocks, int64_t* out,
                          float4* cout, hipStream_t s) {
  const double qs = pow2d(kFastBits - qexp);
  if (mt.normal_plane)
    hipLaunchKernelGGL((k_moments<true, 1>), dim3(nblocks), dim3(kMoBS), 0, s, src, coef, mt, qs,
                       partials, done, out, qexp, cout);
  else
    hipLaunchKernelGGL((k_moments<false, 1>), dim3(nblocks), dim3(kMoBS), 0, s, src, coef, mt, qs,
                       partials, done, out, qexp, cout);
}

int moments_sp_blocks(int64_t n) {
  // (512 workgroups measured no faster: the launch is bound by its latency chain and the tail)
  return (int)std::max<int64_t>(1, std::min<int64_t>(256, sp_supers(n)));
}

void launch_moments_sp(PointsView src, const float4* tiles, const float4* supers, float margin,
                       const float4* coef, const ModelTest& mt, int qexp, int64_t* partials,
                       unsigned* done, int nblocks, int64_t* out, float4* cout, hipStream_t s) {
  const double qs = pow2d(kFastBits - qexp);
  // (NORMAL_PLANE: the model test reads the copy's normals, src.nrm; margin = the NP prune margin)
  auto* k = mt.normal_plane ? (cout ? k_moments_sp<1, true> : k_moments_sp<0, true>)
                            : (cout ? k_moments_sp<1, false> : k_moments_sp<0, false>);
  hipLaunchKernelGGL(k, dim3(nblocks), dim3(kMoBS), 0, s, src, tiles, supers, margin, coef, mt,
                     qs, partials, done, out, qexp, cout);
}

void launch_moments(PointsView src, const float4* coef, const ModelTest& mt, int qexp,
                    int64_t* partials, unsigned* done, int nblocks, int64_t* out, hipStream_t s) {
  const double qs = pow2d(kFastBits - qexp);
  if (mt.normal_plane)
    hipLaunchKernelGGL((k_moments<true, 0>), dim3(nblocks), dim3(kMoBS), 0, s, src, coef, mt, qs,
                       partials, done, out, qexp, nullptr);
  else
    hipLaunchKernelGGL((k_moments<false, 0>), dim3(nblocks), dim3(kMoBS), 0, s, src, coef, mt, qs,
                       partials, done, out, qexp, nullptr);
}

void launch_pick_p1(const PickArgs& a, hipStream_t s) {
  hipLaunchKernelGGL(k_pick_p1, dim3(1), dim3(kPickBS), 0, s, a);
}

void launch_publish(const PubArgs& a, hipStream_t s) {
  hipLaunchKernelGGL(k_publish, dim3(1), dim3(256), 0, s, a);
}

int select_tiles(int64_t n) { return (int)((n + kSelTile - 1) / kSelTile); }

// selectWithinDistance in two halves: head = per-tile counts + scan (totals[0..1] final),
// tail = ordered scatter of the inlier ids / survivors
void launch_select_head(PointsView src, const float4* coef, const ModelTest& mt, int32_t* tile_in,
                        int32_t* tile_off_in, int32_t* tile_off_out, int32_t* totals,
                        hipStream_t s) {
  const int nt = select_tiles(src.n);
  if (nt == 0) {
    (void)hipMemsetAsync(totals, 0, 2 * sizeof(int32_t), s);
    return;
  }
  if (mt.normal_plane)
    hipLaunchKernelGGL(k_select_count<true>, dim3(nt), dim3(kSelBS), 0, s, src, coef, mt, tile_in);
  else
    hipLaunchKernelGGL(k_select_count<false>, dim3(nt), dim3(kSelBS), 0, s, src, coef, mt, tile_in);
  hipLaunchKernelGGL(k_scan_tiles, dim3(1), dim3(kScanBS), 0, s, tile_in, nt, src.n, tile_off_in,
                     tile_off_out, totals);
}

void launch_select_tail(PointsView src, const float4* coef, const ModelTest& mt,
                        const int32_t* tile_off_in, const int32_t* tile_off_out, int32_t* inl_gid,
                        float* inl_xyz, const PointsOut* dst, hipStream_t s) {
  const int nt = select_tiles(src.n);
  if (nt == 0) return;
  PointsOut d = dst ? *dst : PointsOut{nullptr, nullptr, nullptr, nullptr, nullptr};
  if (mt.normal_plane)
    hipLaunchKernelGGL(k_select_scatter<true>, dim3(nt), dim3(kSelBS), 0, s, src, coef, mt,
                       tile_off_in, tile_off_out, inl_gid, inl_xyz, d, dst ? 1 : 0);
  else
    hipLaunchKernelGGL(k_select_scatter<false>, dim3(nt), dim3(kSelBS), 0, s, src, coef, mt,
                       tile_off_in, tile_off_out, inl_gid, inl_xyz, d, dst ? 1 : 0);
}

void launch_select(PointsView src, const float4* coef, const ModelTest& mt, int32_t* tile_in,
                   int32_t* tile_off_in, int32_t* tile_off_out, int32_t* totals, int32_t* inl_gid,
                   float* inl_xyz, const PointsOut* dst, hipStream_t s) {
  launch_select_head(src, coef, mt, tile_in, tile_off_in, tile_off_out, totals, s);
  launch_select_tail(src, coef, mt, tile_off_in, tile_off_out, inl_gid, inl_xyz, dst, s);
}

void launch_score_np(PointsView src, const HypRec* hyps, int D, const ModelTest& mt,
                     int32_t* counts, int num_cus, hipStream_t s) {
  if (D <= 0 || src.n <= 0) return;
  const int Dp = (D + kWave - 1) / kWave * kWave;
  auto go = [&](auto kern, int P, int per_cu) {
    const int64_t chunks = (src.n + (int64_t)kNpBS * P - 1) / ((int64_t)kNpBS * P);
    const int64_t cap = (int64_t)num_cus * per_cu;
    const unsigned grid = (unsigned)std::max<int64_t>(1, std::min<int64_t>(chunks, cap));
    hipLaunchKernelGGL(kern, dim3(grid), dim3(kNpBS), 0, s, src, hyps, Dp, mt.lambda, mt.thr,
                       counts);
  };
  // LDS per block: 16 KB counts + 32 B x HT planes + 4 KB x P point normals + 6 KB queue.
  // Measured on C5 (10M points, 4096 planes/launch; round 1, tools/bench_c5.py):
  // <P=2, HT=256> x4/CU 2.55 T tests/s > <2,128> 2.50 > <2,64> 2.43 > <4,256> x3 2.40 >
  // <1,256> 2.21 > <4,512>, <8,256>, <4,1024> x2 1.69-1.73 (occupancy-bound: 2 waves/SIMD)
  go(k_score_np<2, 256>, 2, 4);
}

void launch_pack_point_normals(const float* raw, int64_t stride_f, int curv_off, PointsView src,
                               int32_t id_base, float4* out, hipStream_t s, bool normalize) {
  if (src.n <= 0) return;
  hipLaunchKernelGGL(k_pack_point_normals, dim3(cdiv(src.n, 256)), dim3(256), 0, s, raw, stride_f,
                     curv_off, src, id_base, out, normalize ? 1 : 0);
}

void launch_upload_gather(const float* raw, int64_t stride_f, const int32_t* idx, int64_t n,
                          int32_t id_base, PointsOut out, hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_upload_gather, dim3(cdiv(n, 256)), dim3(256), 0, s, raw, stride_f, idx, n,
                     id_base, out);
}

void launch_absmax(PointsView src, uint32_t* out4, hipStream_t s) {
  (void)hipMemsetAsync(out4, 0, 4 * sizeof(uint32_t), s);
  if (src.n <= 0) return;
  unsigned g = cdiv(src.n, 256);
  if (g > 1024) g = 1024;
  hipLaunchKernelGGL(k_absmax, dim3(g), dim3(256), 0, s, src, out4);
}

}  // namespace dlg
