// fsum.hip -- PCL's float refit on the device (gfx950): the nine sequential float sums of
// computeMeanAndCovarianceMatrix, bit-exact, in parallel (algorithm and proof: fsum.hpp), then
// the float eigen33 of optimizeModelCoefficients.
//
// Kernels (stream order; the inlier count lives on the device, so every grid is fixed and the
// kernels loop over the work the count implies):
//   k_fs_prep   units of 4096 inliers (64 chunks): per-chunk double sums of the nine terms, one
//               thread per chunk (all nine chains in registers), per-unit sums; the last
//               workgroup scans the units (double prefixes, optionally from a rank's base)
//   k_fs_inc    units again, thread (chunk, chain group): each chunk run once from its first
//               guess fl(double prefix) -> its float increment o - g (double); per-unit sums,
//               the last workgroup scans them.  The prefix of the increments is the refined
//               guess: exact wherever every earlier chunk's increment is independent of its
//               start (the common case), so the records below sit at (or a few quanta from)
//               the value the walk brings, even where the double prefix drifts by thousands of
//               quanta from the float chain (sums hovering near zero)
//   k_fs_l1     (unit, chain) items: the chain's terms staged in LDS, the refined guesses, then
//               lane (chunk, member) runs the chunk from g_k + member q(g_k): the chunk
//               records, written as coalesced 16-byte rows
//   k_fs_walk   one wave per chain: the speculative 64-wide walk over the chunk records from
//               the chain's start value (+0, or the previous rank's end value); a chunk the
//               lemma does not cover is rerun from its exact start.  The last chain to finish
//               runs the refit tail (fs_refit_tail) when the caller asks for it.
// The walk is wave-uniform: every lane holds one record, the carried value is uniform.
#include "kernels.hpp"
#include "dev_common.hpp"
#include "fsum.hpp"
#include "comm.hpp"

#include <hip/hip_ext.h>

#include <atomic>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <stdexcept>
#include <string>
#include <vector>

#define HIPCHK_FS(expr)                                                                       \
  do {                                                                                        \
    const hipError_t e_ = (expr);                                                             \
    if (e_ != hipSuccess)                                                                     \
      throw std::runtime_error(std::string(#expr) + " -> " + hipGetErrorString(e_));          \
  } while (0)

namespace dlg {
namespace {

constexpr int kFsUC = 64;                     // chunks per unit
constexpr int kFsUnit = kFsChunk * kFsUC;     // 4096 inliers per unit
constexpr int kFsPad = kFsChunk + 1;          // LDS row stride of a chunk (spreads the banks)

struct FsDev {
  const float* px;
  const float* py;
  const float* pz;
  int stride;
  const int32_t* n_dev;
  FsBuffers b;
  uint32_t gen;  // this launch's stamp (window transfer tables of older launches are ignored)
};

__device__ __forceinline__ FsNode* fs_rec(const FsBuffers& b, int c, int64_t k) {
  return b.rec + (int64_t)c * b.cap + k;
}

template <int C>
__device__ __forceinline__ void fs_acc9(double (&a)[kFsChains], float x, float y, float z) {
  a[C] += (double)fs_term(C, x, y, z);
  if constexpr (C + 1 < kFsChains) fs_acc9<C + 1>(a, x, y, z);
}

// inclusive prefix sum of a double over the wave, by DPP row shifts and row broadcasts (no LDS
// instruction: ds_bpermute shuffles cost ~100 clocks each on this path)
template <int kCtrl, int kRowMask>
__device__ __forceinline__ double dpp_dbl(double v) {
  const uint64_t b = (uint64_t)__double_as_longlong(v);
  const uint32_t lo = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(uint32_t)b, kCtrl, kRowMask,
                                                            0xF, false);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(uint32_t)(b >> 32), kCtrl,
                                                            kRowMask, 0xF, false);
  return __longlong_as_double((int64_t)(((uint64_t)hi << 32) | lo));
}

__device__ __forceinline__ double wave_incl_scan(double v, int) {
  v += dpp_dbl<0x111, 0xF>(v);  // row_shr:1 (lanes shifted in from outside the row read 0)
  v += dpp_dbl<0x112, 0xF>(v);  // row_shr:2
  v += dpp_dbl<0x114, 0xF>(v);  // row_shr:4
  v += dpp_dbl<0x118, 0xF>(v);  // row_shr:8
  v += dpp_dbl<0x142, 0xA>(v);  // row_bcast:15 into rows 1 and 3
  v += dpp_dbl<0x143, 0xC>(v);  // row_bcast:31 into rows 2 and 3
  return v;
}

__device__ __forceinline__ double rld(double v, int l) {
  const uint64_t u = (uint64_t)__double_as_longlong(v);
  return __longlong_as_double((int64_t)(
      (uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)u, l) |
      ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(u >> 32), l) << 32)));
}

// the last workgroup of a unit pass scans the per-unit sums usum into the exclusive prefixes
// upre (from base9, or 0); ticket = the pass's ticket word
__device__ void fs_scan_body(const FsDev& d, int64_t U, const double* base9, double* blk,
                             double* tot_out);

__device__ void fs_scan_units(const FsDev& d, int64_t U, const double* base9, unsigned* ticket,
                              double* blk, double* tot_out = nullptr) {
  const int t = threadIdx.x;
  __builtin_amdgcn_s_waitcnt(0);
  __shared__ unsigned s_ticket;
  __syncthreads();
  if (t == 0)
    s_ticket = __hip_atomic_fetch_add(ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __syncthreads();
  if (s_ticket != gridDim.x - 1) return;
  if (t == 0) *ticket = 0u;
  fs_scan_body(d, U, base9, blk, tot_out);
}

// upre = exclusive prefixes of usum from base9 (or 0); tot_out non-null: only the totals (and
// the count n in tot_out[9]) are written.  Wave w scans chains w, w + 4, w + 8, 64 units per
// DPP wave scan (the prefixes are guesses: any fixed summation order serves).
__device__ void fs_scan_body(const FsDev& d, int64_t U, const double* base9, double*,
                             double* tot_out) {
  const int t = threadIdx.x, w = t >> 6, l = t & 63;
#pragma unroll
  for (int m = 0; m < 3; ++m) {
    const int c = w + 4 * m;
    if (c >= kFsChains) break;  // (wave-uniform)
    double run = base9 ? base9[c] : 0.0;
    for (int64_t ub = 0; ub < U; ub += kWave) {
      const int64_t uu = ub + l;
      const double v = uu < U ? __longlong_as_double(__hip_atomic_load(
                                    reinterpret_cast<const int64_t*>(d.b.usum) + uu * kFsChains + c,
                                    __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))
                              : 0.0;
      const double inc = wave_incl_scan(v, l);
      if (!tot_out && uu < U) d.b.upre[uu * kFsChains + c] = run + (inc - v);
      run += rld(inc, kWave - 1);
    }
    if (tot_out && l == 0) tot_out[c] = run;
  }
  if (tot_out && t == 0) tot_out[kFsChains] = (double)*d.n_dev;
}

// several ranks: this rank's base = the double totals of the ranks before it (list order), the
// global inlier count; then the unit scan from that base.  One workgroup.
// shift (the rebase, several ranks): every chain's base moved by g2 - (the first walk's start),
// so that the refined guesses follow the chain from the propagated guess g2
__global__ __launch_bounds__(256) void k_fs_base(FsDev d, const double* __restrict__ gath, int rank,
                                                 int world, double* __restrict__ base9,
                                                 int64_t* __restrict__ n_global,
                                                 const float* __restrict__ gath2,
                                                 const float* __restrict__ g2) {
  __shared__ double blk[64 * kFsChains];
  __shared__ double sb[kFsChains];
  const int t = threadIdx.x;
  if (t < kFsChains) {
    double b = 0.0;
    for (int r = 0; r < rank; ++r) b += gath[r * (kFsChains + 1) + t];
    if (g2) b += (double)g2[t] - (double)gath2[(rank * 2 + 1) * kFsChains + t];
    sb[t] = b;
    base9[t] = b;
  }
  if (t == kFsChains) {
    int64_t ng = 0;
    for (int r = 0; r < world; ++r) ng += (int64_t)gath[r * (kFsChains + 1) + kFsChains];
    *n_global = ng;
  }
  __syncthreads();
  const int64_t n = *d.n_dev;
  fs_scan_body(d, (n + kFsUnit - 1) / kFsUnit, sb, blk, nullptr);
}

// several ranks: the refit tail on the broadcast global sums (identical on every rank)
__global__ void k_fs_tail(const float* __restrict__ sums9, const int64_t* __restrict__ n_global,
                          const float4* __restrict__ cin, float4* __restrict__ cout,
                          int32_t* __restrict__ res) {
  float a9[kFsChains];
  for (int k = 0; k < kFsChains; ++k) a9[k] = sums9[k];
  const int64_t n = *n_global;
  const float4 ci = *cin;
  const float cv[4] = {ci.x, ci.y, ci.z, ci.w};
  float co[4];
  bool unc = false;
  fs_refit_tail(a9, n, cv, co, &unc);
  *cout = make_float4(co[0], co[1], co[2], co[3]);
  res[0] = unc ? 1 : 0;
  res[1] = (int32_t)n;
  for (int k = 0; k < kFsChains; ++k) res[2 + k] = __float_as_int(a9[k]);
}

// ---- k_fs_prep --------------------------------------------------------------------------------
// thread (chunk k, quarter h): the nine double sums of its 16 terms; wave w then adds the four
// quarters of chains w, w + 4, w + 8 per chunk and reduces them over the unit (DPP)
constexpr int kFpBS = 256;
__global__ __launch_bounds__(kFpBS) void k_fs_prep(FsDev d, const double* __restrict__ base9,
                                                   double* __restrict__ tot_out) {
  __shared__ float sx[kFsUC * kFsPad], sy[kFsUC * kFsPad], sz[kFsUC * kFsPad];
  __shared__ double sq[4 * kFsChains * kFsUC];  // [quarter][chain][chunk]
  const int64_t n = *d.n_dev;
  const int64_t U = (n + kFsUnit - 1) / kFsUnit;
  const int t = threadIdx.x, k = t & 63, h = t >> 6;
  for (int64_t u = blockIdx.x; u < U; u += gridDim.x) {
    const int64_t e0 = u * kFsUnit;
    const int cnt = (int)(n - e0 < kFsUnit ? n - e0 : kFsUnit);
    const int nch = (cnt + kFsChunk - 1) / kFsChunk;
    __syncthreads();
    for (int j = t; j < cnt; j += kFpBS) {
      const int64_t e = (e0 + j) * d.stride;
      const int li = (j >> 6) * kFsPad + (j & 63);
      sx[li] = d.px[e]; sy[li] = d.py[e]; sz[li] = d.pz[e];
    }
    __syncthreads();
    {
      double a[kFsChains] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
      const int j0 = k * kFsChunk + h * (kFsChunk / 4);
      int len = cnt - j0 < kFsChunk / 4 ? cnt - j0 : kFsChunk / 4;
      if (len < 0) len = 0;
      for (int i = 0; i < len; ++i) {
        const int li = k * kFsPad + h * (kFsChunk / 4) + i;
        fs_acc9<0>(a, sx[li], sy[li], sz[li]);
      }
#pragma unroll
      for (int c = 0; c < kFsChains; ++c) sq[(h * kFsChains + c) * kFsUC + k] = a[c];
    }
    __syncthreads();
#pragma unroll
    for (int m = 0; m < 3; ++m) {
      const int c = h + 4 * m;
      if (c >= kFsChains) break;  // (wave-uniform)
      const double v = ((sq[c * kFsUC + k] + sq[(kFsChains + c) * kFsUC + k]) +
                        sq[(2 * kFsChains + c) * kFsUC + k]) +
                       sq[(3 * kFsChains + c) * kFsUC + k];
      if (k < nch) d.b.csum[(u * kFsUC + k) * kFsChains + c] = v;
      const double s = wave_incl_scan(k < nch ? v : 0.0, k);
      if (k == kWave - 1)
        __hip_atomic_store(reinterpret_cast<int64_t*>(d.b.usum) + u * kFsChains + c,
                           __double_as_longlong(s), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  // the last workgroup scans the unit sums (agent-scope stores acknowledged before the ticket,
  // read back with agent-scope loads: k_moments' pattern); with tot_out (several ranks) it only
  // totals them -- the scan waits for the other ranks' totals (k_fs_base)
  fs_scan_units(d, U, base9, d.b.ticket, nullptr, tot_out);
}

// ---- k_fs_inc ---------------------------------------------------------------------------------
// in place: csum (chunk double sums) -> the chunks' float increments, usum -> their unit sums,
// upre (double prefixes) -> the increments' prefixes.  Each unit is read and rewritten by one
// workgroup; the scan runs after every workgroup has passed its ticket.
// the chunk's float runs of chains CG, CG + 4 (and CG + 8 for CG = 0) from v[], interleaved
template <int CG>
__device__ __forceinline__ void fs_inc_run(const float* sx, const float* sy, const float* sz,
                                           int li0, int len, float (&v)[3]) {
#pragma unroll 4
  for (int j = 0; j < len; ++j) {
    const float x = sx[li0 + j], y = sy[li0 + j], z = sz[li0 + j];
    v[0] = v[0] + fs_term(CG, x, y, z);
    v[1] = v[1] + fs_term(CG + 4, x, y, z);
    if constexpr (CG + 8 < kFsChains) v[2] = v[2] + fs_term(CG + 8, x, y, z);
  }
}

constexpr int kFiBS = 256;  // 64 chunks x 4 chain groups (chains g, g + 4, g + 8)
__global__ __launch_bounds__(kFiBS) void k_fs_inc(FsDev d, const double* __restrict__ base9) {
  __shared__ float sx[kFsUC * kFsPad], sy[kFsUC * kFsPad], sz[kFsUC * kFsPad];
  __shared__ double scs[kFsUC * kFsChains];
  __shared__ double spre[kFsChains];
  const int64_t n = *d.n_dev;
  const int64_t U = (n + kFsUnit - 1) / kFsUnit;
  const int t = threadIdx.x, k = t & 63, cg = t >> 6;
  for (int64_t u = blockIdx.x; u < U; u += gridDim.x) {
    const int64_t e0 = u * kFsUnit;
    const int cnt = (int)(n - e0 < kFsUnit ? n - e0 : kFsUnit);
    const int nch = (cnt + kFsChunk - 1) / kFsChunk;
    __syncthreads();
    for (int j = t; j < cnt; j += kFiBS) {
      const int64_t e = (e0 + j) * d.stride;
      const int li = (j >> 6) * kFsPad + (j & 63);
      sx[li] = d.px[e]; sy[li] = d.py[e]; sz[li] = d.pz[e];
    }
    for (int p = t; p < nch * kFsChains; p += kFiBS)
      scs[p] = d.b.csum[u * kFsUC * kFsChains + p];
    if (t < kFsChains) spre[t] = d.b.upre[u * kFsChains + t];
    __syncthreads();
    // first guesses at chunk k: the unit's double prefix + the chunks before it (DPP scans of
    // the sums shifted by one chunk), chains cg, cg + 4, cg + 8
    float g[3];
#pragma unroll
    for (int m = 0; m < 3; ++m) {
      const int c = cg + 4 * m < kFsChains ? cg + 4 * m : cg;
      const double pv = k > 0 && k - 1 < nch ? scs[(k - 1) * kFsChains + c] : 0.0;
      g[m] = (float)(spre[c] + wave_incl_scan(pv, k));
    }
    float v[3] = {g[0], g[1], g[2]};
    if (k < nch) {
      const int len = cnt - k * kFsChunk < kFsChunk ? cnt - k * kFsChunk : kFsChunk;
      switch (cg) {  // (wave-uniform: the chains' terms resolved outside the loop)
        case 0: fs_inc_run<0>(sx, sy, sz, k * kFsPad, len, v); break;
        case 1: fs_inc_run<1>(sx, sy, sz, k * kFsPad, len, v); break;
        case 2: fs_inc_run<2>(sx, sy, sz, k * kFsPad, len, v); break;
        default: fs_inc_run<3>(sx, sy, sz, k * kFsPad, len, v); break;
      }
    }
#pragma unroll
    for (int m = 0; m < 3; ++m) {
      const int c = cg + 4 * m;
      if (c >= kFsChains) break;  // (wave-uniform)
      const double inc = k < nch ? (double)v[m] - (double)g[m] : 0.0;
      if (k < nch) d.b.csum[(u * kFsUC + k) * kFsChains + c] = inc;
      const double s = wave_incl_scan(inc, k);
      if (k == kWave - 1)
        __hip_atomic_store(reinterpret_cast<int64_t*>(d.b.usum) + u * kFsChains + c,
                           __double_as_longlong(s), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  fs_scan_units(d, U, base9, d.b.ticket, nullptr);
}

__device__ __forceinline__ float rdl(float v, int l) {
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), l));
}

typedef float f32x4 __attribute__((ext_vector_type(4)));

// a record unpacked for the walk, with its per-record constants (q = quantum of g, iq = 1/q, gq =
// g / q, d0 = member 0's increment, P = the in-unit prefix of the member-0 increments, mu3 = the
// fast path's margin)
struct FsWalkRec {
  float g, mu3;
  float o0, o1, o2, o3, m0, m1, m2, m3, q0, q1, q2, q3;
  double d0, P;
  // (derived on use: fewer live registers)
  __device__ double q() const { return (double)fs_quantum(g); }
  __device__ double iq() const { return fs_inv_quantum(g); }
  __device__ double gd() const { return (double)g; }
};

__device__ __forceinline__ FsWalkRec fs_walk_rec(const f32x4& r0, const f32x4& r1, const f32x4& r2,
                                                 const f32x4& r3) {
  FsWalkRec w;
  w.g = r0.x;
  w.mu3 = r0.w;
  w.o0 = r1.x; w.o1 = r1.y; w.o2 = r1.z; w.o3 = r1.w;
  w.m0 = r2.x; w.m1 = r2.y; w.m2 = r2.z; w.m3 = r2.w;
  w.q0 = r3.x; w.q1 = r3.y; w.q2 = r3.z; w.q3 = r3.w;
  w.d0 = w.q0 >= 0.0f ? (double)w.o0 - (double)w.g : 0.0;
  w.P = __longlong_as_double((int64_t)(((uint64_t)__float_as_uint(r0.z) << 32) |
                                       __float_as_uint(r0.y)));
  return w;
}

// inclusive prefix sum of an int over the wave (DPP, as wave_incl_scan)
template <int kCtrl, int kRowMask>
__device__ __forceinline__ int dpp_i32(int v) {
  return __builtin_amdgcn_update_dpp(0, v, kCtrl, kRowMask, 0xF, false);
}
__device__ __forceinline__ int wave_incl_scan_i32(int v) {
  v += dpp_i32<0x111, 0xF>(v);
  v += dpp_i32<0x112, 0xF>(v);
  v += dpp_i32<0x114, 0xF>(v);
  v += dpp_i32<0x118, 0xF>(v);
  v += dpp_i32<0x142, 0xA>(v);
  v += dpp_i32<0x143, 0xC>(v);
  return v;
}

// float minimum over the wave by DPP (lane 63 ends with it; no LDS instruction)
template <int kCtrl, int kRowMask>
__device__ __forceinline__ float dpp_min_step(float v) {
  const float o = __int_as_float(__builtin_amdgcn_update_dpp(__float_as_int(v), __float_as_int(v),
                                                              kCtrl, kRowMask, 0xF, false));
  return fminf(v, o);
}
__device__ __forceinline__ float wave_min(float v) {
  v = dpp_min_step<0x111, 0xF>(v);
  v = dpp_min_step<0x112, 0xF>(v);
  v = dpp_min_step<0x114, 0xF>(v);
  v = dpp_min_step<0x118, 0xF>(v);
  v = dpp_min_step<0x142, 0xA>(v);
  v = dpp_min_step<0x143, 0xC>(v);
  return rdl(v, kWave - 1);
}

// the integer-stepping table of a window's records (fs_seq_window), one record per lane: Q =
// the window's smallest quantum of a nonzero guess or usable output, per record the member
// increments E_i = (o_i - i q(g_k) - g_{k+1}) / Q (0 past the last record; F_i = E_0 for a
// record that takes only its exact start), margins floor(mu_i / Q) (saturated, -1: none), the
// shift s = log2(q(g_k) / Q) and flags.  Computed once per window in k_fs_l1, in parallel.
__device__ __forceinline__ void fs_seq_prep(const FsWalkRec wr, int cnt, int lane, uint4* sq0,
                                            uint4* sq1, uint4* sq2) {
  const bool act = lane < cnt;
  const bool u0 = wr.q0 >= 0.0f, u1 = wr.q1 >= 0.0f, u2 = wr.q2 >= 0.0f, u3 = wr.q3 >= 0.0f;
  float qv = INFINITY;
  auto qmin = [&](float v, bool use) {
    if (use && v != 0.0f) qv = fminf(qv, fs_quantum(v));  // (NaN quanta of non-finite values: ignored)
  };
  if (act) {
    qmin(wr.g, true);
    qmin(wr.o0, u0); qmin(wr.o1, u1); qmin(wr.o2, u2); qmin(wr.o3, u3);
  }
  float Qf = wave_min(qv);
  if (!(Qf < INFINITY)) Qf = 1.40129846e-45f;  // (every value zero)
  const double iQ = 1.0 / (double)Qf;  // (exact: powers of two)
  const float qk = fs_quantum(wr.g);
  // s = log2(q(g_k) / Q); a lane whose quantum is below Q (a zero guess) or not finite only takes
  // its exact start (L = 0, member 0)
  const bool gfin = fabsf(wr.g) <= 3.40282347e+38f;
  // (log2 of a power of two from its bits: exponent field, or the bit position when subnormal)
  auto lg2 = [](float p) {
    const uint32_t b = __float_as_uint(p), e = (b >> 23) & 0xFFu;
    return e ? (int)e - 127 : (int)__builtin_ctz(b | 0x80000000u) - 149;
  };
  int sh = lg2(qk) - lg2(Qf);
  const bool exact_only = !gfin || !(qk >= Qf);
  if (exact_only || sh < 0) sh = 0;
  if (sh > 30) sh = 30;
  // E_k[i] (0 past the window's last lane: its end value is taken from the member directly)
  const float gn = __int_as_float(
      __builtin_amdgcn_update_dpp(0, __float_as_int(wr.g), 0x130, 0xF, 0xF, false));  // g_{k+1}
  const bool lastl = lane == cnt - 1;
  auto emem = [&](float o, int i, bool u, bool* ok) {
    if (lastl) {
      *ok = u;
      return 0;
    }
    // (o - g_{k+1}, both multiples of Q, is exact below 2^52 Q; the bound keeps it exact)
    const double dd = (double)o - (double)gn;
    const double e = (dd - (double)i * (double)qk) * iQ;
    *ok = u && fabs(dd * iQ) < 1099511627776.0 && fabs(e) < 1048576.0 && e == floor(e);
    return *ok ? (int)e : 0;
  };
  bool k0, k1, k2, k3;
  const int E0 = emem(wr.o0, 0, u0, &k0), E1 = emem(wr.o1, 1, u1, &k1),
            E2 = emem(wr.o2, 2, u2, &k2), E3 = emem(wr.o3, 3, u3, &k3);
  // (a lane taking only its exact start steps with E0 whatever the lead's bits)
  const int F1 = exact_only ? E0 : E1, F2 = exact_only ? E0 : E2, F3 = exact_only ? E0 : E3;
  auto marg = [&](float mu) {  // floor(mu / Q), saturated; -1: no shift tolerated
    const double m = floor((double)mu * iQ);
    return m >= 0.0 ? (int64_t)fmin(m, 1073741824.0) : (int64_t)-1;
  };
  const int64_t M0 = marg(wr.m0), M1 = marg(wr.m1), M2 = marg(wr.m2), M3 = marg(wr.m3);
  // a translation record: fast (every member's increment the same) with all four E usable
  const bool tr = act && wr.mu3 >= 0.0f && !exact_only && k0 && k1 && k2 && k3 && E1 == E0 &&
                  E2 == E0 && E3 == E0;
  const double q2 = 2.0 * (double)qk;
  const bool c0 = (double)wr.q0 <= q2, c1 = (double)wr.q1 <= q2, c2 = (double)wr.q2 <= q2,
             c3 = (double)wr.q3 <= q2;
  *sq0 = make_uint4((uint32_t)E0, (uint32_t)F1, (uint32_t)F2, (uint32_t)F3);
  *sq1 = make_uint4((uint32_t)(int32_t)M0, (uint32_t)(int32_t)M1, (uint32_t)(int32_t)M2,
                    (uint32_t)(int32_t)M3);
  const uint32_t fl = (uint32_t)sh | (uint32_t)exact_only << 8 | (uint32_t)gfin << 9 |
                      (uint32_t)k0 << 10 | (uint32_t)k1 << 11 | (uint32_t)k2 << 12 |
                      (uint32_t)k3 << 13 | (uint32_t)c0 << 14 | (uint32_t)c1 << 15 |
                      (uint32_t)c2 << 16 | (uint32_t)c3 << 17 | (uint32_t)tr << 18;
  *sq2 = make_uint4(fl, __float_as_uint(Qf), 0u, 0u);
}

// Window transfer table (the walk's lookup for a window it would walk record by record): the
// window's records applied to each of the entry leads -kFtLo..kFtW-1-kFtLo, 64 at once (one
// builder item per half of the table), lane = entry
// lead L (entering at t = g_0 + L Q, Q the window's smallest quantum).  Record k is applied as
// fs_seq_window applies it: covered by the lemma (member i = (L_k >> s_k) & 3, the grid, margin
// and quanta conditions) it steps L_{k+1} = L_k + E_k[i]; otherwise the lane reruns the chunk's
// terms (staged in LDS, summed in order) from its exact start g_k + L_k Q and re-expresses the
// result as a lead on g_{k+1}.  A lane whose start or re-expressed lead is not exact is dropped.
// Every lane kept holds the window's exit value -- a literal run or lemma-proven shift of the
// chain from that entry, the value any exact walk carries out of the window -- and its mask bit.
// Chains hovering near zero (many start-dependent records, a few reruns per window) are then
// walked one lookup per window instead of record by record.  The tables are built by the walk
// kernel's own builder workgroups while the walkers run (k_fs_walk): a table is published with
// this launch's stamp in every 8-byte entry; the walker prefetches the tables of the next 16
// windows into LDS when it first needs one of them, reads an entry again from memory when its
// prefetched copy was not there yet, and uses an entry only if it carries the stamp; otherwise
// it walks the window itself -- nobody waits.
constexpr int kFtHalves = 2;                // builder items per window (64 leads each)
constexpr int kFtW = kFtHalves * kWave;      // table width: entry leads -kFtLo .. kFtW - 1 - kFtLo
constexpr int kFtLo = kFtW / 2;
constexpr int kFtGroup = 8;  // windows whose tables the walker prefetches at once
constexpr int kFtLdsWords = kFtGroup * kFtW + kWave;  // (8-byte words: entries, then the quanta)
struct FsTabLds {
  uint4 sq[kWave][3];
  float g[kWave];
  float4 o[kWave];
  float term[kWave];
};
__device__ __forceinline__ void fs_wtab_item(const FsDev& d, int c, int64_t u, int half, int lane,
                                             FsTabLds& L_) {
  const int64_t n = *d.n_dev;
  const int64_t K = fs_chunks(n);
  const int64_t base = u * kWave;
  const int nch = K - base < kWave ? (int)(K - base) : kWave;
  const int cnt = n - u * kFsUnit < kFsUnit ? (int)(n - u * kFsUnit) : kFsUnit;
  const float4 sm = d.b.win[(int64_t)c * d.b.wcap + u];
  if (nch <= 0 || (sm.z >= 0.0f && sm.w == sm.w)) return;  // (fast: the summaries / speculation)
  __builtin_amdgcn_wave_barrier();
  if (lane < nch) {
    const uint4* q = d.b.srec + 3 * ((int64_t)c * d.b.cap + base + lane);
    L_.sq[lane][0] = q[0]; L_.sq[lane][1] = q[1]; L_.sq[lane][2] = q[2];
    const FsNode* r = fs_rec(d.b, c, base + lane);
    L_.g[lane] = r->g;
    L_.o[lane] = make_float4(r->o[0], r->o[1], r->o[2], r->o[3]);
  }
  __builtin_amdgcn_wave_barrier();
  const uint32_t qb = L_.sq[0][2].y;  // the window's Q (every record holds it)
  const double Q = (double)__uint_as_float(qb), iQ = 1.0 / Q;  // (exact: powers of two)
  int64_t L = half * kWave + lane - kFtLo;
  bool ok = true;
  float out = 0.0f;
  for (int k = 0; k < nch; ++k) {
    const uint4 sq0 = L_.sq[k][0], sq1 = L_.sq[k][1], sq2 = L_.sq[k][2];
    const float4 o4 = L_.o[k];
    const uint32_t fl = sq2.x;
    const int sh = (int)(fl & 0xFFu);
    const bool exact_only = (fl >> 8) & 1u, gfin = (fl >> 9) & 1u;
    const bool grid = (L & ((1ll << sh) - 1)) == 0;
    const int i = (int)((L >> sh) & 3);
    const int64_t D = L - ((int64_t)i << sh);
    const bool ki = (fl >> (10 + i)) & 1u, ci = (fl >> (14 + i)) & 1u;
    const int64_t Mi = (int32_t)(i == 0 ? sq1.x : i == 1 ? sq1.y : i == 2 ? sq1.z : sq1.w);
    bool cov = gfin && (L < 1073741824 && L > -1073741824) && grid && ki &&
               (D == 0 || (ci && (D < 0 ? -D : D) <= Mi));
    if (exact_only) cov = gfin && L == 0 && ((fl >> 10) & 1u);
    const bool last = k == nch - 1;
    if (cov) {
      const float oi = i == 0 ? o4.x : i == 1 ? o4.y : i == 2 ? o4.z : o4.w;
      if (last) out = (float)((double)oi + (double)D * Q);  // (exact: the lemma)
      else L += (int32_t)(i == 0 ? sq0.x : i == 1 ? sq0.y : i == 2 ? sq0.z : sq0.w);
    }
    if (ballot(ok && !cov)) {  // the uncovered lanes rerun the chunk from their exact start
      const int len = cnt - k * kFsChunk < kFsChunk ? cnt - k * kFsChunk : kFsChunk;
      {  // the chunk's terms into LDS (one per lane, coalesced)
        const int64_t e = ((base + k) * kFsChunk + (lane < len ? lane : 0)) * d.stride;
        const float tv = fs_term(c, d.px[e], d.py[e], d.pz[e]);
        __builtin_amdgcn_wave_barrier();
        L_.term[lane] = tv;
        __builtin_amdgcn_wave_barrier();
      }
      const double tv = (double)L_.g[k] + (double)L * Q;
      float v = (float)tv;
      bool run = ok && !cov && (double)v == tv && (L < 1073741824 && L > -1073741824);
      if (run) {
        if (len == kFsChunk) {  // (the terms read ahead: one LDS latency, 64 adds)
          float tm[kFsChunk];
#pragma unroll
          for (int j = 0; j < kFsChunk; ++j) tm[j] = L_.term[j];
#pragma unroll
          for (int j = 0; j < kFsChunk; ++j) v = v + tm[j];
        } else {
          for (int j = 0; j < len; ++j) v = v + L_.term[j];
        }
        if (last) {
          out = v;
        } else {  // the exact lead on the next record's guess (TwoSum: it must be exact)
          const double ta = (double)v, gb = -(double)L_.g[k + 1];
          const double sd = ta + gb, bv = sd - ta;
          const double er = (ta - (sd - bv)) + (gb - bv);
          const double Ld = sd * iQ;
          if (er == 0.0 && Ld == floor(Ld) && fabs(Ld) < 1073741824.0) L = (int64_t)Ld;
          else run = false;
        }
      }
      if (!cov && !run) ok = false;
    }
  }
  // every entry and the quantum carry this launch's stamp: each is one 8-byte store, read whole,
  // so a reader needs no ordering -- an entry is valid iff its stamp is this launch's
  const uint64_t ev = (uint64_t)__float_as_uint(out) | ((uint64_t)(ok ? d.gen : 0u) << 32);
  __hip_atomic_store(reinterpret_cast<uint64_t*>(d.b.wtab + ((int64_t)c * d.b.wcap + u) * kFtW +
                                                  half * kWave + lane),
                     ev, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (lane == 0 && half == 0)
    __hip_atomic_store(reinterpret_cast<uint64_t*>(d.b.wq + (int64_t)c * d.b.wcap + u),
                       (uint64_t)qb | ((uint64_t)d.gen << 32), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
}

// ---- k_fs_l1 ----------------------------------------------------------------------------------
constexpr int kFlBS = kFsUC * kFsFan;  // 64 chunks x 4 members
__global__ __launch_bounds__(kFlBS) void k_fs_l1(FsDev d) {
  __shared__ float sp[kFsUC * kFsPad];
  __shared__ float4 sn[kFsUC * 4];  // the unit's records, 4 rows of 16 bytes each
  __shared__ float sg[kFsUC];
  const int64_t n = *d.n_dev;
  const int64_t U = (n + kFsUnit - 1) / kFsUnit;
  const int t = threadIdx.x;
  for (int64_t it = blockIdx.x; it < U * kFsChains; it += gridDim.x) {
    const int64_t u = it / kFsChains;
    const int c = (int)(it % kFsChains);
    const int64_t e0 = u * kFsUnit;
    const int cnt = (int)(n - e0 < kFsUnit ? n - e0 : kFsUnit);
    const int nch = (cnt + kFsChunk - 1) / kFsChunk;
    __syncthreads();
    for (int j = t; j < cnt; j += kFlBS) {
      const int64_t e = (e0 + j) * d.stride;
      sp[(j >> 6) * kFsPad + (j & 63)] = fs_term(c, d.px[e], d.py[e], d.pz[e]);
    }
    if (t < kWave) {
      // the guess at chunk t: fl(prefix of the increments), unit prefix + chunks before it
      const double pv = t > 0 && t - 1 < nch ? d.b.csum[(u * kFsUC + t - 1) * kFsChains + c] : 0.0;
      const double pre = d.b.upre[u * kFsChains + c] + wave_incl_scan(pv, t);
      if (t < nch) sg[t] = (float)pre;
    }
    __syncthreads();
    {  // lane (chunk k, member i) runs the chunk from g_k + i q(g_k)
      const int k = t >> 2, i = t & 3;
      if (k < nch) {
        const float g = sg[k];
        float a;
        const bool ok = fs_member_start(g, i, &a);
        const int len = cnt - k * kFsChunk < kFsChunk ? cnt - k * kFsChunk : kFsChunk;
        FsState st = fs_start(a);
        for (int j = 0; j < len; ++j) fs_step(st, sp[k * kFsPad + j]);
        const FsRun r = fs_finish(st);
        float* row = reinterpret_cast<float*>(&sn[k * 4]);
        row[4 + i] = ok ? r.o : 0.0f;
        row[8 + i] = ok ? r.mu : 0.0f;
        row[12 + i] = ok ? r.qm : __builtin_nanf("");
        if (i == 0) {
          row[0] = g;
          row[1] = row[2] = row[3] = 0.0f;
        }
      }
    }
    __syncthreads();
    if (t < kWave) {
      // the walk's speculation data in the record's spare words: the exclusive prefix (double,
      // pad0:pad1) of the member-0 increments over the unit's chunks, and pad2 = mu3, the fast
      // path's margin: when all four members are usable, share one increment and keep their
      // quanta <= 2 q(g), any start t = g + d q(g) with |t - g| <= min_i mu_i - 3 q(g) is
      // covered by its member (|D| <= |t - g| + 3 q) and yields t + the increment.  mu3 < 0:
      // the record needs the full lemma (fs_apply) at every start.
      float* row = reinterpret_cast<float*>(&sn[t * 4]);
      double d0 = 0.0;
      float mu3 = -1.0f;
      if (t < nch) {
        const float g = row[0];
        const double q = (double)fs_quantum(g);
        bool fast = true;
        double mum = INFINITY;
        for (int i = 0; i < kFsFan; ++i) {
          const float o = row[4 + i], mu = row[8 + i], qm = row[12 + i];
          if (!(qm >= 0.0f) || !((double)qm <= 2.0 * q)) fast = false;
          const double di = (double)o - ((double)g + (double)i * q);
          if (i == 0) d0 = di;
          else if (di != d0) fast = false;
          mum = fmin(mum, (double)mu);
        }
        if (!(d0 == d0)) {  // (a non-finite run: left to the exact paths)
          d0 = 0.0;
          fast = false;
        }
        const double m3 = mum - 3.0 * q;
        if (fast && m3 >= 0.0) {
          float f = (float)m3;
          if ((double)f > m3) f = nextafterf(f, 0.0f);  // (rounded down)
          mu3 = f;
        }
      }
      const double inc = wave_incl_scan(d0, t);
      const double ex = inc - d0;
      // the window summary (this unit's 64 records: k_fs_walk passes such a window in one step).
      // Link: member 0's output is the next chunk's guess, bit for bit (past the unit's last
      // chunk: the walk compares o0_last with the next window's g0).  A start t equal
      // to the window's first guess then runs through every guess of the window exactly (each
      // member-0 run is the computation), ending at the last chunk's o0.  A start t = g0 + dl,
      // dl != 0: every record fast, |dl| <= min mu3 and dl a multiple of every quantum q(g_k)
      // (the largest) make each start g_k + dl and the end o0_last + dl (the fast path, record
      // by record, by induction).  Summary: (g0, o0_last, min mu3 or -1 when a record is not
      // fast, the largest quantum or NaN when a link fails).
      const float gk = t < nch ? row[0] : 0.0f, o0 = t < nch ? row[4] : 0.0f;
      bool lk = true;
      if (t < nch) {
        const float gn = t + 1 < nch ? reinterpret_cast<const float*>(&sn[(t + 1) * 4])[0] : 0.0f;
        lk = row[12] >= 0.0f && (t + 1 >= nch || __float_as_uint(o0) == __float_as_uint(gn));
      }
      const bool valid = ballot(t < nch && !lk) == 0;
      const bool fastall = ballot(t < nch && !(mu3 >= 0.0f)) == 0;
      float mn = t < nch ? mu3 : INFINITY, qx = t < nch ? fs_quantum(gk) : 0.0f;
#pragma unroll
      for (int off = 1; off < kWave; off <<= 1) {
        mn = fminf(mn, __shfl_xor(mn, off, kWave));
        qx = fmaxf(qx, __shfl_xor(qx, off, kWave));
      }
      const float g0 = rdl(gk, 0), ol = rdl(o0, nch - 1);
      if (t == 0)
        d.b.win[c * d.b.wcap + u] =
            make_float4(g0, ol, fastall ? mn : -1.0f, valid ? qx : __builtin_nanf(""));
      // (exclusive prefix: inc - d0 may round; the walk verifies every speculated start anyway)
      if (t < nch) {
        const uint64_t eb = (uint64_t)__double_as_longlong(ex);
        row[1] = __uint_as_float((uint32_t)eb);
        row[2] = __uint_as_float((uint32_t)(eb >> 32));
        row[3] = mu3;
      }
      // the integer-stepping table of the record (lanes past nch: unused)
      const float4 q0 = sn[t * 4], q1 = sn[t * 4 + 1], q2 = sn[t * 4 + 2], q3 = sn[t * 4 + 3];
      uint4 s0, s1, s2;
      fs_seq_prep(fs_walk_rec(f32x4{q0.x, q0.y, q0.z, q0.w}, f32x4{q1.x, q1.y, q1.z, q1.w},
                              f32x4{q2.x, q2.y, q2.z, q2.w}, f32x4{q3.x, q3.y, q3.z, q3.w}),
                  nch, t, &s0, &s1, &s2);
      if (t < nch) {
        uint4* o = d.b.srec + 3 * ((int64_t)c * d.b.cap + u * kFsUC + t);
        o[0] = s0; o[1] = s1; o[2] = s2;
      }
    }
    __syncthreads();
    for (int p = t; p < nch * 4; p += kFlBS)
      reinterpret_cast<float4*>(fs_rec(d.b, c, u * kFsUC + (p >> 2)))[p & 3] = sn[p];
  }
}

// ---- k_fs_walk --------------------------------------------------------------------------------

// lane l + 1's value (DPP wave_shl:1; the last lane gets its own)
__device__ __forceinline__ double dpp_next(double v) {
  const uint64_t b = (uint64_t)__double_as_longlong(v);
  const uint32_t lo = (uint32_t)__builtin_amdgcn_update_dpp((int)(uint32_t)b, (int)(uint32_t)b,
                                                            0x130, 0xF, 0xF, false);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_update_dpp((int)(uint32_t)(b >> 32),
                                                            (int)(uint32_t)(b >> 32), 0x130, 0xF,
                                                            0xF, false);
  return __longlong_as_double((int64_t)(((uint64_t)hi << 32) | lo));
}

// chunk k rerun from v (its exact start): its terms one per lane, summed in order
__device__ __forceinline__ float fs_rerun(const FsDev& d, int c, int64_t k, int64_t n, float v,
                                          int lane) {
  const int64_t e0 = k * kFsChunk;
  const int len = n - e0 < kFsChunk ? (int)(n - e0) : kFsChunk;
  const int64_t e = (e0 + (lane < len ? lane : 0)) * d.stride;
  // (inline asm with its own drain: a compiler-visible load here would make the compiler wait on
  // the load counter at the top of every walk iteration, i.e. on the ring's prefetches)
  float x, y, z;
  asm volatile(
      "global_load_dword %0, %3, off\n\t"
      "global_load_dword %1, %4, off\n\t"
      "global_load_dword %2, %5, off\n\t"
      "s_waitcnt vmcnt(0)"
      : "=&v"(x), "=&v"(y), "=&v"(z)
      : "v"(d.px + e), "v"(d.py + e), "v"(d.pz + e)
      : "memory");
  const float p = fs_term(c, x, y, z);
  for (int j = 0; j < len; ++j) v = v + rdl(p, j);
  return v;
}

// fs_increment (fsum.hpp) on the unpacked record (scalar selects: no indexed record array)
__device__ __forceinline__ double fs_increment_rec(const FsWalkRec w, double off) {
  const double qd = w.q();
  const double dd = off * w.iq();
  int i = 0;
  if (fabs(dd) < 4503599627370496.0 && dd == floor(dd)) i = (int)(dd - 4.0 * floor(dd * 0.25));
  const bool u0 = w.q0 >= 0.0f, u1 = w.q1 >= 0.0f, u2 = w.q2 >= 0.0f, u3 = w.q3 >= 0.0f;
  const bool ui = i == 0 ? u0 : i == 1 ? u1 : i == 2 ? u2 : u3;
  if (!ui) i = u0 ? 0 : u1 ? 1 : u2 ? 2 : 3;
  const bool uf = i == 0 ? u0 : i == 1 ? u1 : i == 2 ? u2 : u3;
  if (!uf) return __builtin_nan("");
  const float oi = i == 0 ? w.o0 : i == 1 ? w.o1 : i == 2 ? w.o2 : w.o3;
  return (double)oi - ((double)w.g + (double)i * qd);
}

// fs_apply (fsum.hpp) for the walk, branch-free on the unpacked record: the same decisions and the
// same result bits
__device__ __forceinline__ bool fs_apply_lean(float t, const FsWalkRec w, float* out) {
  const double q = w.q(), iq = w.iq();
  const double tq = (double)t * iq;
  const bool grid = fabs(tq) < 4503599627370496.0 && tq == floor(tq);
  const double dl = tq - (double)w.g * iq;
  const double d4 = floor(dl * 0.25);
  const double fi = dl - 4.0 * d4;  // 0..3 on the grid
  const int i = grid ? (int)fi : 0;
  const double D = (dl - (double)i) * q;
  const bool b1 = i & 1, b2 = i & 2;
  const float qm = b2 ? (b1 ? w.q3 : w.q2) : (b1 ? w.q1 : w.q0);
  const float oi = b2 ? (b1 ? w.o3 : w.o2) : (b1 ? w.o1 : w.o0);
  const float mui = b2 ? (b1 ? w.m3 : w.m2) : (b1 ? w.m1 : w.m0);
  const bool ok = grid && qm >= 0.0f &&
                  (D == 0.0 || ((double)qm <= 2.0 * q && fabs(D) <= (double)mui));
  *out = D == 0.0 ? oi : (float)((double)oi + D);
  return ok;
}

// steps lanes f, f + 1, ... (until `stop` says so) from the exact value t, each by the full lemma
// (fs_apply_lean) or a rerun; returns the next lane.  (An integer form of the step, in units of
// the window's smallest quantum, measured slower on gfx950: its readlanes into scalar registers
// cost ~50 clocks each.)
template <class Stop>
__device__ __forceinline__ int fs_step_lanes(const FsDev& d, int c, int64_t base, int64_t n,
                                             const FsWalkRec wr, int cnt, int f, float* t,
                                             int lane, Stop stop, int64_t* n_step,
                                             int64_t* n_rerun) {
  for (;;) {
    float o3;
    const bool ok2 = fs_apply_lean(*t, wr, &o3);
    ++*n_step;
    if ((ballot(ok2) >> f) & 1) {  // (a ballot bit: cheaper than a readlane into SALU)
      *t = rdl(o3, f);
    } else {
      ++*n_rerun;
      *t = fs_rerun(d, c, base + f, n, *t, lane);
    }
    ++f;
    if (f >= cnt || stop(f)) return f;
  }
}

// A window's records (64 records of 64 bytes, the global layout: 4 KB) are moved into LDS by
// global_load_lds_dwordx4 (4 instructions, no registers); two slots: the window being walked and
// the next one the summaries cannot skip, prefetched.  The loads are counted by vmcnt in issue
// order: with the prefetch's 4 loads issued after the current window's, vmcnt(4) waits for the
// current window (a rerun's own loads drain the counter anyway).
constexpr int kFsSpecIter = 2;  // rounds of member choice per speculation pass
constexpr bool kFsSeq = true;   // after a failed pass: integer stepping (fs_seq_window) ...
constexpr int kFsSeqMin = 4;    // ... in windows with more records than this that are not fast
constexpr bool kFsSeqFirst = true;  // (such windows: no speculation pass first)
constexpr int kFsWinBytes = kWave * (int)sizeof(FsNode);
constexpr int kFsSeqBytes = kWave * 3 * (int)sizeof(uint4);  // a window's integer-stepping tables
constexpr int kFsSlotBytes = kFsWinBytes + kFsSeqBytes;

// a window's tables (3 KB: 3 loads of 1 KB) into LDS behind its records
__device__ __forceinline__ void fs_seq_load(const uint4* T, int64_t base, int64_t K,
                                            uint32_t lds, int lane) {
  const int64_t w0 = base < K ? base : (K - 1) / kWave * kWave;
  const char* src = reinterpret_cast<const char*>(T + 3 * w0) + 16 * lane;
  const int64_t lim = 3 * K * (int64_t)sizeof(uint4) - 16 - 3 * w0 * (int64_t)sizeof(uint4);
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    const int64_t off = (int64_t)j * 1024 + 16 * lane;
    const char* p = off <= lim ? src + j * 1024 : reinterpret_cast<const char*>(T + 3 * w0);
    asm volatile("global_load_lds_dwordx4 %0, off" : : "v"(p), "{m0}"(lds + j * 1024) : "memory");
  }
}

__device__ __forceinline__ void fs_ring_load(const FsNode* R, int64_t base, int64_t K,
                                             __attribute__((address_space(3))) void* slot,
                                             int lane) {
  // (past the last record: the last window's loads re-read valid memory, never used)
  const int64_t w0 = base < K ? base : (K - 1) / kWave * kWave;
  const char* src = reinterpret_cast<const char*>(R + w0) + 16 * lane;
  const int64_t lim = K * (int64_t)sizeof(FsNode) - 16 - w0 * (int64_t)sizeof(FsNode);
  // (inline asm: the compiler neither sees these loads nor drains them before its own LDS and
  // VMEM instructions; the walk waits for them explicitly)
  const uint32_t lds = (uint32_t)(uintptr_t)slot;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int64_t off = (int64_t)j * 1024 + 16 * lane;
    const char* p = off <= lim ? src + j * 1024 : reinterpret_cast<const char*>(R + w0);
    asm volatile("global_load_lds_dwordx4 %0, off" : : "v"(p), "{m0}"(lds + j * 1024) : "memory");
  }
}

struct FsWalkCounters {
  int64_t win = 0, pass = 0, slow = 0, step = 0, rerun = 0, clk_step = 0, group_fast = 0, table = 0;
  // windows walked although tabled: no table published yet, lead not exact / out of the
  // table's range, the lead's lane dropped by the builder
  int64_t miss_none = 0, miss_range = 0, miss_mask = 0;
  int64_t lead_hist = 0;  // (diagnostic) 8-bit counts of |lead| < 128, < 512, < 4096, larger, inexact
};

__device__ __forceinline__ float g0f(const float4& sm, int f) {  // the first guess of window f
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(sm.x), f));
}

// Exact stepping in integers, lanes f..cnt-1 of a window from the exact value t at lane f.
// Every value involved (the guesses, the usable members' outputs, the chain's values where a
// record covers them) is a multiple of Q, the window's smallest quantum of a nonzero guess or
// output, so the chain is followed as its lead over the guesses, L_k = (t_k - g_k) / Q, an int:
// record k applied to t_k = g_k + L_k Q selects member i = (L_k >> s_k) & 3 (q(g_k) = 2^s_k Q),
// and when the lemma covers that start (fs_apply: on the grid, member usable, D = L_k - i 2^s_k
// zero, or within the margin with the member's quanta <= 2 q(g_k)) the next lead is
// L_{k+1} = L_k + E_k[i], E_k[i] = (o_i - i q(g_k) - g_{k+1}) / Q.  One step is a few integer
// operations and a DPP lane shift (|E| < 2^20, |L| < 2^30: 24-bit multiplies, no overflow); the
// coverage is checked for all lanes afterwards, the first uncovered lane is rerun from its exact
// start g_u + L_u Q and the stepping resumes after it.  Returns the value after the window.
__device__ __forceinline__ float fs_seq_window(const FsDev& d, int c, int64_t base, int64_t n,
                                               const FsWalkRec wr, const uint4 sq0,
                                               const uint4 sq1, const uint4 sq2, int cnt, int f,
                                               float t, int lane, FsWalkCounters& ct) {
  const bool act = lane < cnt;
  // the record's table (k_fs_l1: fs_seq_prep)
  const int E0 = (int)sq0.x, F1 = (int)sq0.y, F2 = (int)sq0.z, F3 = (int)sq0.w;
  const int64_t M0 = (int32_t)sq1.x, M1 = (int32_t)sq1.y, M2 = (int32_t)sq1.z, M3 = (int32_t)sq1.w;
  const uint32_t fl = sq2.x;
  const int sh = (int)(fl & 0xFFu);
  const bool exact_only = (fl >> 8) & 1u, gfin = (fl >> 9) & 1u;
  const bool k0 = (fl >> 10) & 1u, k1 = (fl >> 11) & 1u, k2 = (fl >> 12) & 1u, k3 = (fl >> 13) & 1u;
  const bool c0 = (fl >> 14) & 1u, c1 = (fl >> 15) & 1u, c2 = (fl >> 16) & 1u, c3 = (fl >> 17) & 1u;
  const bool tr = act && ((fl >> 18) & 1u);
  const float Qf = __uint_as_float(__builtin_amdgcn_readfirstlane(sq2.y));
  const double Q = (double)Qf, iQ = 1.0 / Q;  // (exact: powers of two)
  while (f < cnt) {
    // the start's lead: t - g_f with its rounding error (TwoSum: the lead must be exact)
    const double ta = (double)t, gb = -(double)rdl(wr.g, f);
    const double sd = ta + gb, bv = sd - ta;
    const double er = (ta - (sd - bv)) + (gb - bv);
    const double Ld = sd * iQ;
    if (!(fabs(Ld) < 1073741824.0) || Ld != floor(Ld) || er != 0.0) {
      // (the start is off the window's grid or far from the guess: no record covers it)
      ++ct.rerun;
      t = fs_rerun(d, c, base + f, n, t, lane);
      ++f;
      continue;
    }
    // the stepping runs over nodes: a record whose increment depends on its start, or a run of
    // translation records (fast, one increment whatever the member) taken as one step with the
    // run's summed increment.  Node j's data are compacted into lane j (ds_permute over a
    // permutation: node starts to their node index, every other lane to a distinct lane >= m).
    const bool in = act && lane >= f;
    const int trv = tr ? 1 : 0;
    const int trprev = __builtin_amdgcn_update_dpp(0, trv, 0x138, 0xF, 0xF, false);  // lane - 1
    const bool ns = in && (lane == f || !tr || !trprev);
    const uint64_t nsm = ballot(ns);
    const int m = (int)__builtin_popcountll(nsm);
    const int nk = (int)__builtin_popcountll(nsm & ((2ull << lane) - 1ull)) - 1;  // (lane 63: all)
    const int ev = in && tr ? E0 : 0;
    const int sxi = wave_incl_scan_i32(ev);
    const int sx = sxi - ev;  // exclusive prefix of the translation increments
    const int sx_tot = __builtin_amdgcn_readlane(sxi, kWave - 1);
    const int dest = in ? (ns ? nk : m + ((lane - f) - (nk + 1))) : lane < f ? (cnt - f) + lane : lane;
    const int pa = dest * 4;
    const int sxj = __builtin_amdgcn_ds_permute(pa, sx);
    const int shj0 = __builtin_amdgcn_ds_permute(pa, sh | (trv << 8));
    const int e0j = __builtin_amdgcn_ds_permute(pa, E0);
    const int f1j = __builtin_amdgcn_ds_permute(pa, F1);
    const int f2j = __builtin_amdgcn_ds_permute(pa, F2);
    const int f3j = __builtin_amdgcn_ds_permute(pa, F3);
    const int sxn = __builtin_amdgcn_update_dpp(sxj, sxj, 0x130, 0xF, 0xF, false);  // lane + 1
    const bool trj = (shj0 >> 8) != 0;
    const int etot = (lane == m - 1 ? sx_tot : sxn) - sxj;  // a translation run's increment
    const int shn = trj ? 0 : (shj0 & 0xFF);
    const int G0 = trj ? etot : e0j, G1 = trj ? etot : f1j, G2 = trj ? etot : f2j,
              G3 = trj ? etot : f3j;
    int cur = (int)Ld, keepn = 0;
#pragma unroll 2
    for (int j = 0; j < m; ++j) {
      keepn = lane == j ? cur : keepn;
      // the member's bits as all-ones / zero masks (signed bit-field extracts), the increment
      // picked by bit-field inserts
      const unsigned m0 = (unsigned)__builtin_amdgcn_sbfe(cur, shn, 1);
      const unsigned m1 = (unsigned)__builtin_amdgcn_sbfe(cur, shn + 1, 1);
      const unsigned lo = (m0 & (unsigned)G1) | (~m0 & (unsigned)G0);
      const unsigned hi = (m0 & (unsigned)G3) | (~m0 & (unsigned)G2);
      const int e = (int)((m1 & hi) | (~m1 & lo));
      cur = __builtin_amdgcn_update_dpp(cur, cur + e, 0x138, 0xF, 0xF, false);  // wave_shr:1
    }
    ct.step += m;
    // every record's lead: its node's lead plus the translation increments before it in the run
    const int keep = __builtin_amdgcn_ds_bpermute(nk * 4, keepn) +
                     (sx - __builtin_amdgcn_ds_bpermute(nk * 4, sxj));
    // coverage of every lane's start (fs_apply's decisions on the integer lead)
    const int64_t L = keep;
    const bool grid = (L & ((1ll << sh) - 1)) == 0;
    const int i = (int)((L >> sh) & 3);
    const int64_t D = L - ((int64_t)i << sh);
    const bool b1 = (i & 2) != 0, b0 = (i & 1) != 0;
    const bool ki = b1 ? (b0 ? k3 : k2) : (b0 ? k1 : k0);
    const bool ci = b1 ? (b0 ? c3 : c2) : (b0 ? c1 : c0);
    const int64_t Mi = b1 ? (b0 ? M3 : M2) : (b0 ? M1 : M0);
    bool cov = gfin && (L < 1073741824 && L > -1073741824) && grid && ki &&
               (D == 0 || (ci && (D < 0 ? -D : D) <= Mi));
    if (exact_only) cov = gfin && L == 0 && k0;
    const uint64_t bad = ballot(act && lane >= f && !cov);
    if (bad == 0) {
      const float oi = b1 ? (b0 ? wr.o3 : wr.o2) : (b0 ? wr.o1 : wr.o0);
      const float out = (float)((double)oi + (double)D * Q);  // (exact: the lemma)
      t = rdl(out, cnt - 1);
      break;
    }
    const int u = (int)__builtin_ctzll(bad);
    // lane u's exact start (a float: g_u + L_u Q is the chain's value), rerun
    const float tu = (float)((double)rdl(wr.g, u) +
                             (double)__builtin_amdgcn_readlane((int)keep, u) * Q);
    ++ct.rerun;
    t = fs_rerun(d, c, base + u, n, tu, lane);
    f = u + 1;
  }
  return t;
}

// one window's walk from the exact value t: speculation passes (fast path, the full lemma where
// it does not decide), lanes stepped alone from the first failed one; returns the value after the
// window's last chunk
__device__ __forceinline__ float fs_walk_window(const FsDev& d, int c, int64_t base, int64_t n,
                                                const FsWalkRec wr, const uint4 sq0,
                                                const uint4 sq1, const uint4 sq2, int cnt, float t,
                                                int lane, FsWalkCounters& ct) {
  const bool fastrec = wr.mu3 >= 0.0f;
  ++ct.win;
  // many records whose increment depends on the start (a sum hovering near zero): after a failed
  // speculation pass the rest of the window is stepped in integers; with few, speculating again
  // after the failed lane is cheaper
  const bool seq = kFsSeq && __builtin_popcountll(ballot(lane < cnt && !fastrec)) > kFsSeqMin;
  if (seq && kFsSeqFirst) {
    const int64_t clk1 = d.b.wst ? (int64_t)clock64() : 0;
    t = fs_seq_window(d, c, base, n, wr, sq0, sq1, sq2, cnt, 0, t, lane, ct);
    if (d.b.wst) ct.clk_step += (int64_t)clock64() - clk1;
    return t;
  }
  int s = 0;
  while (s < cnt) {
    ++ct.pass;
    const bool act = lane >= s && lane < cnt;
    const uint64_t pb = (uint64_t)__double_as_longlong(wr.P);
    const double Ps = __longlong_as_double((int64_t)(
        (uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)pb, s) |
        ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(pb >> 32), s) << 32)));
    // the speculated starts: t + the member-0 increments of lanes s.., corrected where a chunk's
    // increment depends on its start (its member chosen by the walk's lead on the guesses at s)
    double corr = 0.0;
    const uint64_t slowm = ballot(act && !fastrec);
    const double tb = (double)t + (wr.P - Ps);  // (the member-0 increments alone)
    if (slowm) {
      // the records whose increment depends on the start (member i = lead / q mod 4): each
      // lane's lead over its guess from the speculated start, the corrections' prefix from the
      // members those leads select, repeated while a lead changes (every round settles at least
      // the first lane whose member changed: a sum hovering near zero has many such records)
      double off = tb - wr.gd();
      for (int it = 0; it < kFsSpecIter; ++it) {
        const double cl = act && !fastrec ? fs_increment_rec(wr, off) - wr.d0 : 0.0;
        const double inc = wave_incl_scan(cl, lane);
        corr = dpp_dbl<0x138, 0xF>(inc);  // wave_shr:1 (lane 0 reads 0): the exclusive prefix
        const double on = (tb + corr) - wr.gd();
        if (ballot(act && !fastrec && !(on == off)) == 0) break;
        off = on;
      }
    }
    const double tl = tb + corr;
    // the next lane's speculated start (DPP wave shift: no LDS instruction on this path)
    const double tn = dpp_next(tl);
    const bool last = lane == cnt - 1;
    // fast path (see k_fs_l1): a float start within mu3 of the guess, on its quantum grid
    const double dq = tl * wr.iq();
    double out = tl + wr.d0;
    bool ver = fastrec && (double)(float)tl == tl && fabs(tl - wr.gd()) <= (double)wr.mu3 &&
               dq == floor(dq) && (double)(float)out == out && (last || out == tn);
    if (ballot(act && !ver)) {
      ++ct.slow;
      // the full lemma where the fast path does not decide
      float o2;
      const float tf = (float)tl;
      const bool ok = (double)tf == tl && fs_apply_lean(tf, wr, &o2);
      if (!ver) {
        out = (double)o2;
        ver = ok && (last || out == tn);
      }
    }
    const uint64_t bad = ballot(act && !ver);
    if (bad == 0) {
      t = rdl((float)out, cnt - 1);
      break;
    }
    int f = (int)__builtin_ctzll(bad);
    if (seq) {
      // lanes s..f-1 verified, f's start is exact: the rest of the window in integer steps
      t = f == s ? t : rdl((float)out, f - 1);
      const int64_t clk1 = d.b.wst ? (int64_t)clock64() : 0;
      t = fs_seq_window(d, c, base, n, wr, sq0, sq1, sq2, cnt, f, t, lane, ct);
      if (d.b.wst) ct.clk_step += (int64_t)clock64() - clk1;
      break;
    }
    // lanes s..f-1 verified: f's start is exact.  Step lane by lane from f while the records
    // need the full lemma, then speculate again.
    t = f == s ? t : rdl((float)out, f - 1);
    const int64_t clk1 = d.b.wst ? (int64_t)clock64() : 0;
    const uint64_t fastm = ballot(fastrec);
    f = fs_step_lanes(d, c, base, n, wr, cnt, f, &t, lane,
                      [&](int l) { return ((fastm >> l) & 1) != 0; }, &ct.step, &ct.rerun);
    if (d.b.wst) ct.clk_step += (int64_t)clock64() - clk1;
    s = f;
  }
  return t;
}

// Walks windows [w_lo, w_hi) of chain c from the value t (the batch loop of summaries, window
// walks and the record ring).  kRecord: vw[w] = the value the walk enters window w with.
// kRepair (t is the exact start of the span, vw holds a walk of the span from another start):
// stops at the first window whose entry value equals vw[w] bit for bit -- from there both walks
// are the same computation -- and returns true.  *tp = the value after the last window walked.
template <bool kRepair, bool kRecord>
__device__ bool fs_walk_span(const FsDev& d, int c, int64_t w_lo, int64_t w_hi, float* tp,
                             int lane, __attribute__((address_space(3))) char* ring,
                             __attribute__((address_space(3))) uint64_t* tl, FsWalkCounters& ct) {
  const int64_t n = *d.n_dev;
  const int64_t K = fs_chunks(n);
  const int64_t NW = (K + kWave - 1) / kWave;
  const FsNode* R = fs_rec(d.b, c, 0);
  const uint4* T = d.b.srec + 3 * (int64_t)c * d.b.cap;
  const float4* S = d.b.win + c * d.b.wcap;
  float* V = d.b.vw + c * d.b.wcap;
  float t = *tp;
  auto slot = [&](int j) {
    return (__attribute__((address_space(3))) void*)(ring + j * kFsSlotBytes);
  };
  auto tslot = [&](int j) { return (uint32_t)(uintptr_t)slot(j) + (uint32_t)kFsWinBytes; };
  int64_t pre_w = -1;  // the window prefetched into slot pre_s (or none)
  int pre_s = 0;
  int64_t tg0 = -(int64_t)kFtGroup - 1;  // the first window of the tables in tl
  bool met = false;
  for (int64_t wb = w_lo; wb < w_hi && !met; wb += kWave) {
    // the batch's summaries, lane = window; a window is skippable only if its last record also
    // links to the next window's first guess
    const int nb = w_hi - wb < kWave ? (int)(w_hi - wb) : kWave;
    float4 sm = make_float4(0.0f, 0.0f, -1.0f, __builtin_nanf(""));
    float gnx = 0.0f;
    const bool has_next = wb + lane + 1 < NW;
    if (lane < nb) sm = S[wb + lane];
    if (lane < nb && has_next) gnx = S[wb + lane + 1].x;
    const float vb = kRepair && lane < nb ? V[wb + lane] : 0.0f;
    const bool valid = lane < nb && sm.w == sm.w &&
                       (!has_next || __float_as_uint(sm.y) == __float_as_uint(gnx));
    const uint64_t stat = ballot(lane < nb && !valid);  // (walked at any lag: prefetch candidates)
    // (fs_wtab_item builds tables only for windows without a fast summary)
    const uint64_t tabled = ballot(lane < nb && !(sm.z >= 0.0f && sm.w == sm.w));
    const double iqx = valid ? 1.0 / (double)sm.w : 0.0;  // (exact: a power of two)
    int i = 0;
    while (i < nb) {
      // windows i.. from the exact value t: lag dl = t - g0_i, the same for every linked window
      const float g0 = rdl(sm.x, i);
      const bool zero = __float_as_uint(t) == __float_as_uint(g0);
      const double dl = (double)t - (double)g0;
      const double dq = dl * iqx;
      const bool ok = lane >= i && valid &&
                      (zero || (fabs(dl) <= (double)sm.z && fabs(dq) < 4503599627370496.0 &&
                                dq == floor(dq)));
      const uint64_t nm = ~ballot(ok) & (~0ull << i) & (nb == kWave ? ~0ull : (1ull << nb) - 1);
      const int f = nm ? (int)__builtin_ctzll(nm) : nb;
      // entry values of windows i..f: linked windows passed with lag dl enter at g0 + dl
      // (exact: the lemma); window f at t after them
      const float ent = zero ? sm.x : (float)((double)sm.x + dl);
      if (kRepair) {
        if (ballot(lane >= i && lane < f && __float_as_uint(ent) == __float_as_uint(vb))) {
          met = true;
          break;
        }
      }
      if (kRecord && lane >= i && lane < f) V[wb + lane] = ent;
      if (f > i) {
        const float ol = rdl(sm.y, f - 1);
        t = zero ? ol : (float)((double)ol + dl);  // (exact: the lemma, record by record)
        ct.group_fast += f - i;
      }
      if (f >= nb) break;
      if (kRepair && __float_as_uint(t) == __float_as_uint(rdl(vb, f))) {
        met = true;
        break;
      }
      if (kRecord && lane == 0) V[wb + f] = t;
      const int64_t w = wb + f;
      if ((tabled >> f) & 1) {  // the window's transfer table (fs_wtab_item): the exit value
                                // when the entry lead is in it
        if (w < tg0 || w >= tg0 + kFtGroup) {  // the next kFtGroup windows' tables into LDS
          tg0 = w;
          uint64_t e[kFtGroup * kFtHalves];
#pragma unroll
          for (int j = 0; j < kFtGroup * kFtHalves; ++j)
            e[j] = w + j / kFtHalves < NW
                       ? __hip_atomic_load(reinterpret_cast<const uint64_t*>(
                                               d.b.wtab + (c * d.b.wcap + w) * kFtW + j * kWave + lane),
                                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                       : 0ull;
          const uint64_t qv = lane < kFtGroup && w + lane < NW
                                  ? __hip_atomic_load(reinterpret_cast<const uint64_t*>(
                                        d.b.wq + c * d.b.wcap + w + lane),
                                    __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                                  : 0ull;
          __builtin_amdgcn_wave_barrier();
#pragma unroll
          for (int j = 0; j < kFtGroup * kFtHalves; ++j) tl[j * kWave + lane] = e[j];
          if (lane < kFtGroup) tl[kFtGroup * kFtW + lane] = qv;
          __builtin_amdgcn_wave_barrier();
        }
        const int gj = (int)(w - tg0);
        uint64_t qv = tl[kFtGroup * kFtW + gj];
        if ((uint32_t)(qv >> 32) != d.gen)  // (not built when prefetched: read it again)
          qv = __hip_atomic_load(reinterpret_cast<const uint64_t*>(d.b.wq + c * d.b.wcap + w),
                                 __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if ((uint32_t)(qv >> 32) != d.gen) {
          ++ct.miss_none;
        } else {
          const double Q = (double)__uint_as_float((uint32_t)qv);
          // the lead t - g_0 with its rounding error (TwoSum: it must be exact), in units of Q
          const double ta = (double)t, gb = -(double)g0f(sm, f);
          const double sd = ta + gb, bv = sd - ta;
          const double er = (ta - (sd - bv)) + (gb - bv);
          const double Ld = sd * (1.0 / Q) + (double)kFtLo;
          const bool inr = er == 0.0 && Ld == floor(Ld) && Ld >= 0.0 && Ld < (double)kFtW;
          if (inr) {
            const int li = (int)Ld;
            uint64_t ev = tl[gj * kFtW + li];
            if ((uint32_t)(ev >> 32) != d.gen)
              ev = __hip_atomic_load(reinterpret_cast<const uint64_t*>(
                                         d.b.wtab + (c * d.b.wcap + w) * kFtW + li),
                                     __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if ((uint32_t)(ev >> 32) == d.gen) {
              t = __uint_as_float((uint32_t)ev);
              ++ct.table;
              i = f + 1;
              continue;
            }
            ++ct.miss_mask;
          } else {
            ++ct.miss_range;
            if (d.b.wst) {
              const double aL = fabs(Ld - (double)kFtLo);
              const int bkt = (er != 0.0 || Ld != floor(Ld)) ? 4 : aL < 128 ? 0 : aL < 512 ? 1
                              : aL < 4096 ? 2 : 3;
              if (((ct.lead_hist >> (8 * bkt)) & 0xFF) < 0xFF) ct.lead_hist += 1ll << (8 * bkt);
            }
          }
        }
      }
      // window f record by record
      const int cur = pre_w == w ? pre_s : pre_s ^ 1;
      if (pre_w != w) {
        fs_ring_load(R, w * kWave, K, slot(cur), lane);
        fs_seq_load(T, w * kWave, K, tslot(cur), lane);
      }
      // prefetch the next window the summaries cannot skip at any lag (inside the span)
      const uint64_t nx = f + 1 < kWave ? stat & (~0ull << (f + 1)) : 0ull;
      pre_w = nx ? wb + (int64_t)__builtin_ctzll(nx) : -1;
      pre_s = cur ^ 1;
      if (pre_w >= 0) {
        fs_ring_load(R, pre_w * kWave, K, slot(pre_s), lane);
        fs_seq_load(T, pre_w * kWave, K, tslot(pre_s), lane);
        asm volatile("s_waitcnt vmcnt(7)" ::: "memory");
      } else {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      f32x4 r0, r1, r2, r3;
      uint4 q0, q1, q2;
      const uint32_t la = (uint32_t)(uintptr_t)(
          (__attribute__((address_space(3))) char*)slot(cur) + sizeof(FsNode) * lane);
      const uint32_t lt = tslot(cur) + 3u * 16u * (uint32_t)lane;
      // (inline asm: the compiler would otherwise drain every outstanding load before an LDS
      // read that may alias an LDS-DMA write)
      asm volatile(
          "ds_read_b128 %0, %7\n\t"
          "ds_read_b128 %1, %7 offset:16\n\t"
          "ds_read_b128 %2, %7 offset:32\n\t"
          "ds_read_b128 %3, %7 offset:48\n\t"
          "ds_read_b128 %4, %8\n\t"
          "ds_read_b128 %5, %8 offset:16\n\t"
          "ds_read_b128 %6, %8 offset:32\n\t"
          "s_waitcnt lgkmcnt(0)"
          : "=&v"(r0), "=&v"(r1), "=&v"(r2), "=&v"(r3), "=&v"(q0), "=&v"(q1), "=&v"(q2)
          : "v"(la), "v"(lt)
          : "memory");
      const int64_t b0 = w * kWave;
      const int cn = K - b0 < kWave ? (int)(K - b0) : kWave;
      t = fs_walk_window(d, c, b0, n, fs_walk_rec(r0, r1, r2, r3), q0, q1, q2, cn, t, lane, ct);
      i = f + 1;
    }
  }
  __builtin_amdgcn_s_waitcnt(0);  // (a last prefetch: never read, but drained)
  *tp = t;
  return met;
}

// The walk: one wave per chain over all its windows, from the exact start (start9, or zero) or,
// kFwGuess (several ranks, rank r > 0), from the refined guess at the rank's first inlier; it
// stores the start it took after the end values (sums[9 + c]) and, kFwRecord, every window's entry
// value for k_fs_repair.  Several ranks walk twice (launch_fs_refit): a segment walked from its
// double-prefix guess alone hovers near zero in some chains, its start is off by many quanta of
// the small binades there, a walk from the exact start never meets it and the repairs walked
// every segment a second time, one rank after another (round 4).
// The last chain to finish runs the refit tail when asked.
constexpr int kFwBS = kWave;
constexpr int kFwGuess = 1, kFwRecord = 2;  // k_fs_walk's mode bits
// segmented walk: the last of a chain's segment walkers to finish joins the chain's segments
// itself (k_fs_segfix's body) instead of a separate k_fs_segfix launch
constexpr int kFwJoin = 4;
constexpr int kFwSegShift = 8;               // mode >> kFwSegShift: segments per chain (> 1)
// segments a chain's NW windows are walked in (at most S, at least kFsSegWin windows each)
__device__ __forceinline__ int fs_seg_count(int64_t NW, int S) {
  const int64_t m = NW / kFsSegWin;
  return (int)(m < 1 ? 1 : m < S ? m : S);
}
__device__ void fs_walk_finish(const FsDev& d, int c, float t, int lane, int64_t n,
                               const float4* __restrict__ cin, float4* __restrict__ cout,
                               int32_t* __restrict__ res);
__device__ void fs_seg_join(const FsDev& d, int c, const float* __restrict__ start9, int S,
                            const float4* __restrict__ cin, float4* __restrict__ cout,
                            int32_t* __restrict__ res, int lane,
                            __attribute__((address_space(3))) char* ring,
                            __attribute__((address_space(3))) uint64_t* tl);
__device__ __forceinline__ void fs_put_counters(const FsDev& d, int c, const FsWalkCounters& ct,
                                                int64_t clk0, bool add) {
  int64_t* w = d.b.wst + 8 * c;
  const int64_t v[8] = {ct.win, ct.pass | (ct.miss_none << 32), ct.slow | (ct.miss_range << 32),
                        ct.step | (ct.lead_hist << 24), ct.rerun | (ct.miss_mask << 32),
                        (int64_t)clock64() - clk0, ct.clk_step, ct.group_fast + (ct.table << 32)};
  for (int k = 0; k < 8; ++k) {
    if (add) atomicAdd(reinterpret_cast<unsigned long long*>(w + k), (unsigned long long)v[k]);
    else w[k] = v[k];
  }
}
__global__ __launch_bounds__(kFwBS) void k_fs_walk(FsDev d, const float* __restrict__ start9,
                                                   int mode, const float4* __restrict__ cin,
                                                   float4* __restrict__ cout,
                                                   int32_t* __restrict__ res) {
  __shared__ __attribute__((aligned(16))) char ring_raw[2 * kFsSlotBytes];
  __shared__ uint64_t tl_raw[kFtLdsWords];
  auto* ring = (__attribute__((address_space(3))) char*)ring_raw;
  auto* tl = (__attribute__((address_space(3))) uint64_t*)tl_raw;
  const int S = mode >> kFwSegShift;  // (segmented walk: S segments per chain)
  const bool segmented = S > 1;
  const int nwalk = kFsChains * (segmented ? S : 1);
  const int c = (int)blockIdx.x % kFsChains, sg = (int)blockIdx.x / kFsChains;
  const int lane = threadIdx.x;
  const int64_t n = *d.n_dev;
  const int64_t NW = (fs_chunks(n) + kWave - 1) / kWave;
  if ((int)blockIdx.x >= nwalk) {
    // a table builder: (window, chain) items in window order, so the walkers find the early
    // windows' tables first
    FsTabLds& L_ = *reinterpret_cast<FsTabLds*>(ring_raw);
    static_assert(sizeof(FsTabLds) <= 2 * kFsSlotBytes, "builder state fits the ring's LDS");
    for (int64_t it = blockIdx.x - nwalk; it < NW * kFsChains * kFtHalves; it += gridDim.x - nwalk)
      fs_wtab_item(d, (int)(it % kFsChains), it / (kFsChains * kFtHalves),
                   (int)((it / kFsChains) % kFtHalves), lane, L_);
    return;
  }
  // walk counters (dlg_float_sums' walk_stats): windows walked record by record, speculation
  // passes, passes with lanes the fast path could not decide, lanes stepped alone, reruns, clocks
  // (all, stepping), windows passed by their summaries
  const int64_t clk0 = d.b.wst ? (int64_t)clock64() : 0;
  FsWalkCounters ct;
  float t = start9 ? start9[c] : 0.0f;
  float t0 = t;
  if (segmented) {
    // segment sg of the chain's windows, from the refined guess at its first record (segment 0:
    // the exact start), recording the windows' entries for k_fs_segfix
    const int Se = fs_seg_count(NW, S);
    if (sg >= Se) return;
    const int64_t w_lo = NW * sg / Se, w_hi = NW * (sg + 1) / Se;
    if (sg > 0) t = fs_rec(d.b, c, w_lo * kWave)->g;
    t0 = t;
    fs_walk_span<false, true>(d, c, w_lo, w_hi, &t, lane, ring, tl, ct);
  } else {
    if ((mode & kFwGuess) && NW > 0) t = fs_rec(d.b, c, 0)->g;
    if (lane == 0) d.b.sums[kFsChains + c] = t;  // (the start taken; k_fs_guess2 reads it)
    if (mode & kFwRecord)
      fs_walk_span<false, true>(d, c, 0, NW, &t, lane, ring, tl, ct);
    else
      fs_walk_span<false, false>(d, c, 0, NW, &t, lane, ring, tl, ct);
  }
  if (d.b.wst && lane == 0) fs_put_counters(d, c, ct, clk0, segmented);
  if (segmented) {
    if (lane == 0) {
      d.b.seg[(c * kFsSegMax + sg) * 2] = t0;
      d.b.seg[(c * kFsSegMax + sg) * 2 + 1] = t;
    }
    if (!(mode & kFwJoin)) return;
    // the chain's last segment to finish joins them (one wave per workgroup: the release fence
    // waits for every lane's stores -- the segment's (start, end) and its recorded window
    // entries -- before the arrival; the joiner's acquire fence drops its stale L1 lines)
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    unsigned arrived = 0;
    if (lane == 0)
      arrived = __hip_atomic_fetch_add(d.b.ticket + 2 + c, 1u, __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_AGENT);
    arrived = __builtin_amdgcn_readfirstlane(arrived);
    if (arrived != (unsigned)fs_seg_count(NW, S) - 1) return;
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    if (lane == 0) d.b.ticket[2 + c] = 0u;  // (zero again for the next launch)
    fs_seg_join(d, c, start9, S, cin, cout, res, lane, ring, tl);
    return;
  }
  fs_walk_finish(d, c, t, lane, n, cin, cout, res);
}

// the chain's end value into sums; with cout, the last chain to finish runs the refit tail
__device__ void fs_walk_finish(const FsDev& d, int c, float t, int lane, int64_t n,
                               const float4* __restrict__ cin, float4* __restrict__ cout,
                               int32_t* __restrict__ res) {
  __shared__ unsigned s_ticket;
  if (lane == 0) {
    __hip_atomic_store(reinterpret_cast<int32_t*>(d.b.sums) + c, __float_as_int(t),
                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __builtin_amdgcn_s_waitcnt(0);
    s_ticket = cout ? __hip_atomic_fetch_add(d.b.ticket + 1, 1u, __ATOMIC_RELAXED,
                                             __HIP_MEMORY_SCOPE_AGENT)
                    : 0u;
  }
  __syncthreads();
  if (!cout || s_ticket != kFsChains - 1 || lane != 0) return;
  d.b.ticket[1] = 0u;
  float a9[kFsChains];
  for (int k = 0; k < kFsChains; ++k)
    a9[k] = __int_as_float(__hip_atomic_load(reinterpret_cast<const int32_t*>(d.b.sums) + k,
                                             __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
  const float4 ci = *cin;
  const float cv[4] = {ci.x, ci.y, ci.z, ci.w};
  float co[4];
  bool unc = false;
  fs_refit_tail(a9, n, cv, co, &unc);
  *cout = make_float4(co[0], co[1], co[2], co[3]);
  res[0] = unc ? 1 : 0;
  res[1] = (int32_t)n;
  for (int k = 0; k < kFsChains; ++k) res[2 + k] = __float_as_int(a9[k]);
}

// several ranks, rank > 0: k_fs_walk ran from the rank's guess (from_guess) while the ranks
// before it walked theirs; with the exact start from the previous rank, the chain is walked again
// from it only until it enters a window with the value the recorded walk entered it with (from
// there both are the same computation, so the recorded end is exact).  A chain whose guess was
// exact is not walked at all; one with a constant lag passes its windows by their summaries.
__global__ __launch_bounds__(kFwBS) void k_fs_repair(FsDev d, const float* __restrict__ start9) {
  __shared__ __attribute__((aligned(16))) char ring_raw[2 * kFsSlotBytes];
  __shared__ uint64_t tl_raw[kFtLdsWords];
  auto* ring = (__attribute__((address_space(3))) char*)ring_raw;
  auto* tl = (__attribute__((address_space(3))) uint64_t*)tl_raw;
  const int c = blockIdx.x, lane = threadIdx.x;
  const int64_t n = *d.n_dev;
  const int64_t NW = (fs_chunks(n) + kWave - 1) / kWave;
  FsWalkCounters ct;
  float t = start9[c];
  if (lane == 0) d.b.sums[kFsChains + c] = t;
  if (NW == 0) {  // (an empty shard passes its start on)
    if (lane == 0) d.b.sums[c] = t;
    return;
  }
  if (__float_as_uint(t) == __float_as_uint(d.b.vw[c * d.b.wcap])) return;  // (sums: exact)
  // (recording: a later repair compares with this walk; windows left with an older walk's entry
  // are ones both walks enter alike or lie past a meeting point -- every walk recorded there
  // ends at the same value)
  const bool met = fs_walk_span<true, true>(d, c, 0, NW, &t, lane, ring, tl, ct);
  if (!met && lane == 0) d.b.sums[c] = t;  // (met: the recorded walk's end is exact)
}

// several ranks, between the two walks: rank r's propagated guess.  gath2[j] holds rank j's first
// walk (ends, then the starts it took); rank 0's walk was exact, and every chain behaves like a
// translation over a small shift of its start, so rank j's guess moved by the rank before's
// error-so-far:  G''_j = End_{j-1} + (G''_{j-1} - G_{j-1})  (in double, rounded each step;
// G''_0 = G_0 = 0).  Measured on C3's inlier list in 8 shards: within 2 quanta of the exact
// start, where the double-prefix guesses G_j were off by up to ~1400.
__global__ void k_fs_guess2(const float* __restrict__ gath2, int rank, float* __restrict__ g2) {
  const int c = threadIdx.x;
  if (c >= kFsChains) return;
  float gc = 0.0f;
  for (int j = 1; j <= rank; ++j) {
    const float* pj = gath2 + (j - 1) * 2 * kFsChains;
    gc = (float)((double)pj[c] + ((double)gc - (double)pj[kFsChains + c]));
  }
  g2[c] = gc;
}

// one rank, segmented walk: chain c's segments joined in order.  Segment 0 started exactly; a
// later segment whose recorded start equals the exact end of the one before was exact itself,
// else it is walked again from that end until it meets its recorded walk (k_fs_repair's rule).
// Then as k_fs_walk's end: sums, and the last chain to finish runs the refit tail.
__device__ void fs_seg_join(const FsDev& d, int c, const float* __restrict__ start9, int S,
                            const float4* __restrict__ cin, float4* __restrict__ cout,
                            int32_t* __restrict__ res, int lane,
                            __attribute__((address_space(3))) char* ring,
                            __attribute__((address_space(3))) uint64_t* tl) {
  const int64_t n = *d.n_dev;
  const int64_t NW = (fs_chunks(n) + kWave - 1) / kWave;
  const float* sg = d.b.seg + c * kFsSegMax * 2;
  float t = start9 ? start9[c] : 0.0f;
  if (NW > 0) {
    const int Se = fs_seg_count(NW, S);
    t = sg[1];
    FsWalkCounters ct;
    for (int s = 1; s < Se; ++s) {
      const float s0 = sg[2 * s], e0 = sg[2 * s + 1];
      if (__float_as_uint(t) != __float_as_uint(s0)) {
        const int64_t w_lo = NW * s / Se, w_hi = NW * (s + 1) / Se;
        if (!fs_walk_span<true, false>(d, c, w_lo, w_hi, &t, lane, ring, tl, ct)) continue;
      }
      t = e0;
    }
  }
  fs_walk_finish(d, c, t, lane, n, cin, cout, res);
}

// (DLG_OPT_FS_JOIN 0: the joins as their own launch, one wave per chain -- round 5's form)
__global__ __launch_bounds__(kFwBS) void k_fs_segfix(FsDev d, const float* __restrict__ start9,
                                                     int S, const float4* __restrict__ cin,
                                                     float4* __restrict__ cout,
                                                     int32_t* __restrict__ res) {
  __shared__ __attribute__((aligned(16))) char ring_raw[2 * kFsSlotBytes];
  __shared__ uint64_t tl_raw[kFtLdsWords];
  auto* ring = (__attribute__((address_space(3))) char*)ring_raw;
  auto* tl = (__attribute__((address_space(3))) uint64_t*)tl_raw;
  fs_seg_join(d, (int)blockIdx.x, start9, S, cin, cout, res, (int)threadIdx.x, ring, tl);
}

size_t align256(size_t b) { return (b + 255) & ~(size_t)255; }

}  // namespace

size_t fs_scratch_bytes(int64_t n_cap, int world) {
  const int64_t nc = n_cap > 0 ? n_cap : 1;
  const int64_t K = fs_chunks(nc), U = (K + kFsUC - 1) / kFsUC;
  return align256(sizeof(double) * K * kFsChains) + 2 * align256(sizeof(double) * U * kFsChains) +
         align256(sizeof(FsNode) * K * kFsChains) + align256(3 * sizeof(uint4) * K * kFsChains) +
         align256(sizeof(float4) * U * kFsChains) +
         align256(sizeof(float) * 64) +
         align256(sizeof(double) * 32) + align256(sizeof(double) * (kFsChains + 1) * world) +
         align256(sizeof(float) * 2 * kFsChains * world) +
         align256(sizeof(float) * 2 * kFsChains * kFsSegMax) +
         align256(sizeof(float) * U * kFsChains) + align256(sizeof(uint2) * U * kFsChains * kFtW) +
         align256(sizeof(uint2) * U * kFsChains) + 256;
}

FsBuffers fs_carve(void* base, int64_t n_cap, int world) {
  const int64_t nc = n_cap > 0 ? n_cap : 1;
  const int64_t K = fs_chunks(nc), U = (K + kFsUC - 1) / kFsUC;
  uint8_t* p = static_cast<uint8_t*>(base);
  FsBuffers b;
  b.csum = reinterpret_cast<double*>(p);
  p += align256(sizeof(double) * K * kFsChains);
  b.usum = reinterpret_cast<double*>(p);
  p += align256(sizeof(double) * U * kFsChains);
  b.upre = reinterpret_cast<double*>(p);
  p += align256(sizeof(double) * U * kFsChains);
  b.rec = reinterpret_cast<FsNode*>(p);
  b.cap = K;
  p += align256(sizeof(FsNode) * K * kFsChains);
  b.srec = reinterpret_cast<uint4*>(p);
  p += align256(3 * sizeof(uint4) * K * kFsChains);
  b.win = reinterpret_cast<float4*>(p);
  b.wcap = U;
  p += align256(sizeof(float4) * U * kFsChains);
  b.sums = reinterpret_cast<float*>(p);  // [0..8] end values, [9..17] starts, [32..40] the
  b.start9 = b.sums + 32;                 // received starts, [48..56] the propagated guesses
  b.g2 = b.sums + 48;
  p += align256(sizeof(float) * 64);
  b.tot = reinterpret_cast<double*>(p);       // [0..9] this rank's totals + count, [16..24] base
  b.base9 = b.tot + 16;
  b.n_global = reinterpret_cast<int64_t*>(b.tot + 26);
  p += align256(sizeof(double) * 32);
  b.gath = reinterpret_cast<double*>(p);      // [world][10]
  p += align256(sizeof(double) * (kFsChains + 1) * world);
  b.gath2 = reinterpret_cast<float*>(p);      // [world][18]
  p += align256(sizeof(float) * 2 * kFsChains * world);
  b.seg = reinterpret_cast<float*>(p);        // [9][kFsSegMax][2]
  p += align256(sizeof(float) * 2 * kFsChains * kFsSegMax);
  b.vw = reinterpret_cast<float*>(p);
  p += align256(sizeof(float) * U * kFsChains);
  b.wtab = reinterpret_cast<uint2*>(p);
  p += align256(sizeof(uint2) * U * kFsChains * kFtW);
  b.wq = reinterpret_cast<uint2*>(p);
  p += align256(sizeof(uint2) * U * kFsChains);
  b.ticket = reinterpret_cast<unsigned*>(p);  // [0]: k_fs_prep / k_fs_inc, [1]: k_fs_walk,
                                              // [2 + c]: chain c's segments done (kFwJoin)
  return b;
}

namespace {
std::atomic<uint32_t> s_gen{0};  // launch stamps of the window tables (0: never a valid entry)

__global__ void k_fs_poison(uint2* __restrict__ p, int64_t n, uint32_t stamp) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) p[i] = make_uint2(0x3F800000u + (uint32_t)(i & 0xFFFF), stamp);
}
}  // namespace

hipError_t fs_reset(const FsBuffers& b, hipStream_t s, bool poison) {
  const int64_t nt = (int64_t)kFsChains * b.wcap * kFtW, nq = (int64_t)kFsChains * b.wcap;
  if (poison) {
    const uint32_t next = s_gen.load() + 1u;  // (the stamp the next launch will use)
    hipLaunchKernelGGL(k_fs_poison, dim3((unsigned)((nt + 255) / 256)), dim3(256), 0, s, b.wtab, nt,
                       next);
    hipLaunchKernelGGL(k_fs_poison, dim3((unsigned)((nq + 255) / 256)), dim3(256), 0, s, b.wq, nq,
                       next);
  }
  hipError_t e = hipMemsetAsync(b.wtab, 0, sizeof(uint2) * (size_t)nt, s);
  if (e == hipSuccess) e = hipMemsetAsync(b.wq, 0, sizeof(uint2) * (size_t)nq, s);
  if (e == hipSuccess) e = hipMemsetAsync(b.ticket, 0, (2 + kFsChains) * sizeof(unsigned), s);
  return e;
}

void launch_fs_refit(const float* px, const float* py, const float* pz, int stride,
                     const int32_t* n_dev, int64_t n_cap, const FsBuffers& b, const float4* cin,
                     float4* cout, int32_t* res, int num_cus, hipStream_t s, Comm* comm,
                     hipEvent_t ev_walk0, hipEvent_t ev_walk1, hipEvent_t ev_rep0,
                     hipEvent_t ev_rep1, int protocol, int* repairs, int segments,
                     hipEvent_t ev_mid0, hipEvent_t ev_mid1, bool fused_join) {
  uint32_t gen = ++s_gen;
  if (gen == 0) gen = ++s_gen;  // (0 marks a dropped table entry)
  FsDev d{px, py, pz, stride, n_dev, b, gen};
  const unsigned gw = (unsigned)(kFsChains +
      std::max<int64_t>(1, std::min<int64_t>(((n_cap > 0 ? n_cap : 1) + kFsUnit - 1) / kFsUnit *
                                                 kFsChains * kFtHalves,
                                             6 * (int64_t)num_cus)));
  const int64_t nc = n_cap > 0 ? n_cap : 1;
  const int64_t U = (fs_chunks(nc) + kFsUC - 1) / kFsUC;
  const int gp = (int)std::min<int64_t>(U, 2 * (int64_t)num_cus);
  const int gl = (int)std::min<int64_t>(U * kFsChains, 8 * (int64_t)num_cus);
  const int W = comm ? comm->world() : 1, r = comm ? comm->rank() : 0;
  if (W == 1) {
    hipLaunchKernelGGL(k_fs_prep, dim3(gp), dim3(kFpBS), 0, s, d, nullptr, nullptr);
    hipLaunchKernelGGL(k_fs_inc, dim3(gp), dim3(kFiBS), 0, s, d, nullptr);
    hipLaunchKernelGGL(k_fs_l1, dim3(gl), dim3(kFlBS), 0, s, d);
    const int S = std::min(std::max(segments, 1), kFsSegMax);
    if (S > 1) {
      // segmented: kFsChains x S walkers (+ the table builders), then the joins -- by each
      // chain's last segment walker (fused_join), or as a launch of their own
      if (fused_join) {
        DLG_LAUNCH_EV(k_fs_walk, dim3(gw + kFsChains * (S - 1)), dim3(kFwBS), 0, s, ev_walk0,
                              ev_walk1, d, (const float*)nullptr, S << kFwSegShift | kFwJoin, cin,
                              cout, res);
        return;
      }
      DLG_LAUNCH_EV(k_fs_walk, dim3(gw + kFsChains * (S - 1)), dim3(kFwBS), 0, s, ev_walk0,
                            nullptr, d, (const float*)nullptr, S << kFwSegShift,
                            (const float4*)nullptr, (float4*)nullptr, (int32_t*)nullptr);
      DLG_LAUNCH_EV(k_fs_segfix, dim3(kFsChains), dim3(kFwBS), 0, s, nullptr, ev_walk1,
                            d, (const float*)nullptr, S, cin, cout, res);
      return;
    }
    DLG_LAUNCH_EV(k_fs_walk, dim3(gw), dim3(kFwBS), 0, s, ev_walk0, ev_walk1, d,
                          nullptr, 0, cin, cout, res);
    return;
  }
  // several ranks (the list is the ranks' segments in order): each rank's guesses start from the
  // double totals of the ranks before it, and every rank walks its shard at once -- rank 0 from
  // the exact start, rank r > 0 from the refined guess at its first inlier.  The (start, end)
  // pairs are allgathered; rank r > 0 moves its base to the guess they propagate (k_fs_guess2:
  // within a few dozen floats of the exact start, where the double totals can be ~1000 quanta
  // off), rebuilds its records and walks again from that guess, recording its window entries.
  // Then the exact values are handed from rank to rank (RCCL send/recv of 9 floats): rank r
  // repairs its walk from rank r - 1's end values (k_fs_repair: walked again only until it meets
  // the recorded walk -- after the rebase a few windows) and passes its exact end on; the last
  // rank's sums are broadcast.  protocol 1 (round 4, A/B only): no rebase, the first walk records
  // and the repairs start ~1000 quanta off.  protocol 2 (A/B only): parallel repair iterations
  // with a host check instead of the hand-over chain (below).
  hipLaunchKernelGGL(k_fs_prep, dim3(gp), dim3(kFpBS), 0, s, d, nullptr, b.tot);
  comm->allgather(b.tot, b.gath, kFsChains + 1, DType::F64, s);
  hipLaunchKernelGGL(k_fs_base, dim3(1), dim3(256), 0, s, d, b.gath, r, W, b.base9, b.n_global,
                     (const float*)nullptr, (const float*)nullptr);
  hipLaunchKernelGGL(k_fs_inc, dim3(gp), dim3(kFiBS), 0, s, d, b.base9);
  hipLaunchKernelGGL(k_fs_l1, dim3(gl), dim3(kFlBS), 0, s, d);
  FsDev dw = d;  // the launch the recorded walk (and its window tables) belongs to
  if (protocol == 1) {
    DLG_LAUNCH_EV(k_fs_walk, dim3(gw), dim3(kFwBS), 0, s, ev_walk0, ev_walk1, d,
                          (const float*)nullptr, r > 0 ? kFwGuess | kFwRecord : 0,
                          (const float4*)nullptr, (float4*)nullptr, (int32_t*)nullptr);
  } else {
    DLG_LAUNCH_EV(k_fs_walk, dim3(gw), dim3(kFwBS), 0, s, ev_walk0,
                          r > 0 ? ev_mid0 : ev_walk1, d, (const float*)nullptr,
                          r > 0 ? kFwGuess : 0, (const float4*)nullptr, (float4*)nullptr,
                          (int32_t*)nullptr);
    comm->allgather(b.sums, b.gath2, 2 * kFsChains, DType::I32, s);
    if (r > 0) {
      // the rebase: the records again, from the base moved to the propagated guess (new stamp:
      // the first walk's window tables are stale), and the walk from that guess
      uint32_t gen2 = ++s_gen;
      if (gen2 == 0) gen2 = ++s_gen;
      dw.gen = gen2;
      hipLaunchKernelGGL(k_fs_guess2, dim3(1), dim3(kWave), 0, s, b.gath2, r, b.g2);
      hipLaunchKernelGGL(k_fs_prep, dim3(gp), dim3(kFpBS), 0, s, dw, nullptr, b.tot);
      hipLaunchKernelGGL(k_fs_base, dim3(1), dim3(256), 0, s, dw, b.gath, r, W, b.base9,
                         b.n_global, (const float*)b.gath2, (const float*)b.g2);
      hipLaunchKernelGGL(k_fs_inc, dim3(gp), dim3(kFiBS), 0, s, dw, b.base9);
      hipLaunchKernelGGL(k_fs_l1, dim3(gl), dim3(kFlBS), 0, s, dw);
      DLG_LAUNCH_EV(k_fs_walk, dim3(gw), dim3(kFwBS), 0, s, ev_mid1, ev_walk1, dw,
                            (const float*)b.g2, kFwRecord, (const float4*)nullptr,
                            (float4*)nullptr, (int32_t*)nullptr);
    }
  }
  if (protocol == 2) {
    // every rank's (end, start): when each rank's start equals the end of the rank before (rank
    // 0 starts exactly), every walk was exact and the last rank's end is the sum.  Otherwise
    // each rank repairs its walk from the guess the pairs now propagate, at once (k_fs_repair
    // from k_fs_guess2's value: the exact start wherever the rank before was exact, so every
    // iteration extends the exact prefix of ranks by at least one), and checks again.  (A host
    // check per iteration: one stream sync each.  Measured at C4 on 8 loopback ranks: ~5
    // iterations a round -- chains crossing a binade inside a shard leave the propagated guess
    // 5-40 floats off.)
    if (ev_rep0) HIPCHK_FS(hipEventRecord(ev_rep0, s));
    std::vector<uint32_t> h((size_t)2 * kFsChains * W);
    for (int it = 0;; ++it) {
      comm->allgather(b.sums, b.gath2, 2 * kFsChains, DType::I32, s);
      HIPCHK_FS(hipMemcpyAsync(h.data(), b.gath2, 4 * h.size(), hipMemcpyDeviceToHost, s));
      comm->sync_stream(s);
      bool exact = true;
      for (int q = 1; q < W && exact; ++q)
        for (int c = 0; c < kFsChains; ++c)
          if (h[(size_t)(2 * q + 1) * kFsChains + c] != h[(size_t)2 * (q - 1) * kFsChains + c]) {
            exact = false;
            break;
          }
      if (exact) {
        if (repairs) *repairs = it;
        break;
      }
      if (it >= W - 1) throw std::logic_error("PCL refit: rank walks did not converge");
      if (r > 0) {
        hipLaunchKernelGGL(k_fs_guess2, dim3(1), dim3(kWave), 0, s, b.gath2, r, b.g2);
        hipLaunchKernelGGL(k_fs_repair, dim3(kFsChains), dim3(kFwBS), 0, s, dw,
                           (const float*)b.g2);
      }
    }
    if (ev_rep1) HIPCHK_FS(hipEventRecord(ev_rep1, s));
    HIPCHK_FS(hipMemcpyAsync(b.sums, b.gath2 + (size_t)2 * kFsChains * (W - 1),
                             sizeof(float) * kFsChains, hipMemcpyDeviceToDevice, s));
    hipLaunchKernelGGL(k_fs_tail, dim3(1), dim3(1), 0, s, b.sums, b.n_global, cin, cout, res);
    return;
  }
  if (r > 0) {
    comm->recv(b.start9, kFsChains, DType::I32, r - 1, s);
    DLG_LAUNCH_EV(k_fs_repair, dim3(kFsChains), dim3(kFwBS), 0, s, ev_rep0, ev_rep1,
                          dw, (const float*)b.start9);
  }
  if (r < W - 1) comm->send(b.sums, kFsChains, DType::I32, r + 1, s);
  comm->broadcast(b.sums, kFsChains, DType::I32, W - 1, s);
  hipLaunchKernelGGL(k_fs_tail, dim3(1), dim3(1), 0, s, b.sums, b.n_global, cin, cout, res);
  if (repairs) *repairs = W - 1;
}

}  // namespace dlg
