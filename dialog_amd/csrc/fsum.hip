// fsum.hip -- PCL's float refit on the device (gfx950): the nine sequential float sums of
// computeMeanAndCovarianceMatrix, bit-exact, in parallel (algorithm and proof: fsum.hpp), then
// the float eigen33 of optimizeModelCoefficients.
//
// Kernels (stream order; the inlier count lives on the device, so every grid is fixed and the
// kernels loop over the work the count implies):
//   k_fs_prep   units of 4096 inliers: per-chunk double sums of the nine terms (the guesses),
//               per-unit sums; the last workgroup scans the units (double prefixes)
//   k_fs_run    (unit, chain) items: level-1 fan runs of the 64 chunks from their guesses (4
//               starts each, 256 lanes, elements staged in LDS), then the unit's level-2 record:
//               one wave per member walks the 64 chunk records (reruns from LDS)
//   k_fs_level  levels >= 3 (more than 128 nodes at level 2): one wave per member walks 64
//               children, descending through per-wave LDS windows of the lower levels
//   k_fs_top    one wave per chain walks the top level from +0 (descents as above); then the
//               refit (fs_refit_tail) by one thread: refined plane + uncertainty flag + sums
// Every wave executes its walk uniformly (all lanes the same values): the lanes are only used to
// load a 64-node window or a chunk's 64 elements at once.
#include "kernels.hpp"
#include "dev_common.hpp"
#include "fsum.hpp"

#include <cstdint>

namespace dlg {
namespace {

constexpr int kFsUnit = kFsChunk * kFsArity;  // 4096 inliers per level-2 node
constexpr int kFsTopMax = 128;                // the top walk's node count bound
constexpr int kFsPad = kFsChunk + 1;          // LDS row stride of a chunk (spreads the banks)
constexpr int kFsWinLevels = 3;               // LDS windows for levels 1..3 per wave

struct FsDev {
  const float* px;
  const float* py;
  const float* pz;
  int stride;
  const int32_t* n_dev;
  FsBuffers b;
};

__device__ __forceinline__ int fs_top_level(int64_t n) {
  int L = 1;
  while (fs_nodes(n, L) > kFsTopMax) ++L;
  return L;
}

__device__ __forceinline__ FsNode* fs_node_ptr(const FsBuffers& b, int L, int c, int64_t k) {
  return reinterpret_cast<FsNode*>(b.nodes[L]) + (int64_t)c * b.cap[L] + k;
}

__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// ---- k_fs_prep --------------------------------------------------------------------------------
constexpr int kFpBS = 256;
__global__ __launch_bounds__(kFpBS) void k_fs_prep(FsDev d) {
  __shared__ float sx[kFsArity * kFsPad], sy[kFsArity * kFsPad], sz[kFsArity * kFsPad];
  __shared__ double scs[kFsArity * kFsChains];
  const int64_t n = *d.n_dev;
  const int64_t U = (n + kFsUnit - 1) / kFsUnit;
  const int t = threadIdx.x;
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
    for (int p = t; p < nch * kFsChains; p += kFpBS) {
      const int k = p / kFsChains, c = p % kFsChains;
      const int len = cnt - k * kFsChunk < kFsChunk ? cnt - k * kFsChunk : kFsChunk;
      double s = 0.0;
      for (int j = 0; j < len; ++j) {
        const int li = k * kFsPad + j;
        s += (double)fs_term(c, sx[li], sy[li], sz[li]);
      }
      scs[p] = s;
      d.b.csum[(u * kFsArity + k) * kFsChains + c] = s;
    }
    __syncthreads();
    if (t < kFsChains) {
      double s = 0.0;
      for (int k = 0; k < nch; ++k) s += scs[k * kFsChains + t];
      __hip_atomic_store(reinterpret_cast<int64_t*>(d.b.usum) + u * kFsChains + t,
                         __double_as_longlong(s), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  // the last workgroup scans the unit sums (agent-scope stores acknowledged before the ticket,
  // read back with agent-scope loads: k_moments' pattern)
  __builtin_amdgcn_s_waitcnt(0);
  __shared__ unsigned s_ticket;
  __syncthreads();
  if (t == 0)
    s_ticket = __hip_atomic_fetch_add(d.b.ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __syncthreads();
  if (s_ticket != gridDim.x - 1) return;
  if (t == 0) *d.b.ticket = 0u;
  double* blk = scs;  // (reused: 64 units x 9 per block)
  double run = 0.0;
  for (int64_t ub = 0; ub < U; ub += kFsArity) {
    const int nb = (int)(U - ub < kFsArity ? U - ub : kFsArity);
    __syncthreads();
    for (int p = t; p < nb * kFsChains; p += kFpBS)
      blk[p] = __longlong_as_double(__hip_atomic_load(
          reinterpret_cast<const int64_t*>(d.b.usum) + ub * kFsChains + p, __ATOMIC_RELAXED,
          __HIP_MEMORY_SCOPE_AGENT));
    __syncthreads();
    if (t < kFsChains) {
      for (int q = 0; q < nb; ++q) {
        d.b.upre[(ub + q) * kFsChains + t] = run;
        run += blk[q * kFsChains + t];
      }
    }
  }
}

// ---- k_fs_run ---------------------------------------------------------------------------------
// the level-2 walk's store: the unit's chunk records and elements in LDS
struct FsUnitStore {
  const FsNode* sn;
  int64_t k0, K;
  const float *sx, *sy, *sz;
  int c, cnt;
  __device__ const FsNode& node(int, int64_t k) { return sn[k - k0]; }
  __device__ int64_t nodes(int) const { return K; }
  __device__ FsRun rerun(int64_t k, float v) {
    const int kk = (int)(k - k0);
    const int len = cnt - kk * kFsChunk < kFsChunk ? cnt - kk * kFsChunk : kFsChunk;
    FsState st = fs_start(v);
    for (int j = 0; j < len; ++j) {
      const int li = kk * kFsPad + j;
      fs_step(st, fs_term(c, sx[li], sy[li], sz[li]));
    }
    return fs_finish(st);
  }
};

constexpr int kFrBS = kFsArity * kFsFan;  // 64 chunks x 4 members
__global__ __launch_bounds__(kFrBS) void k_fs_run(FsDev d) {
  __shared__ float sx[kFsArity * kFsPad], sy[kFsArity * kFsPad], sz[kFsArity * kFsPad];
  __shared__ FsNode sn[kFsArity];
  __shared__ float sg[kFsArity];
  __shared__ double s_cs[kFsArity];
  const int64_t n = *d.n_dev;
  const int64_t U = (n + kFsUnit - 1) / kFsUnit, K = fs_nodes(n, 1);
  const int t = threadIdx.x, lane = t & (kWave - 1), wv = t / kWave;
  for (int64_t it = blockIdx.x; it < U * kFsChains; it += gridDim.x) {
    const int64_t u = it / kFsChains;
    const int c = (int)(it % kFsChains);
    const int64_t e0 = u * kFsUnit;
    const int cnt = (int)(n - e0 < kFsUnit ? n - e0 : kFsUnit);
    const int nch = (cnt + kFsChunk - 1) / kFsChunk;
    __syncthreads();
    for (int j = t; j < cnt; j += kFrBS) {
      const int64_t e = (e0 + j) * d.stride;
      const int li = (j >> 6) * kFsPad + (j & 63);
      sx[li] = d.px[e]; sy[li] = d.py[e]; sz[li] = d.pz[e];
    }
    if (t < nch) s_cs[t] = d.b.csum[(u * kFsArity + t) * kFsChains + c];
    __syncthreads();
    if (t < nch) {
      // the guess at chunk t: fl(double prefix of the terms), unit prefix + chunks before it
      double pre = d.b.upre[u * kFsChains + c];
      for (int k = 0; k < t; ++k) pre += s_cs[k];
      sg[t] = (float)pre;
    }
    __syncthreads();
    {  // level 1: lane (chunk k, member i) runs the chunk from g_k + i q(g_k)
      const int k = t >> 2, i = t & 3;
      if (k < nch) {
        const float g = sg[k];
        float a;
        const bool ok = fs_member_start(g, i, &a);
        const int len = cnt - k * kFsChunk < kFsChunk ? cnt - k * kFsChunk : kFsChunk;
        FsState st = fs_start(a);
        for (int j = 0; j < len; ++j) {
          const int li = k * kFsPad + j;
          fs_step(st, fs_term(c, sx[li], sy[li], sz[li]));
        }
        const FsRun r = fs_finish(st);
        sn[k].o[i] = ok ? r.o : 0.0f;
        sn[k].mu[i] = ok ? r.mu : 0.0f;
        sn[k].qm[i] = ok ? r.qm : __builtin_nanf("");
        if (i == 0) {
          sn[k].g = g;
          sn[k].pad0 = sn[k].pad1 = sn[k].pad2 = 0.0f;
        }
      }
    }
    __syncthreads();
    // level-1 records out (the top walk's descents read them)
    for (int p = t; p < nch * 4; p += kFrBS) {
      const float4* src = reinterpret_cast<const float4*>(&sn[p >> 2]) + (p & 3);
      reinterpret_cast<float4*>(fs_node_ptr(d.b, 1, c, u * kFsArity + (p >> 2)))[p & 3] = *src;
    }
    {  // level 2: wave wv walks member wv of the unit through the chunk records
      float a;
      const bool ok = fs_member_start(sg[0], wv, &a);
      FsUnitStore st{sn, u * kFsArity, K, sx, sy, sz, c, cnt};
      float mu = INFINITY, qm = 0.0f, o = 0.0f;
      if (ok) o = fs_walk(st, 1, u * kFsArity, nch, a, &mu, &qm, nullptr);
      if (lane == 0) {
        FsNode* nd = fs_node_ptr(d.b, 2, c, u);
        nd->o[wv] = ok ? o : 0.0f;
        nd->mu[wv] = ok ? mu : 0.0f;
        nd->qm[wv] = ok ? qm : __builtin_nanf("");
        if (wv == 0) {
          nd->g = sg[0];
          nd->pad0 = nd->pad1 = nd->pad2 = 0.0f;
        }
      }
    }
  }
}

// ---- walks over the global records ---------------------------------------------------------
// per-wave LDS windows of 64 nodes for levels 1..kFsWinLevels; higher levels through a one-node
// slot.  Reruns keep the chunk's elements in the lanes' registers (one element per lane) and step
// through them with readlane.
struct FsGlobalStore {
  const FsDev* d;
  int c;
  int64_t n;
  FsNode* win;      // [kFsWinLevels][64] (LDS, this wave's)
  FsNode* slot;     // one node (LDS, this wave's)
  int64_t base[kFsWinLevels + 1];
  int64_t cnt[kFsMaxLevels + 1];
  __device__ void init(const FsDev* dd, int cc, int64_t nn, FsNode* w, FsNode* s) {
    d = dd; c = cc; n = nn; win = w; slot = s;
    for (int l = 0; l <= kFsWinLevels; ++l) base[l] = -1;
    for (int l = 1; l <= kFsMaxLevels; ++l) cnt[l] = fs_nodes(n, l);
  }
  __device__ int64_t nodes(int L) const { return cnt[L]; }
  __device__ const FsNode& node(int L, int64_t k) {
    const int lane = threadIdx.x & (kWave - 1);
    if (L <= kFsWinLevels) {
      const int64_t b = k & ~(int64_t)(kWave - 1);
      FsNode* w = win + (L - 1) * kWave;
      if (base[L] != b) {
        wave_sync();
        if (b + lane < cnt[L]) {
          const float4* src = reinterpret_cast<const float4*>(fs_node_ptr(d->b, L, c, b + lane));
          float4* dst = reinterpret_cast<float4*>(w + lane);
          const float4 v0 = src[0], v1 = src[1], v2 = src[2], v3 = src[3];
          dst[0] = v0; dst[1] = v1; dst[2] = v2; dst[3] = v3;
        }
        wave_sync();
        base[L] = b;
      }
      return w[k - b];
    }
    wave_sync();
    if (lane < 4)
      reinterpret_cast<float4*>(slot)[lane] =
          reinterpret_cast<const float4*>(fs_node_ptr(d->b, L, c, k))[lane];
    wave_sync();
    return *slot;
  }
  __device__ FsRun rerun(int64_t k, float v) {
    const int lane = threadIdx.x & (kWave - 1);
    const int64_t e = k * kFsChunk + lane;
    const int len = n - k * kFsChunk < kFsChunk ? (int)(n - k * kFsChunk) : kFsChunk;
    float x = 0.0f, y = 0.0f, z = 0.0f;
    if (lane < len) {
      x = d->px[e * d->stride]; y = d->py[e * d->stride]; z = d->pz[e * d->stride];
    }
    FsState st = fs_start(v);
    for (int j = 0; j < len; ++j) {
      const float xj = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(x), j));
      const float yj = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(y), j));
      const float zj = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(z), j));
      fs_step(st, fs_term(c, xj, yj, zj));
    }
    return fs_finish(st);
  }
};

// ---- k_fs_level: level l >= 3 records (only when level l - 1 has more than kFsTopMax nodes) --
constexpr int kFlBS = kWave * kFsFan;
template <int l>
__global__ __launch_bounds__(kFlBS) void k_fs_level(FsDev d) {
  __shared__ FsNode s_win[kFsFan][kFsWinLevels * kWave];
  __shared__ FsNode s_slot[kFsFan];
  const int64_t n = *d.n_dev;
  if (fs_top_level(n) < l) return;
  const int64_t M = fs_nodes(n, l), Mc = fs_nodes(n, l - 1);
  const int wv = threadIdx.x / kWave, lane = threadIdx.x & (kWave - 1);
  for (int64_t it = blockIdx.x; it < M * kFsChains; it += gridDim.x) {
    const int64_t k = it / kFsChains;
    const int c = (int)(it % kFsChains);
    const int64_t c0 = k * kFsArity;
    const int64_t cc = Mc - c0 < kFsArity ? Mc - c0 : kFsArity;
    FsGlobalStore st;
    st.init(&d, c, n, s_win[wv], &s_slot[wv]);
    const float g = st.node(l - 1, c0).g;  // (the guess at the node's first element)
    float a;
    const bool ok = fs_member_start(g, wv, &a);
    float mu = INFINITY, qm = 0.0f, o = 0.0f;
    if (ok) o = fs_walk(st, l - 1, c0, cc, a, &mu, &qm, nullptr);
    if (lane == 0) {
      FsNode* nd = fs_node_ptr(d.b, l, c, k);
      nd->o[wv] = ok ? o : 0.0f;
      nd->mu[wv] = ok ? mu : 0.0f;
      nd->qm[wv] = ok ? qm : __builtin_nanf("");
      if (wv == 0) {
        nd->g = g;
        nd->pad0 = nd->pad1 = nd->pad2 = 0.0f;
      }
    }
    wave_sync();
  }
}

// ---- k_fs_top: the chains' values, then the refit ----------------------------------------------
constexpr int kFtBS = kWave * kFsChains;
__global__ __launch_bounds__(kFtBS) void k_fs_top(FsDev d, const float4* __restrict__ cin,
                                                  float4* __restrict__ cout,
                                                  int32_t* __restrict__ res) {
  __shared__ FsNode s_win[kFsChains][kFsWinLevels * kWave];
  __shared__ FsNode s_slot[kFsChains];
  __shared__ float s_sum[kFsChains];
  const int64_t n = *d.n_dev;
  const int c = threadIdx.x / kWave, lane = threadIdx.x & (kWave - 1);
  {
    FsGlobalStore st;
    st.init(&d, c, n, s_win[c], &s_slot[c]);
    const int L = fs_top_level(n);
    float mu = INFINITY, qm = 0.0f;
    const float v = fs_walk(st, L, 0, st.nodes(L), 0.0f, &mu, &qm, nullptr);
    if (lane == 0) s_sum[c] = v;
  }
  __syncthreads();
  if (threadIdx.x != 0) return;
  const float4 ci = *cin;
  const float cv[4] = {ci.x, ci.y, ci.z, ci.w};
  float a[9], co[4];
  for (int k = 0; k < 9; ++k) a[k] = s_sum[k];
  bool unc = false;
  fs_refit_tail(a, n, cv, co, &unc);
  *cout = make_float4(co[0], co[1], co[2], co[3]);
  res[0] = unc ? 1 : 0;
  res[1] = (int32_t)n;
  for (int k = 0; k < 9; ++k) res[2 + k] = __float_as_int(a[k]);
}

int fs_levels_host(int64_t n) {
  int L = 1;
  while (fs_nodes(n, L) > kFsTopMax) ++L;
  return L < 2 ? 2 : L;  // (k_fs_run always writes level 2)
}

size_t align256(size_t b) { return (b + 255) & ~(size_t)255; }

}  // namespace

size_t fs_scratch_bytes(int64_t n_cap) {
  const int64_t nc = n_cap > 0 ? n_cap : 1;
  const int64_t K = fs_nodes(nc, 1), U = fs_nodes(nc, 2);
  size_t b = align256(sizeof(double) * K * kFsChains) + 2 * align256(sizeof(double) * U * kFsChains);
  const int L = fs_levels_host(nc);
  for (int l = 1; l <= L; ++l) b += align256(sizeof(FsNode) * fs_nodes(nc, l) * kFsChains);
  return b + 256;
}

FsBuffers fs_carve(void* base, int64_t n_cap) {
  const int64_t nc = n_cap > 0 ? n_cap : 1;
  const int64_t K = fs_nodes(nc, 1), U = fs_nodes(nc, 2);
  uint8_t* p = static_cast<uint8_t*>(base);
  FsBuffers b;
  b.csum = reinterpret_cast<double*>(p);
  p += align256(sizeof(double) * K * kFsChains);
  b.usum = reinterpret_cast<double*>(p);
  p += align256(sizeof(double) * U * kFsChains);
  b.upre = reinterpret_cast<double*>(p);
  p += align256(sizeof(double) * U * kFsChains);
  const int L = fs_levels_host(nc);
  for (int l = 1; l <= L; ++l) {
    b.nodes[l] = p;
    b.cap[l] = fs_nodes(nc, l);
    p += align256(sizeof(FsNode) * fs_nodes(nc, l) * kFsChains);
  }
  b.ticket = reinterpret_cast<unsigned*>(p);
  return b;
}

void launch_fs_refit(const float* px, const float* py, const float* pz, int stride,
                     const int32_t* n_dev, int64_t n_cap, const FsBuffers& b, const float4* cin,
                     float4* cout, int32_t* res, int num_cus, hipStream_t s) {
  FsDev d{px, py, pz, stride, n_dev, b};
  const int64_t nc = n_cap > 0 ? n_cap : 1;
  const int64_t U = fs_nodes(nc, 2);
  const int gp = (int)std::min<int64_t>(U, 2 * (int64_t)num_cus);
  const int gr = (int)std::min<int64_t>(U * kFsChains, 4 * (int64_t)num_cus);
  hipLaunchKernelGGL(k_fs_prep, dim3(gp), dim3(kFpBS), 0, s, d);
  hipLaunchKernelGGL(k_fs_run, dim3(gr), dim3(kFrBS), 0, s, d);
  const int L = fs_levels_host(nc);
  for (int l = 3; l <= L; ++l) {
    const int g = (int)std::min<int64_t>(fs_nodes(nc, l) * kFsChains, 4 * (int64_t)num_cus);
    switch (l) {
      case 3: hipLaunchKernelGGL(k_fs_level<3>, dim3(g), dim3(kFlBS), 0, s, d); break;
      case 4: hipLaunchKernelGGL(k_fs_level<4>, dim3(g), dim3(kFlBS), 0, s, d); break;
      case 5: hipLaunchKernelGGL(k_fs_level<5>, dim3(g), dim3(kFlBS), 0, s, d); break;
      default: break;  // (n < 2^31: at most 5 levels)
    }
  }
  hipLaunchKernelGGL(k_fs_top, dim3(1), dim3(kFtBS), 0, s, d, cin, cout, res);
}

}  // namespace dlg
