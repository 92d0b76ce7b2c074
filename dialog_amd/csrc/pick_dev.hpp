// pick_dev.hpp -- RandomSampleConsensus::computeModel's decision over one batch of draws when
// the probability is 1 (log(1 - p) = -inf, so k = +inf and only the iteration cap ends the loop;
// PCL 1.8 ransac.hpp computeModel): the loop ends at the need_good-th good draw (need_good =
// max_iterations + 1) and keeps the first good draw with the largest count (strict '>').  A bad
// draw only consumes a getSamples try; with fewer than 1000 bad draws in the batch no run of
// 1000 can end the loop early.  out[0] = batch index of the best draw (-1: none), out[1] = 1 if
// the loop ended inside the batch.  The winner's HypRec and samples are copied to best /
// best_smp.  Speculative: the host replays the same counts (RansacControl::consume) after the
// round's sync and redoes the round on any disagreement.
//
// One workgroup of NT threads runs it: k_pick_p1, or the last workgroup of the pruned scoring
// launch (COH: the counts were summed by this launch's atomics, so they are read with
// device-coherent loads).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

#include "dev_common.hpp"
#include "kernels.hpp"

namespace dlg {

template <bool COH>
__device__ __forceinline__ int32_t pick_count(const int32_t* p) {
  if constexpr (COH) return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  else return *p;
}

template <int NT, bool COH>
__device__ __forceinline__ void pick_body(const PickArgs& a) {
  constexpr int kW = NT / kWave;
  __shared__ int s_good[kW], s_bad[kW];
  __shared__ unsigned long long s_key[kW];
  __shared__ int s_end;
  const int32_t* __restrict__ res = a.res;
  const int Dp = a.Dp, D = a.D, need_good = a.need_good;
  const int t = threadIdx.x, lane = t & (kWave - 1), w = t / kWave;
  // (D <= kMaxHypPerLaunch: at most kPer draws per thread, their flags and counts loaded
  // together up front -- the fused pick's coherent loads would otherwise wait out one by one)
  constexpr int kPer = (kMaxHypPerLaunch + NT - 1) / NT;
  const int per = (D + NT - 1) / NT;
  const int d0 = min(D, t * per), d1 = min(D, d0 + per);
  int gf[kPer], cnt[kPer];
#pragma unroll
  for (int i = 0; i < kPer; ++i) gf[i] = d0 + i < d1 ? res[Dp + d0 + i] : 0;
#pragma unroll
  for (int i = 0; i < kPer; ++i) cnt[i] = d0 + i < d1 ? pick_count<COH>(res + d0 + i) : 0;
  int g = 0, b = 0;
#pragma unroll
  for (int i = 0; i < kPer; ++i) {
    if (d0 + i < d1) {
      if (gf[i]) ++g; else ++b;
    }
  }
  // block exclusive scan of the good counts (wave scans + wave totals)
  int incl = g;
#pragma unroll
  for (int o = 1; o < kWave; o <<= 1) {
    const int v = __shfl_up(incl, o);
    if (lane >= o) incl += v;
  }
  int bt = b;
#pragma unroll
  for (int o = 1; o < kWave; o <<= 1) bt += __shfl_xor(bt, o);
  if (lane == kWave - 1) s_good[w] = incl;
  if (lane == 0) s_bad[w] = bt;
  if (t == 0) s_end = -1;
  __syncthreads();
  int base = 0, total_good = 0, total_bad = 0;
  for (int q = 0; q < kW; ++q) {
    base += q < w ? s_good[q] : 0;
    total_good += s_good[q];
    total_bad += s_bad[q];
  }
  base += incl - g;
  // the draw at which the need_good-th good draw happens
  if (base < need_good && base + g >= need_good) {
    int c = base, e = -1;
#pragma unroll
    for (int i = 0; i < kPer; ++i)
      if (e < 0 && d0 + i < d1 && gf[i] && ++c == need_good) e = d0 + i;
    s_end = e;
  }
  __syncthreads();
  const int end = s_end;  // -1: the loop goes on past this batch
  // first maximum over the good draws up to the end: key = (count, ~index)
  unsigned long long key = 0ull;
#pragma unroll
  for (int i = 0; i < kPer; ++i) {
    const int d = d0 + i;
    if (d >= d1 || (end >= 0 && d > end) || !gf[i]) continue;
    const unsigned long long k = ((unsigned long long)(uint32_t)cnt[i] << 32) |
                                 (unsigned long long)(0xFFFFFFFFu - (uint32_t)d);
    key = k > key ? k : key;
  }
#pragma unroll
  for (int o = 1; o < kWave; o <<= 1) {
    const unsigned long long v = __shfl_xor(key, o);
    key = v > key ? v : key;
  }
  if (lane == 0) s_key[w] = key;
  __syncthreads();
  if (t == 0) {
    unsigned long long k = 0ull;
    for (int q = 0; q < kW; ++q) k = s_key[q] > k ? s_key[q] : k;
    const int bd = k ? (int)(0xFFFFFFFFu - (uint32_t)(k & 0xFFFFFFFFull)) : -1;
    a.out[0] = bd;
    a.out[1] = (end >= 0 && total_bad < 1000 && total_good >= need_good) ? 1 : 0;
    if (bd >= 0) {
      *a.best = a.hyps[bd];
      a.best_smp[0] = a.samples[3 * bd];
      a.best_smp[1] = a.samples[3 * bd + 1];
      a.best_smp[2] = a.samples[3 * bd + 2];
    }
  }
}

}  // namespace dlg
