// dev_common.hpp -- device helpers shared by the scoring kernels (kernels.hip, spatial.hip):
// wave primitives, PCL's plane distance in Eigen SSE op order, and the exact 3-way bf16 split +
// sign-byte counting of the bf16 matrix-core scoring path (see k_score_bf16 in kernels.hip).
#pragma once

#include <hip/hip_runtime.h>

#include <hip/hip_ext.h>

#include <cstdint>

// A launch that carries timing events on its own dispatch (hipExtLaunchKernelGGL) only when one
// is asked for, else the plain launch.  (Round 6 suspected the extended dispatch of the ~5 us
// gaps in front of k_prune_supers, k_score_tiles_ex, k_ustamp, k_fs_walk, k_fs_segfix and
// k_sel1_morton; the kernel trace with plain launches shows the same gaps: not the cause.)
#define DLG_LAUNCH_EV(kernel, grid, block, shmem, stream, ev0, ev1, ...)                      \
  do {                                                                                         \
    if ((ev0) != nullptr || (ev1) != nullptr)                                                  \
      hipExtLaunchKernelGGL(kernel, grid, block, shmem, stream, ev0, ev1, 0u, __VA_ARGS__);    \
    else                                                                                       \
      hipLaunchKernelGGL(kernel, grid, block, shmem, stream, __VA_ARGS__);                     \
  } while (0)

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


typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));

constexpr uint32_t kBf16One = 0x3F80u;

struct Split3 {
  uint32_t p1, p2, p3;  // bf16 bit patterns
};

__device__ __forceinline__ Split3 split3(float v) {
  const uint32_t u = __float_as_uint(v);
  const float v1 = __uint_as_float(u & 0xFFFF0000u);
  const float r1 = v - v1;  // exact (the low 16 significand bits)
  const uint32_t u2 = __float_as_uint(r1) & 0xFFFF0000u;
  const float r2 = r1 - __uint_as_float(u2);  // exact, <= 8 significant bits
  return Split3{u >> 16, u2 >> 16, __float_as_uint(r2) >> 16};
}

__device__ __forceinline__ uint32_t pk(uint32_t lo, uint32_t hi) { return lo | (hi << 16); }

__device__ __forceinline__ bf16x8 as_bf16x8(u32x4 v) { return __builtin_bit_cast(bf16x8, v); }

// sign bytes of r0..r3 (0xFF if negative) -> acc += 255 * #negative
__device__ __forceinline__ uint32_t count4(float r0, float r1, float r2, float r3, uint32_t acc) {
  // v_perm_b32 selectors: 9 = sign(S1) x 8, 11 = sign(S0) x 8, 12 = 0x00
  const uint32_t lo = __builtin_amdgcn_perm(__float_as_uint(r0), __float_as_uint(r1), 0x0C0C0B09u);
  const uint32_t hi = __builtin_amdgcn_perm(__float_as_uint(r2), __float_as_uint(r3), 0x0B090C0Cu);
  return __builtin_amdgcn_sad_u8(lo, hi, acc);
}

__device__ __forceinline__ float min3_abs(float m, float a, float b) {
  float o;
  asm("v_min3_f32 %0, %1, |%2|, |%3|" : "=v"(o) : "v"(m), "v"(a), "v"(b));
  return o;
}

}  // namespace
}  // namespace dlg
