// spatial.hpp -- spatially ordered copy of a cloud's active points and the pruned scoring kernel.
//
// countWithinDistance (SampleConsensusModelPlane, PCL 1.8 [SURVEY.md §8(a) a9]) only needs the
// number of inliers per hypothesis, which does not depend on the order the points are visited.
// The cloud's finite active points are therefore also kept in Morton order (10 bits per axis),
// cut into tiles of 32 consecutive points and super-tiles of 32 tiles, each with a bounding
// sphere.  A plane whose computed distance to a sphere's centre exceeds
//     cthr + radius + 2 e_max          (e_max = 64 u S_max >= every rounding error involved)
// cannot have a single PCL inlier in that sphere, so its tests there are decided without being
// evaluated; every other (tile, plane) pair is scored exactly as k_score_bf16 scores it (bf16
// matrix cores + exact re-decision inside the rounding band).  Counts stay bit-identical to the
// exhaustive kernels.
//
// The list-ordered SoA of kernels.hpp stays the source of truth for sampling positions, select
// and the inlier lists; the spatial copy is compacted with the same refined-plane predicate in
// every extract round, so it always holds exactly the finite active points.
#pragma once

#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>

#include "kernels.hpp"

namespace dlg {

constexpr int kTileP = 32;       // points per tile (the 32 rows of one MFMA block)
constexpr int kSuperTiles = 16;  // tiles per super-tile (a power of two <= 32)
constexpr int kSuperP = kTileP * kSuperTiles;

inline int64_t sp_tiles(int64_t n) { return (n + kTileP - 1) / kTileP; }
inline int64_t sp_supers(int64_t n) { return (n + kSuperP - 1) / kSuperP; }

struct SpatialView {
  const float* x;
  const float* y;
  const float* z;
  int64_t n;
  const float4* tiles;   // [sp_tiles(n)]  (cx, cy, cz, r): every point of the tile within r of c
  const float4* supers;  // [sp_supers(n)]
};

// the pruning test: may the sphere sp = (c, r) hold a point that passes PCL's test for the plane
// cf?  No when fl(|n.c + d|) > (margin + r)(1 + 2^-20) (module comment).  NaN planes: never near.
__device__ __forceinline__ float prune_lim(float margin, float r) {
  return (margin + r) * (1.0f + 0x1p-20f);
}
__device__ __forceinline__ bool sphere_near(float4 cf, float4 sp, float margin) {
  const float h = __builtin_fmaf(cf.x, sp.x, __builtin_fmaf(cf.y, sp.y, __builtin_fmaf(cf.z, sp.z, cf.w)));
  return fabsf(h) <= prune_lim(margin, sp.w);
}

// Curve keys over [-amax, amax] per axis, 10 bits per axis: Hilbert (hilbert, the default) or
// Morton; non-finite points get key 0xFFFFFFFF (sorted last) and are counted into *n_nonfinite
// (never inliers of any plane: PCL's distance is NaN or inf); aos[i] = (x, y, z, 0) of point i
void launch_morton_keys(PointsView src, float ax, float ay, float az, uint32_t* keys,
                        int32_t* idx, int32_t* n_nonfinite, float4* aos, hipStream_t s,
                        bool hilbert = true);
size_t morton_sort_temp_bytes(int64_t n);
hipError_t morton_sort(void* tmp, size_t tmp_bytes, uint32_t* keys_in, uint32_t* keys_out,
                       int32_t* idx_in, int32_t* idx_out, int64_t n, hipStream_t s);
// dst[i] = src[order[i]] (x, y, z; gid = order[i]), i < n
void launch_gather_order(const float4* src, const int32_t* order, int64_t n, PointsOut dst,
                         hipStream_t s);
// tile and super-tile bounding spheres of n points; with n_dev the count is read on the device
// (*n_dev <= n, the grid is sized for n)
void launch_sphere_bounds(const float* x, const float* y, const float* z, int64_t n,
                          const int32_t* n_dev, float4* tiles, float4* supers, hipStream_t s);
// margin = smallest float >= (cthr + 2 e_max)(1 + 2^-19), e_max = 64 u 2.0001 (ax + ay + az)
float prune_margin(float cthr, const float amax[3]);
// pruned countWithinDistance of D plane hypotheses over the spatial points (k_prune_supers +
// k_score_tiles_rl); counts[D] zeroed by the caller; lp / lp_n: scratch of sp_supers(n) *
// prune_list_stride(D) uint16 and sp_supers(n) + 1 int32 (per super-tile plane lists).
// amax: the cloud's per-axis max |coordinate| (the scoring band's S bound).
// list stride per super-tile (D rounded up to 64 entries: dword-aligned entry pairs)
inline int prune_list_stride(int D) { return (D + 63) / 64 * 64; }
// the plane model's (tile, plane) scorer: exact PCL-order evaluation with lanes as planes
// (k_score_tiles_ex, default) or 32 x 32 bf16 matrix-core blocks with band re-decision
// (k_score_tiles_rl); identical counts
constexpr int kTileScorerExact = 0;   // k_score_tiles_ex<2> (default)
constexpr int kTileScorerBf16 = 1;    // k_score_tiles_rl
constexpr int kTileScorerMfma = 2;    // k_score_tiles_ex<2, MF>: 16-plane groups on f32 MFMA
constexpr int kTileScorerMfmaX = 18;  // A/B check: the same, every result re-decided exactly
constexpr int kTileScorerMfmaW = 19;  // A/B check: the same with a band of 64 u S
// A/B-only variants (same counts; tests/test_score_variants.py runs each)
constexpr int kTileScorerExK1 = 11, kTileScorerExK4 = 14;
constexpr int kTileScorerExPk = 12;
constexpr int kTileScorerClaimR4 = 15, kTileScorerClaimClass = 16, kTileScorerClaimTail = 17;  // A/B
// the pruned scorer's int32 buffer: a fixed header of kPwHeader words -- the item counters (one
// per XCD, each on its own 128-byte line, kPruneWorkStride words apart), per XCD the counts of its
// super-tiles in each of kPwBuckets list-length classes (k_prune_supers appends them,
// k_score_tiles_ex's last workgroup zeroes them again) and that workgroup's ticket -- then the
// sp_supers(n) list lengths (the launches' lp_n points there), then per XCD and class the
// super-tiles (claimed longest-list class first)
constexpr int kPruneWorkStride = 32, kPwBuckets = 8;
constexpr int kPwBucket = 8 * kPruneWorkStride, kPwTicket = 16 * kPruneWorkStride;
constexpr int kPwHeader = 17 * kPruneWorkStride;
// list-length class of a super-tile: 0 (>= 2048 near planes) .. 7 (< 128)
__host__ __device__ inline int pw_class(int cnt) {
  return cnt >= 2048 ? 0 : cnt >= 1024 ? 1 : cnt >= 768 ? 2 : cnt >= 512 ? 3 : cnt >= 384 ? 4
       : cnt >= 256 ? 5 : cnt >= 128 ? 6 : 7;
}
inline int64_t prune_work_words(int64_t ns) {
  return kPwHeader + ns + (int64_t)kPwBuckets * 8 * ((ns + 7) / 8);
}
// SACMODEL_NORMAL_PLANE scoring over the spatial copy: its (normalised normal, curvature) per
// point, and the model's lambda / threshold; margin then comes from prune_margin(lim_max, amax)
struct PrunedNp {
  const float4* nrm;
  double lambda, thr;
  float4* cn = nullptr;  // [D] scratch: the hypotheses' normalized (a, b, c) (k_prune_supers)
};
void launch_score_pruned(const SpatialView& v, const HypRec* hyps, int D, float cthr, float margin,
                         const float amax[3], int32_t* counts, uint16_t* lp, int32_t* lp_n,
                         int num_cus, hipStream_t s,
                         unsigned long long* stats = nullptr,  // [6] counters (A/B tool)
                         const PrunedNp* np = nullptr,
                         const PickArgs* pick = nullptr,  // fused speculative pick (one rank)
                         hipEvent_t ev_start = nullptr,   // timing events of the launch pair
                         hipEvent_t ev_stop = nullptr,
                         int tile_scorer = kTileScorerExact);
// the NORMAL_PLANE prefilter limit of the largest w (host restatement of np_de_limit): every
// point's d_euclid limit is <= this when 0 <= w < 1 for all points; +inf otherwise
float np_lim_max(double w_max, double thr);
// gather the pristine normals into the Morton-ordered copy: dst[i] = src[order[i]]
void launch_gather_nrm(const float4* src, const int32_t* order, int64_t n, float4* dst,
                       hipStream_t s);
// min / max of the curvature (.w) of n normals (NaN ignored) -> out2 (as ordered uint bits)
void launch_curv_range(const float4* nrm, int64_t n, uint32_t* out2, hipStream_t s);

}  // namespace dlg
