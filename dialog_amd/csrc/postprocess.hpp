// postprocess.hpp -- postProcessPlanes kernels (postprocess.hip): leftover absorption by the
// point-in-polygon test and clusterFilt's connected components.  Driven by postprocess_host.cpp.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

#include "normals.hpp"
#include "pp_math.hpp"

namespace dlg {

// one workgroup of the point-in-polygon test: candidates [cbeg, cbeg + ccnt) (<= 256) of one
// plane against its border edges [ebeg, eend)
struct PipTask {
  int32_t plane;
  int32_t cbeg;
  int32_t ccnt;
  int32_t ebeg;
  int32_t eend;
};

// candidates of plane p: unprocessed points whose distance to their projection on plane p is
// <= t_dist, grouped by plane in ascending point order.  Pass 1 (cand == nullptr): per-block
// counts bcnt[P x pip_blocks(n)], their exclusive scan boff (hipCUB, tmp >= pip_scan_tmp_bytes),
// offs[P + 1] = plane ranges; pass 2 writes cand[offs[p] ...].
int pip_blocks(int n);
size_t pip_scan_tmp_bytes(size_t count);
hipError_t launch_pip_candidates(const float* X, const float* Y, const float* Z, int n,
                                 const uint8_t* processed, const float4* planes, int n_planes,
                                 float t_dist, uint32_t* bcnt, uint32_t* boff, void* tmp,
                                 size_t tmp_bytes, int32_t* cand, uint32_t* offs, hipStream_t s);
// candidates of each plane reordered by the points' 3-D Morton code (lo_scale: bbox minimum and
// 16383 / extent); cand_out = the permuted list (same plane ranges)
size_t pip_sort_tmp_bytes(int count);
hipError_t launch_pip_sort(const int32_t* cand, int count, const uint32_t* offs, int n_planes,
                           int max_count, const float* X, const float* Y, const float* Z,
                           float4 lo_scale, uint64_t* keys, uint64_t* keys_alt, int32_t* cand_out,
                           void* tmp, size_t tmp_bytes, hipStream_t s);
// rays[p * kPipRays + k] = ray direction k of plane p (normalize(edge dir x plane normal))
// mask[c] ^= parity bit k of candidate c's crossings with the task's edges
void launch_pip_test(const PipTask* tasks, int n_tasks, const int32_t* cand, const float* X,
                     const float* Y, const float* Z, const float4* planes, const float4* rays,
                     const PipEdge* edges, const int64_t* edge_off, uint32_t* mask, hipStream_t s);
// inside <=> at least 5 of the 10 rays cross the border an odd number of times:
// absorbed[p * n + point] = 1, processed[point] = 1, abs_cnt[p] += 1
void launch_pip_mark(const int32_t* cand, const uint32_t* mask, const uint32_t* offs,
                     int n_planes, int max_count, int n, uint8_t* absorbed, uint8_t* processed,
                     uint32_t* abs_cnt, hipStream_t s);
// exact-coordinate table of the cloud (open addressing, -1 = empty; equal points -> lowest
// index) and the lookup of plane points in it: nn[q] for the hits, the misses (and queries
// with a coordinate of magnitude < 2^-50) go to rest[] for the grid search
void launch_xyz_insert(const float* X, const float* Y, const float* Z, int n, int32_t* table,
                       uint32_t tmask, hipStream_t s);
void launch_xyz_lookup(const float* qx, const float* qy, const float* qz, int m,
                       const int32_t* table, uint32_t tmask, const float* X, const float* Y,
                       const float* Z, int32_t* nn, int32_t* rest, uint32_t* n_rest,
                       hipStream_t s);
// processed[nn[j]] = 1
void launch_mark_nn(const int32_t* nn, int m, uint8_t* processed, hipStream_t s);
// flags[i] = !processed[i]
void launch_invert_flags(const uint8_t* processed, int n, uint8_t* flags, hipStream_t s);
// out[i] = map[sel[i]]
void launch_gather_ids(const int32_t* sel, int n, const int32_t* map, int32_t* out, hipStream_t s);

// clusterFilt: connected components of the radius graph (union-find over sorted positions);
// keep[point] = component size > t_cluster_num (compared as size_t, like the reference)
void launch_cc(const GridDesc& G, const GridBufs& B, int n, float r2, int64_t t_cluster_num,
               int32_t* parent, uint32_t* size, uint8_t* keep, hipStream_t s);

}  // namespace dlg
