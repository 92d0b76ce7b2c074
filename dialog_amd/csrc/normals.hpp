// normals.hpp -- uniform-grid neighbour search, normal estimation and RegulateNormal BFS kernels
// (normals.hip), driven by normals_host.cpp.
#pragma once

#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>

namespace dlg {

// Uniform grid over the cloud's bounding box; cell edge >= the search radius so a radius query
// touches at most the 27 cells around its own.  Cell key = (cz * gy + cy) * gx + cx < ncells
// <= 2^30; key ncells marks a non-finite point (sorted last, never inserted).
struct GridDesc {
  float lo[3];
  float cell;
  float inv_cell;
  int g[3];
  uint32_t ncells;
  int key_bits;
};

// Device buffers of one grid (owned by the caller).  Sorted order: position t holds point
// idx_out[t] with coordinates (sx, sy, sz)[t]; the open-addressing cell table maps an occupied
// cell's key to its [begin, end) range of sorted positions.
struct GridBufs {
  uint32_t* keys_in = nullptr;
  uint32_t* keys_out = nullptr;
  int32_t* idx_in = nullptr;
  int32_t* idx_out = nullptr;
  float* sx = nullptr;
  float* sy = nullptr;
  float* sz = nullptr;
  uint32_t* tkeys = nullptr;
  int2* trange = nullptr;
  uint32_t tmask = 0;
  void* sort_tmp = nullptr;
  size_t sort_tmp_bytes = 0;
};

// bounding box of the finite points: per-block partial (min xyz, max xyz) -> out[6 * blocks]
int bbox_blocks(int n);
void launch_bbox(const float* X, const float* Y, const float* Z, int n, float* partial,
                 hipStream_t s);

size_t sort_tmp_bytes(int n, int key_bits);
// sort by cell, fill the cell table; n_occupied (device, 16 B): [0] = occupied cells,
// [2..3] = uint64 sum over cells of occupancy^2
// rec (optional, n records of scratch): the points are first packed as (x, y, z, 0) records so
// the sorted gather reads one 16-byte record per point instead of three scattered floats
hipError_t grid_build(const float* X, const float* Y, const float* Z, int n, const GridDesc& G,
                      GridBufs& B, uint32_t* n_occupied, hipStream_t s, float4* rec = nullptr);
// strided host-layout xyz records (uploaded raw) -> SoA
void launch_deinterleave(const float* raw, int n, int64_t stride_floats, float* X, float* Y,
                         float* Z, hipStream_t s);

// radius normals: out[i] = (nx, ny, nz, curvature) for original point i
void launch_normals_radius(const GridDesc& G, const GridBufs& B, int n, float r2, const float vp[3],
                           float4* normals, hipStream_t s);
// k nearest neighbours (k <= kMaxKnn) over a grid hierarchy, FLANN order (d2, index)
constexpr int kMaxKnn = 64;
constexpr int kMaxLevels = 12;
struct KnnLevels {
  int levels;
  GridDesc G[kMaxLevels];
  const float* sx[kMaxLevels];
  const float* sy[kMaxLevels];
  const float* sz[kMaxLevels];
  const int32_t* idx[kMaxLevels];
  const int32_t* pos_of[kMaxLevels];  // inverse of idx: point -> sorted position
  const uint32_t* tkeys[kMaxLevels];
  const int2* trange[kMaxLevels];
  uint32_t tmask[kMaxLevels];
};
// one level: queries qlist[0..nq) (nullptr at level 0: every point, level-0 order); queries with
// fewer than k neighbours inside the level's guaranteed radius are appended to next[]
// one level: queries = sorted positions qpos[0..nq) of level `level` (nullptr: all of them);
// a query with fewer than k neighbours inside the level's guaranteed radius sets
// defer_next[its sorted position at level + 1]
// pcl_float: PCL's single-pass float moments over the (d2, index)-ordered list + float eigen33
// (bit-exact with PCL's arithmetic as restated); else centred double moments + double eigen33
// defer: per-level flag arrays (level t at defer + t * defer_stride, indexed by point); a
// deferred query is flagged at level l + 1, or (from level 0) l + 2 when it saw fewer than k / 4
// candidates (surface-like density: the radius it needs is more than twice this level's), never
// above level lmax
void launch_normals_knn(const KnnLevels& L, int level, const int32_t* qpos, int nq,
                        const float* X, const float* Y, const float* Z, int k, const float vp[3],
                        float4* normals, uint8_t* defer, int64_t defer_stride, int lmax,
                        bool pcl_float, hipStream_t s, int tnext = -1);
// (tnext, levels > 0: the level a deferred query goes to; -1: the next one)
// PCL-float radius normals in chunks of queries (sorted positions [q0, q0 + nq)):
// counts -> exclusive scan (int64 offsets) -> (d2, index) keys filled, sorted per query (one
// wave per query: bitonic in registers up to 1024 keys, heapsort beyond) -> float sums in that
// order, eigen33<float>, curvature, viewpoint flip
void launch_nbr_count(const GridDesc& G, const GridBufs& B, int q0, int nq, float r2,
                      int32_t* cnt, hipStream_t s);
size_t nbr_scan_tmp_bytes(int nq);
hipError_t nbr_scan(void* tmp, size_t tmp_bytes, const int32_t* cnt, int64_t* off, int nq,
                    hipStream_t s);
void launch_nbr_fill_sort_normals(const GridDesc& G, const GridBufs& B, int q0, int nq, float r2,
                                  const int32_t* cnt, const int64_t* off, uint64_t* keys,
                                  const float* X, const float* Y, const float* Z, const float vp[3],
                                  float4* normals, int num_cus, hipStream_t s);
// the same radius normals in one fused pass (k_nbr_fused): all n queries (qlist null) or the
// *qcount sorted positions of qlist; wide = 0: up to 512 neighbours per query, 1: 1024; queries
// with more go to ovf (count *ovf_count)
void launch_nbr_fused(const GridDesc& G, const GridBufs& B, int n, const int32_t* qlist,
                      const uint32_t* qcount, int wide, float r2, const float vp[3],
                      float4* normals, int32_t* ovf, uint32_t* ovf_count, int num_cus,
                      hipStream_t s);
void launch_inverse_perm(const int32_t* idx, int n, int32_t* pos_of, hipStream_t s);
// out[u] = f[idx[u]] (point-indexed flags -> a level's sorted order)
void launch_gather_flags(const uint8_t* f, const int32_t* idx, int n, uint8_t* out, hipStream_t s);

// nearest neighbour (k = 1, ties -> lowest index) in the hierarchy's cloud of external queries
// (qx, qy, qz)[qlist or 0..nq); unresolved queries go to next[] for the level above
void launch_nn1(const KnnLevels& L, int level, const int32_t* qlist, int nq, const float* qx,
                const float* qy, const float* qz, int32_t* nn, int32_t* next, uint32_t* n_next,
                hipStream_t s);
// nrm[i] *= -1 when Vector3f(nrm[i]).dot(Vector3f(ref[nn[i]])) < 0 (strided records)
void launch_flip_to_reference(float* nrm, int64_t stride_f, const float* ref, int64_t ref_stride_f,
                              const int32_t* nn, int n, hipStream_t s);

// ---- preProcess (PlaneDetect.h:448-512) ----
void launch_finite_flags(const float* X, const float* Y, const float* Z, int n, uint8_t* flags,
                         hipStream_t s);
size_t select_tmp_bytes(int n);
// out = indices i (ascending) with flags[i] != 0; *n_out (device) = their number
hipError_t select_flagged(void* tmp, size_t tmp_bytes, const uint8_t* flags, int n, int32_t* out,
                          uint32_t* n_out, hipStream_t s);
void launch_gather3(const int32_t* src, int n, const float* X, const float* Y, const float* Z,
                    float* OX, float* OY, float* OZ, hipStream_t s);
// out[0..2] = sums3[0..2] / float(n) (sums3: fsum's x, y, z chain end values)
void launch_centroid_div(const float* sums3, int n, float* out, hipStream_t s);
void launch_translate(float* X, float* Y, float* Z, int n, const float* p, hipStream_t s);
// index-ordered maximal independent set of the radius graph, one round over the undecided
// sorted positions (qlist == nullptr: all); state: 0 undecided, 1 kept, 2 removed
void launch_mis_round(const int32_t* qlist, int nq, const GridDesc& G, const GridBufs& B, float r2,
                      uint8_t* state, int32_t* next, uint32_t* n_next, hipStream_t s);
void launch_mis_flags(const GridBufs& B, int n, const uint8_t* state, uint8_t* kept, hipStream_t s);
void launch_emit_points(const int32_t* sel, int n, const float* X, const float* Y, const float* Z,
                        const int32_t* src, float* out, int64_t stride_f, int32_t* out_idx,
                        hipStream_t s);

// ---- RegulateNormal, level-synchronous BFS (state in the grid's sorted order) ----
// queue[]: point ids in PCL queue order; the current level is queue[fbase, fbase + nf).
// claim_s: min over claiming queue positions (init ~0); cand: first-claimed positions.
void launch_bfs_prepare(const GridBufs& B, int n, const float4* nrm, float4* nrm_s, int32_t* pos_of,
                        hipStream_t s);
void launch_bfs_seed(int32_t seed, int flip, const int32_t* pos_of, float4* nrm_s,
                     uint8_t* processed_s, int32_t* queue, hipStream_t s);
// one BFS level entirely on the device (state st[4] = fbase, nf, ncand, qt; see normals.hip);
// `grid` workgroups stride over the device-side counts.  Scratch: n entries each.
struct Bfs2Bufs {
  uint32_t* child_cnt;
  uint32_t* cursor;
  uint32_t* offs;
  uint32_t* tile_tot;
  uint32_t* slot_of;
  float* slot_d2;
  int32_t* slot_id;
  uint32_t* cell_done;  // [tmask + 1] points of each grid cell the BFS has settled (zeroed)
};
void launch_bfs2_level(int32_t* queue, long long* st, const int32_t* pos_of, const GridDesc& G,
                       const GridBufs& B, float r2, uint8_t* processed_s, uint32_t* claim_s,
                       float4* nrm_s, int32_t* cand, const Bfs2Bufs& W, int grid, hipStream_t s,
                       bool wave_claim = true);  // (false: one thread per (node, cell))
void launch_bfs_finish(const GridBufs& B, int n, const float4* nrm_s, const uint8_t* processed_s,
                       float4* nrm, uint8_t* processed, hipStream_t s);

// pcl::Normal scatter helpers
void launch_pack_normals(const float4* nrm, int n, float* out, int64_t stride_floats,
                         int curv_offset, hipStream_t s);
void launch_unpack_normals(const float* in, int n, int64_t stride_floats, float4* nrm,
                           hipStream_t s);

}  // namespace dlg
