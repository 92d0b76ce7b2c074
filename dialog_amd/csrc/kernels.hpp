// kernels.hpp -- device kernels of the RANSAC plane path (gfx950 / CDNA4) and their launchers.
//
// Layout in HBM (per rank, per cloud): structure-of-arrays float x[], y[], z[] plus int32 gid[]
// (global point id), active prefix [0, n_active).  Extract-and-remove compacts the survivors
// into a ping-pong set of the same arrays, so every scoring pass streams exactly 12 B per active
// point and the active order stays the PCL "remaining indices" order.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

#include "exact_refit.hpp"

namespace dlg {

// one sampled point of a hypothesis (gathered by list position; zero on ranks not holding it)
struct alignas(16) SampleRec {
  int32_t gid;
  float x, y, z;
};

// plane hypothesis: PCL coefficients + the rounding band of an FMA evaluation around cthr
struct alignas(16) HypRec {
  float a, b, c, d;
  float tlo, thi;  // [cthr - 7 u S, cthr + 7 u S) rounded outwards
  int32_t good;    // SampleConsensusModelPlane::isSampleGood
  float w;         // >= 7 u S (k_prep_bf16 derives the matrix-core band from it)
};

// nrm (optional, SACMODEL_NORMAL_PLANE): per point (n.normalized() as Eigen computes it for
// getAngle3D, curvature) -- normalised once at upload, bit-identical to normalising per test
struct PointsView {
  const float* x;
  const float* y;
  const float* z;
  const int32_t* gid;
  int64_t n;
  const float4* nrm;
};

struct PointsOut {
  float* x;
  float* y;
  float* z;
  int32_t* gid;
  float4* nrm;
};

// inlier test of the select / moments / scoring kernels
//   SACMODEL_PLANE        : |pcl_dot(c, p)| < cthr            (cthr = smallest float >= threshold)
//   SACMODEL_NORMAL_PLANE : |w d_normal + (1 - w) d_euclid| < thr, w = lambda (1 - curvature)
struct ModelTest {
  float cthr;
  int normal_plane;
  double thr;
  double lambda;
};

constexpr int kMaxHypPerLaunch = 4096;  // LDS count array of the scoring kernel
constexpr int kSelTile = 4096;          // points per select/compact workgroup

// Exhaustive scoring kernels (every active point against every hypothesis; the pruned kernel
// of spatial.hpp is the default whenever the cloud has a Morton copy).  All give bit-identical
// counts (tests/test_score_variants.py); dlg_score_benchmark takes these values.
//   exact  : PCL op order (3 mul + 3 add) + compare on the VALU, 4 points per lane
//   bf16   : plane distances on the bf16 matrix cores (3-way split operands, products exact),
//            counting + band tracking on the VALU, exact PCL re-decision inside the rounding band
//   pruned : k_score_bf16's 32 x 32 blocks only for (tile, plane) pairs the bounding spheres
//            cannot rule out (dlg_score_benchmark only: the driver takes it whenever it can)
enum ScoreKernel { kScoreExact = 0, kScoreBf16 = 1, kScorePruned = 2 };
// hyps buffer layout for launch_score: HypRec[kMaxHypPerLaunch] followed by the packed float4
// plane vectors and float band widths (score_scratch_bytes); counts need room for D rounded up
// to a multiple of 64.
// For the bf16 variants the tail also holds each plane's B column (32 bf16 = 4 x uint4) and its
// band (float2).
constexpr size_t kHypScratchBytes =
    kMaxHypPerLaunch * (sizeof(HypRec) + sizeof(float4) + sizeof(float) + 4 * sizeof(uint4) +
                        sizeof(float2));
// positions pos[m] (global list positions; this rank's list starts at lo) -> SampleRecs (zero
// when another rank owns the position).  Lean lists: lidx = the list's pristine indices (null
// while the list is the pristine one), src = the pristine copy, n_list = the list length.
void launch_gather_samples(const int32_t* pos, int m, int64_t lo, PointsView src, SampleRec* out,
                           hipStream_t s, const int32_t* lidx = nullptr, int64_t n_list = 0);
// writes hyps[D] and good[D] (int32 flags next to the counts for one D2H copy)
// round results into the coherent pinned buffer pub (layout below), then pub[0] = seq (release,
// system scope)
// (err: the single-pass selects' sticky look-back error word, or null)
constexpr int kPubTot = 1, kPubPick = 5, kPubErr = 7, kPubSmall = 8, kPubRk = 64;  // + nrk: counts
struct PubArgs {
  const int32_t* totals = nullptr;
  int ntot = 0;
  const float4* small = nullptr;
  int nsmall = 0;
  const int32_t* rk = nullptr;
  int nrk = 0;
  const int32_t* pick = nullptr;
  int npick = 0;
  const int32_t* res = nullptr;
  int nres = 0;
  const int32_t* err = nullptr;
  int32_t* pub = nullptr;
  int32_t seq = 0;
};
void launch_publish(const PubArgs& a, hipStream_t s);
// speculative computeModel decision for probability 1 over one batch (k_pick_p1): out[0] best
// batch index (-1 none), out[1] loop ended inside the batch; winner copied to best / best_smp
struct PickArgs {
  const int32_t* res = nullptr;  // counts[Dp] | good[D]
  int Dp = 0, D = 0, need_good = 0;
  const HypRec* hyps = nullptr;
  const SampleRec* samples = nullptr;
  HypRec* best = nullptr;
  SampleRec* best_smp = nullptr;
  int32_t* out = nullptr;
  unsigned* done = nullptr;  // fused into the pruned scoring: its workgroup ticket (zero between
                             // launches; the last workgroup resets it)
};
void launch_pick_p1(const PickArgs& a, hipStream_t s);
// one rank: positions (pinned host buffer, 3 per draw) -> samples, hypotheses, good flags in
// res[Dp + d] and zeroed counts res[0, Dp)  (gather + build + memset in one launch)
// lidx: the lean list's pristine indices (src = the pristine copy, n_list = list length)
void launch_gather_build(const int32_t* pos_host, int D, PointsView src, SampleRec* samples,
                         float cthr, float ax, float ay, float az, HypRec* hyps, int32_t* res,
                         hipStream_t s, const int32_t* lidx = nullptr, int64_t n_list = 0);

// single-pass select (decoupled look-back) of the lean-list rounds: status words per tile, an
// epoch per launch (so the words never need clearing)
struct Sel1State {
  uint64_t* status = nullptr;
  uint32_t epoch = 0;
  int32_t* err = nullptr;  // sticky: != 0 once a tile's look-back failed (host checks and clears)
  // tile tickets (null: tile = workgroup index): a launch's workgroups take tickets base ..
  // base + ntiles - 1 from *ticket in dispatch order; issued = the host's running total
  unsigned long long* ticket = nullptr;
  uint64_t base = 0;
  uint64_t issued = 0;
};
// tiles (status words) a single-pass select over n points may use (the smallest tile size: an
// upper bound for every kSel1Points choice)
int sel1_tiles(int64_t n);
// points per single-pass select tile (workgroups of tile / 16 threads, 16 points per lane)
constexpr int kSel1Points[3] = {4096, 8192, 16384};
// the Morton copy's select: survivors -> dst, inliers stamped tag[pristine index] = tagv;
// totals[0] = inliers, totals[1] = n_list - inliers, totals[4] = Morton survivors
// pub non-null: the last tile also publishes the round (as launch_publish) once the totals are
// final.  tile_pts: one of kSel1Points
void launch_sel1_morton(PointsView sp, const float4* coef, const ModelTest& mt, Sel1State& L,
                        uint8_t* tag, uint8_t tagv, const PointsOut& dst, int64_t n_list,
                        int32_t* totals, hipStream_t s, const PubArgs* pub, int tile_pts);
// the lean list's compaction from the stamps (lidx null: the pristine list): inlier ids in list
// order -> inl_gid, survivors' pristine indices -> out_lidx; totals[0..1] = (in, out).
// pgid null: the pristine ids are gid_base + pristine index (an upload without setIndices)
void launch_sel1_list(const int32_t* lidx, int64_t n, const uint8_t* tag, uint8_t tagv,
                      const int32_t* pgid, int32_t gid_base, Sel1State& L, int32_t* inl_gid,
                      int32_t* out_lidx, int32_t* totals, hipStream_t s, int tile_pts);
// a lean list's x, y, z, gid (+ normals) from the pristine copy, in place (io.gid holds the
// pristine indices on entry)
void launch_list_materialize(PointsView pristine, int64_t n, const PointsOut& io, hipStream_t s);
void launch_build_hyps(const SampleRec* samples, int D, float cthr, float ax, float ay, float az,
                       HypRec* hyps, int32_t* good, hipStream_t s);
// counts[D] = #{i < n : |plane_h . (x_i, y_i, z_i, 1)| < cthr}, PCL (Eigen SSE) op order, with
// kernel kScoreExact or kScoreBf16.  counts must be zeroed by the caller (same stream).
void launch_score(PointsView src, const HypRec* hyps, int D, float cthr, int32_t* counts,
                  int kernel, int num_cus, hipStream_t s);
// B columns (bf16 split plane coefficients) and band widths of D plane hypotheses for the bf16
// matrix-core scoring kernels, written into the hyps scratch tail; returns pointers to them
void launch_prep_bf16(const HypRec* hyps, int D, const uint4** bcol, const float** band,
                      hipStream_t s);
// SampleConsensusModelNormalPlane::countWithinDistance for D hypotheses (src.nrm required);
// counts need room for D rounded up to 64 and must be zeroed by the caller
void launch_score_np(PointsView src, const HypRec* hyps, int D, const ModelTest& mt,
                     int32_t* counts, int num_cus, hipStream_t s);
// fast refit (exact_refit.hpp): the exact integer moments (kMomDigits int64 digit sums) of the
// inliers of coef, quantised with exponent qexp; partials [kMomDigits][nblocks] scratch, reduced
// by the launch's last workgroup -> out.  done: a device counter, zero before the first launch
// (each launch leaves it zero)
int moments_blocks(int64_t n);
// coef: device float4 (a, b, c, d)
// one rank: moments of the unrefined plane's inliers + reduction + refit in one launch
void launch_moments_refit(PointsView src, const float4* coef, const ModelTest& mt, int qexp,
                          int64_t* partials, unsigned* done, int nblocks, int64_t* out,
                          float4* cout, hipStream_t s);
void launch_moments(PointsView src, const float4* coef, const ModelTest& mt, int qexp,
                    int64_t* partials, unsigned* done, int nblocks, int64_t* out, hipStream_t s);
// lean rounds (plane model): the same moments over the Morton copy reading only the tiles whose
// sphere may hold an inlier (tiles / supers: the copy's spheres, margin: the scoring's
// prune_margin); cout non-null: one rank, refit too (as launch_moments_refit)
int moments_sp_blocks(int64_t n);
void launch_moments_sp(PointsView src, const float4* tiles, const float4* supers, float margin,
                       const float4* coef, const ModelTest& mt, int qexp, int64_t* partials,
                       unsigned* done, int nblocks, int64_t* out, float4* cout, hipStream_t s);
// PCL refit in lean rounds (any rank count: each rank its own shard): the unrefined plane's
// inliers, stamped into a bitmap over pristine indices from the Morton copy's near tiles
// (launch_ustamp), then compacted in
// ascending pristine order = list order into x/y/z arrays (launch_ucompact; clears the bitmap,
// count -> *n_out).  bits: ceil(n_pristine / 32) words, zero on entry.
void launch_ustamp(PointsView sp, const float4* tiles, const float4* supers, float margin,
                   const float4* coef, const ModelTest& mt, uint32_t* bits, hipStream_t s);
int ucompact_tiles(int64_t nwords);
// the unrefined plane's inliers' x, y, z in list order in one list pass (lidx null: the pristine
// list); count to *n_out (k_ulist)
void launch_ulist(const int32_t* lidx, int64_t n, PointsView pristine, const float4* coef,
                  const ModelTest& mt, Sel1State& L, float* ox, float* oy, float* oz,
                  int32_t* n_out, hipStream_t s);
void launch_ucompact(uint32_t* bits, int64_t nwords, PointsView pristine, Sel1State& L, float* ox,
                     float* oy, float* oz, int32_t* n_out, hipStream_t s);

// PCL's float refit on the device (fsum.hip): the nine sequential float sums of
// computeMeanAndCovarianceMatrix evaluated exactly in parallel (fsum.hpp), then the float
// eigen33.  Inliers px/py/pz with element stride `stride` floats, count *n_dev (<= n_cap): this
// rank's segment of the list (the ranks' segments in rank order make up the list).
// res (16 int32): [0] = 1 when a transcendental of eigen33 could not be rounded for certain
// (the host then recomputes the plane from the sums), [1] = n, [2..10] = the nine sums' bits.
struct FsNode;
// one rank: the float-sum walk splits each chain into at most kFsSegMax segments of at least
// kFsSegWin windows (64 records each), walked at once from the refined guesses and joined by
// k_fs_segfix (segments = 1: one walker per chain)
constexpr int kFsSegMax = 16, kFsSegWin = 8;
struct FsBuffers {
  double* csum = nullptr;  // [chunks][9] double sums of the terms
  double* usum = nullptr;  // [units][9]
  double* upre = nullptr;  // [units][9] exclusive prefixes
  FsNode* rec = nullptr;   // chunk records, chain-major: rec[c * cap + k]
  int64_t cap = 0;         // chunks per chain
  uint4* srec = nullptr;   // the records' integer-stepping tables (3 x 16 B each): srec[3 (c * cap + k) + j]
  float4* win = nullptr;   // window summaries (64 records each), chain-major: win[c * wcap + w]
  int64_t wcap = 0;        // windows per chain
  float* sums = nullptr;   // [18] the chains' end values, then the starts the walk took
  float* start9 = nullptr; // [9] several ranks: the chains' values at this rank's first inlier
  float* g2 = nullptr;     // [9] several ranks: the propagated guesses (k_fs_guess2)
  float* gath2 = nullptr;  // [world][18] several ranks: every rank's first-walk sums
  float* seg = nullptr;    // [9][kFsSegMax][2] one rank, segmented walk: each segment's start, end
  double* tot = nullptr;   // [10] several ranks: this rank's double term sums + inlier count
  double* base9 = nullptr; // [9] several ranks: the totals of the ranks before this one
  int64_t* n_global = nullptr;  // several ranks: the inliers of all ranks
  double* gath = nullptr;  // [world][10] several ranks: every rank's tot
  unsigned* ticket = nullptr;  // [2], zero on entry
  int64_t* wst = nullptr;      // [9][8] walk counters (dlg_float_sums), or null
  float* vw = nullptr;         // [9][wcap] several ranks: each window's entry value along the
                               // walk from the rank's guess (k_fs_repair compares against it)
  uint2* wtab = nullptr;       // [9][wcap][128] window transfer tables (fs_wtab_item): (exit value
                               // bits, launch stamp) for entry leads -64..63 in the window's
                               // smallest quantum; stamp 0 or stale: no entry
  uint2* wq = nullptr;         // [9][wcap] (the table's quantum bits, launch stamp)
};
// bytes of scratch for n_cap inliers; carve() lays the buffers out in `base`
// (world: the ranks of the communicator passed to launch_fs_refit; comm null or one rank: the
// whole list is here)
size_t fs_scratch_bytes(int64_t n_cap, int world);
FsBuffers fs_carve(void* base, int64_t n_cap, int world);
// after every fs_carve, before the first launch_fs_refit on it: zero the tickets and the window
// tables (a table entry is valid only with the current launch's stamp, and reused scratch --
// another layout's records, or a hipMalloc recycling freed memory -- could hold a word with that
// stamp).  poison (tests only): first fill the tables with garbage entries carrying the next
// launch's stamp, i.e. exactly what the clear must remove.
hipError_t fs_reset(const FsBuffers& b, hipStream_t s, bool poison = false);
class Comm;
// ev_walk0 / ev_walk1 (optional): timing events around the walks (several ranks: from the first
// walk's dispatch to the second's end); ev_rep0 / ev_rep1 (several ranks, rank > 0): riding
// k_fs_repair's.  protocol (several ranks, DLG_OPT_FS_ONE_WALK): 0 = walk, rebase on the
// propagated guess, walk again, hand the exact chain ends rank to rank (repairs of a few windows);
// 1 = round 4's: no rebase (repairs from ~1000 quanta off); 2 = as 0 with parallel repair
// iterations and host checks instead of the hand-over (A/B and tests only).  *repairs (optional)
// = the repair steps the round took (0 and 1: the W - 1 hops; 2: the iterations).  segments (one
// rank): walkers per chain (1..kFsSegMax; see kFsSegMax).  ev_mid0 / ev_mid1 (several ranks,
// protocols 0 and 2, rank > 0): the first walk's end and the second walk's start, so the two walks
// are timed apart from the exchange and the rebase between them
void launch_fs_refit(const float* px, const float* py, const float* pz, int stride,
                     const int32_t* n_dev, int64_t n_cap, const FsBuffers& b, const float4* cin,
                     float4* cout, int32_t* res, int num_cus, hipStream_t s, Comm* comm = nullptr,
                     hipEvent_t ev_walk0 = nullptr, hipEvent_t ev_walk1 = nullptr,
                     hipEvent_t ev_rep0 = nullptr, hipEvent_t ev_rep1 = nullptr,
                     int protocol = 0, int* repairs = nullptr, int segments = 1,
                     hipEvent_t ev_mid0 = nullptr, hipEvent_t ev_mid1 = nullptr,
                     bool fused_join = true);

// device fast refit: cout = refit_exact of the summed digits, or cin when optimize == 0 or fewer
// than 4 inliers
void launch_refit_moments(const int64_t* moments, int qexp, const float4* cin, int optimize,
                          float4* cout, hipStream_t s);
// select: inliers of coef in list order; optional inlier xyz (AoS, 3 floats); optional
// compaction of the outliers (and their normals) into dst.  tile_in/out: [ntiles] scratch;
// totals[2] = {in, out}.
int select_tiles(int64_t n);
void launch_select(PointsView src, const float4* coef, const ModelTest& mt, int32_t* tile_in,
                   int32_t* tile_off_in, int32_t* tile_off_out, int32_t* totals, int32_t* inl_gid,
                   float* inl_xyz, const PointsOut* dst, hipStream_t s);
// the two halves of launch_select: counts + scan (totals final), then the ordered scatter
void launch_select_head(PointsView src, const float4* coef, const ModelTest& mt, int32_t* tile_in,
                        int32_t* tile_off_in, int32_t* tile_off_out, int32_t* totals,
                        hipStream_t s);
void launch_select_tail(PointsView src, const float4* coef, const ModelTest& mt,
                        const int32_t* tile_off_in, const int32_t* tile_off_out, int32_t* inl_gid,
                        float* inl_xyz, const PointsOut* dst, hipStream_t s);
// raw caller normals (n records of stride_f floats, curvature at curv_off) gathered by the
// cloud's local point index (gid - id_base) -> (normalized normal, curvature), or the raw
// (normal, curvature) when normalize is false
void launch_pack_point_normals(const float* raw, int64_t stride_f, int curv_off, PointsView src,
                               int32_t id_base, float4* out, hipStream_t s, bool normalize = true);
// cloud upload: records of stride_f floats (xyz first), optional index list -> SoA + ids
void launch_upload_gather(const float* raw, int64_t stride_f, const int32_t* idx, int64_t n,
                          int32_t id_base, PointsOut out, hipStream_t s);
// max |x|, |y|, |z| over the cloud (prefilter error bound; NaN ignored, inf kept) and the
// largest |coordinate| of its finite points (fast refit quantum); out: 4 floats (as uint bits)
void launch_absmax(PointsView src, uint32_t* out4, hipStream_t s);

}  // namespace dlg
