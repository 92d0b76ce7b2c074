// driver.hpp -- host-side state shared by the RANSAC driver (driver.cpp) and the normals driver
// (normals_host.cpp): error type, device/pinned buffers, the context and cloud objects.
#pragma once

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

#include "../../include/dialog_ransac.h"
#include "comm.hpp"
#include "kernels.hpp"
#include "sac_control.hpp"
#include "postprocess.hpp"

namespace dlg {

struct DlgError : std::runtime_error {
  DlgError(dlg_status c, const std::string& m) : std::runtime_error(m), code(c) {}
  dlg_status code;
};

#define HIPCHK(expr)                                                                          \
  do {                                                                                        \
    hipError_t e_ = (expr);                                                                   \
    if (e_ != hipSuccess)                                                                     \
      throw DlgError(DLG_ERR_HIP, std::string(#expr) + " -> " + hipGetErrorString(e_));       \
  } while (0)

template <typename T>
struct DevBuf {
  T* p = nullptr;
  size_t cap = 0;
  void ensure(size_t n) {
    if (n <= cap) return;
    if (p) HIPCHK(hipFree(p));
    p = nullptr;
    cap = 0;
    size_t want = std::max<size_t>(n, 16);
    HIPCHK(hipMalloc(reinterpret_cast<void**>(&p), want * sizeof(T)));
    cap = want;
  }
  void release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
  }
};

template <typename T>
struct PinBuf {
  T* p = nullptr;
  size_t cap = 0;
  void ensure(size_t n) {
    if (n <= cap) return;
    if (p) HIPCHK(hipHostFree(p));
    p = nullptr;
    cap = 0;
    size_t want = std::max<size_t>(n, 16);
    HIPCHK(hipHostMalloc(reinterpret_cast<void**>(&p), want * sizeof(T), hipHostMallocDefault));
    cap = want;
  }
  void release() {
    if (p) (void)hipHostFree(p);
    p = nullptr;
    cap = 0;
  }
};

struct SoA {
  DevBuf<float> x, y, z;
  DevBuf<int32_t> gid;
  DevBuf<float4> nrm;  // SACMODEL_NORMAL_PLANE only (normalized normal, curvature)
  bool with_nrm = false;
  void ensure(size_t n) { x.ensure(n); y.ensure(n); z.ensure(n); gid.ensure(n); }
  void ensure_nrm(size_t n) { nrm.ensure(n); with_nrm = true; }
  void release() { x.release(); y.release(); z.release(); gid.release(); nrm.release(); with_nrm = false; }
  PointsView view(int64_t n) const {
    return PointsView{x.p, y.p, z.p, gid.p, n, with_nrm ? nrm.p : nullptr};
  }
  PointsOut out() { return PointsOut{x.p, y.p, z.p, gid.p, with_nrm ? nrm.p : nullptr}; }
};

// one sorted grid of the normals path (normals.hip): points in cell order + occupied-cell table
struct GridLevelBufs {
  DevBuf<float> sx, sy, sz;
  DevBuf<int32_t> idx, pos;
  DevBuf<uint32_t> tkeys;
  DevBuf<int2> trange;
  void release() {
    sx.release(); sy.release(); sz.release(); idx.release(); pos.release(); tkeys.release();
    trange.release();
  }
};

// scratch of the normals / RegulateNormal path (normals_host.cpp)
struct NormalsWork {
  static constexpr int kLevels = 12;
  GridLevelBufs lv[kLevels];
  DevBuf<uint8_t> raw, out, processed, processed_s, sort_tmp, dflags, fs_scr;
  DevBuf<float> x, y, z, qx, qy, qz, partial;
  DevBuf<uint32_t> keys_in, keys_out, counters;
  DevBuf<int32_t> idx_in, queue, cand, ids, ids_alt, pos_of, nn;
  DevBuf<float4> nrm, nrm_s;
  DevBuf<float4> rec;  // grid builds: the points as (x, y, z, 0) records for the sorted gather
  DevBuf<uint32_t> claim, ccnt, coffs, ccur, ctile, cslot, cdone;
  DevBuf<float> sd2;
  DevBuf<int32_t> ncnt;   // PCL-float radius normals: neighbours per query (chunk)
  DevBuf<int64_t> noff;   //   their offsets
  DevBuf<uint64_t> nkeys; //   (d2, index) keys
  DevBuf<int32_t> ovfa, ovfb;  // fused radius normals: queries with too many neighbours
  DevBuf<uint32_t> ovfc;       //   their counts
  DevBuf<long long> bst;
  PinBuf<long long> h_bst;
  DevBuf<unsigned long long> keys64, keys_alt;
  PinBuf<uint32_t> h_cnt;
  void release() {
    for (auto& l : lv) l.release();
    raw.release(); out.release(); processed.release(); processed_s.release(); sort_tmp.release(); dflags.release();
    fs_scr.release();
    x.release(); y.release(); z.release(); qx.release(); qy.release(); qz.release();
    partial.release(); nn.release();
    keys_in.release(); keys_out.release(); counters.release();
    idx_in.release(); queue.release(); cand.release(); ids.release(); ids_alt.release();
    pos_of.release(); nrm.release(); nrm_s.release(); claim.release(); keys64.release();
    keys_alt.release(); h_cnt.release(); ccnt.release(); coffs.release(); ccur.release(); cdone.release();
    sd2.release(); bst.release(); h_bst.release(); ctile.release(); cslot.release();
    ncnt.release(); noff.release(); nkeys.release();
    ovfa.release(); ovfb.release(); ovfc.release(); rec.release();
  }
};

// scratch of postProcessPlanes (postprocess_host.cpp)
struct PostWork {
  DevBuf<uint8_t> processed, flags, absorbed, keep;
  DevBuf<uint32_t> bcnt, boff, offs, abs_cnt, mask, csize;
  DevBuf<int32_t> cand, cand2, ids, parent, sel, rids, out, table, rest;
  DevBuf<PipTask> tasks;
  DevBuf<float4> planes, rays;
  DevBuf<PipEdge> edges;
  DevBuf<int64_t> edge_off;
  void release() {
    processed.release(); flags.release(); absorbed.release(); keep.release();
    bcnt.release(); boff.release(); offs.release(); abs_cnt.release(); mask.release();
    csize.release(); cand.release(); cand2.release(); ids.release(); parent.release(); sel.release();
    rids.release(); out.release(); table.release(); rest.release(); tasks.release(); planes.release(); rays.release();
    edges.release(); edge_off.release();
  }
};

}  // namespace dlg

using namespace dlg;

// execution-path options of a context (dlg_ctx_set_option).  Every combination gives the same
// results: they only select among equivalent paths (tests run each against the oracle).
struct PathOptions {
  int prune = -1;       // Morton copy + pruned scoring: -1 clouds >= 131072 points, 0 never, 1 always
  bool lean = true;     // lean-list rounds (single-pass selects driven by the Morton copy)
  bool spec_pick = true;  // device pick for probability-1 rounds
  bool prune_np = true;   // pruned NORMAL_PLANE scoring
  int score_kernel = kScoreBf16;  // exhaustive scorer: kScoreBf16 or kScoreExact
  bool prune_stats = false;       // accumulate the pruned kernel's work counters (dlg_prune_stats)
  int sel1_tile = 16384;          // points per single-pass select tile (kSel1Points)
  int tile_scorer = DLG_TILE_EXACT;  // pruned plane scorer (spatial.hpp kTileScorer*)
  bool nbr_fused = true;          // PCL-float radius normals in one fused pass (else chunked)
  bool bfs_wave = true;           // RegulateNormal's claim pass: one wave per frontier node
  // PCL float refit (DLG_REFIT_PCL, any rank count): 1 = the nine sums on the device (fsum.hip,
  // exact), 0 = gathered to the host and summed there, 2 = device, and the host recomputes the
  // refit's tail from the published sums every round, 3 = as 2 and the round's select is always
  // redone with the host's plane (exercises the path an uncertain transcendental takes)
  int pcl_dev = 1;
  int hyp_shard = -1;  // every rank holds the whole cloud; rank r scores its slice of each
                       // batch's hypotheses, the counts are allreduced (DLG_OPT_HYP_SHARD: 1 on,
                       // 0 off, -1 = on when every rank holds the same cloud, ids included)
  int fs_protocol = 0;  // several ranks: the PCL refit's protocol (DLG_OPT_FS_ONE_WALK, 0..2)
  int fs_segments = 8;  // one rank: walkers per float chain (DLG_OPT_FS_SEGMENTS)
  bool fs_poison = false;  // tests only: fill the float-sum walk's window tables with garbage
                           // entries stamped for the next launch before the clear (fs_reset)
  int fault_round = 0;     // tests only (DLG_OPT_FAULT_INJECT): > 0 = this rank throws in the
                           // middle of extract round fault_round - 1 (after the round's scoring)
  bool sync_check = false; // DLG_OPT_SYNC_CHECK: per-round allgather of (round, inliers,
                           // coefficient bits, collectives issued), mismatch fails the call
  int sel1_ticket = -1;    // DLG_OPT_SEL1_TICKET: single-pass select tiles numbered by an atomic
                           // ticket (dispatch order) instead of the workgroup index: 1 always,
                           // 0 never, -1 while another context of this process shares the device
  bool bounds_stream = false;  // DLG_OPT_BOUNDS_STREAM: lean rounds' survivor sphere bounds on a
                               // second stream beside the list pass (event-ordered)
  int spatial_curve = 1;  // DLG_OPT_SPATIAL_CURVE: 1 Hilbert, 0 Morton order of the spatial copy
  bool fs_join = true;    // DLG_OPT_FS_JOIN: segmented walk's joins by each chain's last walker
  bool unrefined_list = true;  // DLG_OPT_UNREFINED_LIST: lean PCL refit's inliers by one list pass
};

struct dlg_ctx {
  int device = 0;
  bool counted = false;  // registered in the per-device context count (ctx_shared)
  PathOptions opt;
  int num_cus = 256;
  hipStream_t stream = nullptr;
  std::unique_ptr<Comm> comm;
  // hypothesis sharding (DLG_OPT_HYP_SHARD, SURVEY 8(e)'s small-N fallback): while a call on a
  // replicated cloud runs, `comm` is a one-rank communicator (every rank computes the whole
  // round), `solo` holds the real one and `hcomm` points at it for the scoring's split
  std::unique_ptr<Comm> solo;
  Comm* hcomm = nullptr;
  // the real communicator of the group (the one a failure must abort)
  Comm* group() const { return hcomm ? hcomm : comm.get(); }
  std::string err;
  bool profiling = false;
  bool walk_events = false;  // (profiling level 1: the PCL refit walk's events too)
  bool sp_all = true;  // every rank holds a valid spatial copy (agreed per extraction)
  // scratch
  DevBuf<int32_t> pos;
  DevBuf<SampleRec> samples;
  DevBuf<HypRec> hyps;
  DevBuf<int32_t> res;  // counts[D] | good[D]
  DevBuf<int32_t> tile_in, tile_off_in, tile_off_out, totals;
  dlg::Sel1State sel1;  // single-pass selects: tile status words + launch epoch
  DevBuf<uint64_t> sel1_status;
  DevBuf<int32_t> sel1_err;  // sticky look-back failure word of the single-pass selects
  DevBuf<uint64_t> sel1_tk;  // their tile ticket counter (DLG_OPT_SEL1_TICKET; never reset:
                             // each launch's tickets start at the count issued before it)
  DevBuf<int64_t> partials, moments;  // fast refit: exact moment digits (exact_refit.hpp)
  DevBuf<unsigned> pick_done;          // the fused pick's workgroup ticket (zero between launches)
  DevBuf<unsigned> mom_done;           // k_moments' last-workgroup counter (zero between launches)
  DevBuf<double> scratch_f64;          // max-allreduce of host doubles
  DevBuf<int32_t> inl_gid;
  DevBuf<float> inl_xyz;
  DevBuf<int64_t> gath64;
  DevBuf<int32_t> gath32;
  PinBuf<int32_t> h_pos, h_res, h_tot;
  PinBuf<double> h_mom;
  PinBuf<int64_t> h_g64;
  DevBuf<float4> small;    // winning plane + samples + refined plane (segment_impl)
  DevBuf<float4> np_cn;    // NORMAL_PLANE pruned scoring: the hypotheses' normalized normals
  DevBuf<uint16_t> lp;     // pruned scoring: per super-tile lists of near planes
  DevBuf<int32_t> lp_n;
  DevBuf<unsigned long long> pstats;  // pruned-kernel work counters (DLG_OPT_PRUNE_STATS)
  PinBuf<float4> h_small;
  hipEvent_t ev[4] = {nullptr, nullptr, nullptr, nullptr};
  std::vector<int32_t> h_inl;
  std::vector<float> h_xyz;
  // inlier ids of the previous extract round: D2H into pinned staging is enqueued behind the
  // round's select, the memcpy into the caller's buffer runs while the next round's scoring
  // kernel executes (the host would otherwise only wait for it)
  PinBuf<int32_t> h_stage;
  hipEvent_t ev_stage = nullptr;
  // the deferred inlier copy runs on its own stream, off the rounds' critical path: it waits for
  // ev_inl (the round's select on the main stream); the next select waits for ev_stage
  hipStream_t cstream = nullptr;
  // DLG_OPT_BOUNDS_STREAM: the lean rounds' survivor sphere bounds on sstream beside the list
  // pass (forked by ev_fork, joined by ev_join on the main stream); created on first use
  hipStream_t sstream = nullptr;
  hipEvent_t ev_fork = nullptr, ev_join = nullptr;
  hipEvent_t ev_inl = nullptr;
  hipEvent_t ev_inl_cur = nullptr;    // the marker the copy waits for (ev_inl, or the round's
                                      // end-of-select timing event when profiling)
  hipEvent_t ev_score_end = nullptr;  // (profiling) the last speculative round's scoring end
  bool stage_inflight = false;
  DevBuf<int32_t> pick;   // k_pick_p1 result
  int32_t* pub = nullptr;  // coherent pinned: k_publish's round results (pub[0] = sequence)
  size_t pub_cap = 0;
  int32_t pub_seq = 0;
  // the last compaction's predicted Morton-copy totals, checked at the next publish
  bool sp_check = false;
  int64_t sp_expect_in = 0, sp_expect_out = 0;
  dlg_extract_stats* sel_pending = nullptr;  // select_ms of the last round, not yet read
  hipEvent_t ev_sel[2][2] = {{nullptr, nullptr}, {nullptr, nullptr}};  // per-round pairs
  hipEvent_t ev_walk[2][6] = {};  // [pair][walk start, walk end, repair start, repair end]:   // the PCL refit's walk
  bool walk_rec[2] = {false, false};  // the pair's walk events were recorded this round
  bool rep_rec[2] = {false, false};   // ... and its repair events (several ranks, rank > 0)
  bool mid_rec[2] = {false, false};   // ... and the two walks' inner events (protocols 0, 2)
  int sel_k = 0;
  DevBuf<int32_t> rk;     // every rank's (inliers, survivors) of a round
  PinBuf<int32_t> h_rk;
  PinBuf<int32_t> h_pick;
  int64_t spec_misses = 0;  // speculative picks the host replay overturned
  double t_tot = 0.0;    // (DLG_TRACE) host time the last round's totals arrived
  ShuffleReplay replay;  // drawIndexSample replay table, reused by every segment on this context  // end of a round's totals D2H (work queued after it may still run)
  int32_t* pending_dst = nullptr;
  int64_t pending_n = 0;
  int64_t pending_off = 0;   // ids already copied to the caller (pumped while waiting)
  bool stage_ready = false;  // ev_stage has completed
  int32_t* emit_dst = nullptr;  // a round's inliers to copy (enqueued after the next launches)
  int64_t emit_n = 0;
  NormalsWork nw;
  PostWork pw;
  // PCL float refit on the device (fsum.hip): scratch sized for fs_cap inliers
  DevBuf<uint8_t> fs_scr;
  // the spatial index build's sort scratch (Morton keys and orders, ping-pong; radix-sort
  // temporaries), kept across builds: no allocation per build
  DevBuf<uint32_t> mk0, mk1;
  DevBuf<int32_t> mi0, mi1;
  DevBuf<uint8_t> msort;
  DevBuf<float4> mxyz;  // the points as (x, y, z, 0) records: k_gather_order's source
  int64_t fs_cap = -1;
  FsBuffers fs_b;
  DevBuf<float> fs_x, fs_y, fs_z;  // lean rounds: the unrefined plane's inliers in list order
  DevBuf<int32_t> fs_n;
  int64_t fs_checks = 0, fs_fixes = 0;  // host recomputations of the refit tail, and redone selects
};

struct dlg_cloud {
  dlg_ctx* ctx = nullptr;
  int64_t n_points = 0;  // records of the uploaded dlg_points (normals must match)
  int32_t id_base = 0;
  bool gid_ident = false;  // pristine gid[i] == id_base + i (uploaded without setIndices)
  bool repl_known = false, repl = false;  // several ranks: every rank holds this same cloud
                                          // (decided at the first call, hyp_shard_on)
  bool has_normals = false;
  // the attached normals as given (PCL's normal_x/y/z and curvature, pristine order): RegulateNormal
  // on the device copy (dlg_cloud_regulate_normals) flips these and re-derives the normalised ones
  DevBuf<float4> raw_nrm;
  int64_t n_total = 0;
  int64_t n_active = 0;
  int cur = -1;  // -1 pristine, 0 = A, 1 = B
  SoA pristine, buf[2];
  float amax[3] = {0, 0, 0};
  float fmax = 0.0f;         // largest |coordinate| of the finite points (this rank's)
  bool qexp_known = false;   // fast refit quantum exponent (global over ranks), set lazily
  int qexp = 0;
  // Morton-ordered copy of the finite active points for the pruned scoring kernel (spatial.hpp):
  // built at upload (large clouds), compacted with the list in every SACMODEL_PLANE extract round
  bool sp_built = false;   // the pristine spatial copy exists
  bool sp_valid = false;   // the current spatial copy holds exactly the finite active points
  bool sp_dirty = false;   // sphere bounds of the working copy need recomputing
  int sp_cur = -1;         // -1 pristine, 0 / 1 ping-pong
  int64_t sp_n_pristine = 0, sp_n = 0;
  DevBuf<int32_t> sp_order;  // pristine index of each Morton-copy point (normals gathered by it)
  // curvature range of the uploaded normals (NaN ignored): bounds w = lambda (1 - curvature)
  bool curv_known = false;
  float curv_min = 0.0f, curv_max = 0.0f;
  SoA sp_pristine, sp_buf[2];
  // sphere bounds of the pristine copy and of each ping-pong buffer sp_buf[i]
  DevBuf<float4> sp_tiles_pr, sp_supers_pr, sp_tb[2], sp_sb[2];
  const SoA& sp_soa() const { return sp_cur < 0 ? sp_pristine : sp_buf[sp_cur]; }
  int sp_spare() const { return sp_cur == 0 ? 1 : 0; }
  PointsView view() const {
    const SoA& s = cur < 0 ? pristine : buf[cur];
    return s.view(n_active);
  }
  int spare() const { return cur == 0 ? 1 : 0; }
  // lean-list rounds (driver.cpp): the list buffer holds only pristine indices (in its gid
  // field; x, y, z, normals stale) until a path that reads coordinates materialises it
  bool buf_lean[2] = {false, false};
  bool list_lean() const { return cur >= 0 && buf_lean[cur]; }
  DevBuf<uint32_t> ubits;  // PCL refit in lean rounds: unrefined inliers by pristine index (zero between rounds)
  bool ubits_dirty = false;  // stamped but not (known to be) compacted: cleared before next use
  DevBuf<uint8_t> tag;  // per pristine point: the stamp of the select that took it
  int tagv = 0;         // last stamp used (tag[] is zeroed when the byte wraps)
};

namespace dlg {

inline void set_device(dlg_ctx* c) { HIPCHK(hipSetDevice(c->device)); }
// live contexts of this process per device (the look-back selects' tile numbering: ctx_shared)
void ctx_count_add(int device, int delta);
bool ctx_shared(int device);
// (several ranks over RCCL: a polling wait that ends when the group is aborted, comm.hpp)
inline void sync(dlg_ctx* c) { c->group()->sync_stream(c->stream); }

inline dlg_status fail(dlg_ctx* c, dlg_status code, const std::string& msg) {
  if (c) c->err = msg;
  return code;
}

// runs f with the context's device current; exceptions become status codes + dlg_last_error text
template <typename F>
dlg_status guarded(dlg_ctx* c, F&& f) {
  try {
    if (c) set_device(c);
    f();
    if (c) c->err.clear();
    return DLG_OK;
  } catch (const CommAborted& e) {
    return fail(c, DLG_ERR_COMM, e.what());
  } catch (const DlgError& e) {
    return fail(c, e.code, e.what());
  } catch (const std::exception& e) {
    return fail(c, DLG_ERR_INTERNAL, e.what());
  } catch (...) {
    return fail(c, DLG_ERR_INTERNAL, "unknown error");
  }
}

// guarded for the entry points whose ranks run collectives together: a rank that fails aborts
// its group, so every peer returns DLG_ERR_COMM (naming this rank and its error) instead of
// waiting in the next collective forever (the reference's convention: every caller gets a
// status back, PlaneDetect.h:371-375, 592-596).  A failed group stays aborted.
template <typename F>
dlg_status guarded_group(dlg_ctx* c, F&& f) {
  const dlg_status s = guarded(c, f);
  if (s != DLG_OK && s != DLG_ERR_COMM && c && c->group()->world() > 1)
    c->group()->abort("rank " + std::to_string(c->group()->rank()) + " failed: " + c->err);
  return s;
}

// normals on the device -> the cloud (dlg_cloud_set_normals, dlg_cloud_estimate_normals)
void attach_normals(dlg_ctx* c, dlg_cloud* cl, const float* raw_dev, int64_t stride_f,
                    int curv_off, bool by_pos);

}  // namespace dlg
