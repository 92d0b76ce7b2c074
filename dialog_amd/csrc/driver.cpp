// driver.cpp -- host driver of the MI355X RANSAC plane path and its C ABI (include/dialog_ransac.h).
//
// One RANSAC segment() (PCL 1.8 SACSegmentation<PointXYZ>::segment, SACMODEL_PLANE, SAC_RANSAC;
// reference call pattern Dialog/SimplifyVerticesSize.cpp:62-67) runs as:
//
//   host   : replay SampleConsensusModel::drawIndexSample over list *positions* for a batch of D
//            draws (mt19937(seed) >> 1, swaps kept in a sparse overlay of the shuffled list; the
//            positions do not depend on the data, only on N_active)
//   device : k_gather_samples (positions -> points, per shard) [+ allreduce over ranks]
//            k_build_hyps     (isSampleGood + computeModelCoefficients, PCL op order)
//            k_score          (countWithinDistance for all D draws)    [+ allreduce of counts]
//   host   : replay RandomSampleConsensus::computeModel over the D counts in draw order
//            (strict '>' keeps the first best, k = log(1-p)/log(1-w^3), iteration cap, 1000-bad-
//            draw getSamples limit); next batch only if the loop has not terminated
//   device : refit (PCL float parity mode on the host from the gathered inlier xyz, or fast
//            double moments on the device) and the final selectWithinDistance, which in
//            extract-and-remove mode also compacts the survivors into the ping-pong buffers.
//
// The data-independent part of getSamples (which list positions are swapped) is what lets the
// whole hypothesis batch be scored in one launch while still reproducing PCL's sequential RNG
// use bit-for-bit.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <climits>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <stdexcept>
#include <string>
#include <vector>

#include "../../include/dialog_ransac.h"
#include "comm.hpp"
#include "driver.hpp"
#include "fsum.hpp"
#include "host_math.hpp"
#include "kernels.hpp"
#include "sac_control.hpp"
#include "spatial.hpp"

namespace dlg {

}  // namespace dlg

using namespace dlg;

namespace {

// DLG_TRACE=1: per-round host timing breakdown on stderr (diagnostics only)
bool trace_on() {
  static const bool on = [] {
    const char* e = std::getenv("DLG_TRACE");
    return e && e[0] == '1';
  }();
  return on;
}
double now_ms() {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

// spin until k_publish has released `seq` into c->pub[0] (the round's results are then in
// c->pub).  A stream query backs it up (no event marker on the stream: each one costs the GPU
// a few microseconds between kernels): once the stream has drained the word must be visible; an
// error of the stream surfaces through the query.
void pump_pending(dlg_ctx* c, int64_t ids);

void wait_published(dlg_ctx* c, int32_t seq) {
  Comm* g = c->group();
  const bool poll = g->world() > 1;
  const auto t0 = std::chrono::steady_clock::now();
  for (uint32_t k = 1;; ++k) {
    if (__atomic_load_n(c->pub, __ATOMIC_ACQUIRE) == seq) return;
    // (several ranks: a failed peer's poison, or no progress within the group's timeout, ends
    // the wait -- the round's collectives may be waiting for that peer on the device)
    if (poll && (k & 255u) == 0) {
      g->check();
      if (g->timeout_ms > 0 && (k & 65535u) == 0) {
        const auto ms = std::chrono::duration_cast<std::chrono::milliseconds>(
                            std::chrono::steady_clock::now() - t0).count();
        if (ms > g->timeout_ms) {
          g->abort("rank " + std::to_string(g->rank()) + ": round not published after " +
                   std::to_string(ms) + " ms (DLG_OPT_COMM_TIMEOUT_MS)");
          g->check();
        }
      }
    }
    // the staged ids go to the caller while we wait; until their copy has landed, its event is
    // queried only every 16th spin (a HIP API call takes the runtime lock)
    if (c->stage_ready || (k & 15u) == 0) pump_pending(c, 16384);
    if ((k & 1023u) == 0) {
      const hipError_t e = hipStreamQuery(c->stream);
      if (e == hipSuccess) {
        if (__atomic_load_n(c->pub, __ATOMIC_ACQUIRE) == seq) return;
        throw DlgError(DLG_ERR_INTERNAL, "round results not visible after the round completed");
      }
      if (e != hipErrorNotReady) HIPCHK(e);
    }
#if defined(__x86_64__)
    __builtin_ia32_pause();
#endif
  }
}

// a single-pass select's look-back failed (sticky word set): clear it and fail the call
[[noreturn]] void sel1_failed(dlg_ctx* c) {
  (void)hipMemsetAsync(c->sel1_err.p, 0, sizeof(int32_t), c->stream);
  if (c->sel1_tk.p) {  // (a failed launch may have left tickets untaken)
    (void)hipMemsetAsync(c->sel1_tk.p, 0, sizeof(uint64_t), c->stream);
    c->sel1.issued = 0;
  }
  (void)hipStreamSynchronize(c->stream);
  throw DlgError(DLG_ERR_INTERNAL, "single-pass select did not complete (look-back gave up)");
}

// the previous compaction's Morton-copy totals (in, out) against what the list copy predicted
void check_sp_totals(dlg_ctx* c, const int32_t* sp_tot) {
  if (!c->sp_check) return;
  c->sp_check = false;
  if (c->sp_expect_in != 0 || c->sp_expect_out != 0) {
    if (sp_tot[0] != c->sp_expect_in || sp_tot[1] != c->sp_expect_out)
      throw DlgError(DLG_ERR_INTERNAL, "spatial copy out of step with the active list");
  }
}

// the PCL refit walk's share of a round's select phase (its events ride k_fs_walk's dispatch)
void add_walk_ms(dlg_ctx* c, int k) {
  if (!c->walk_rec[k]) return;
  float ms = 0.f;
  if (c->mid_rec[k]) {
    // several ranks, rank > 0: the two walks apart from the exchange and rebase between them
    float a = 0.f, b = 0.f;
    HIPCHK(hipEventElapsedTime(&a, c->ev_walk[k][0], c->ev_walk[k][4]));
    HIPCHK(hipEventElapsedTime(&b, c->ev_walk[k][5], c->ev_walk[k][1]));
    HIPCHK(hipEventElapsedTime(&ms, c->ev_walk[k][4], c->ev_walk[k][5]));
    c->sel_pending->refit_rebase_ms += ms;
    ms = a + b;
    c->mid_rec[k] = false;
  } else {
    HIPCHK(hipEventElapsedTime(&ms, c->ev_walk[k][0], c->ev_walk[k][1]));
  }
  c->sel_pending->refit_walk_ms += ms;
  c->walk_rec[k] = false;
  if (c->rep_rec[k]) {
    HIPCHK(hipEventElapsedTime(&ms, c->ev_walk[k][2], c->ev_walk[k][3]));
    c->sel_pending->refit_repair_ms += ms;
    c->rep_rec[k] = false;
  }
}

// after a stream synchronisation: the last compaction's Morton-copy totals and select timing
void settle_round(dlg_ctx* c) {
  if (c->sel1_err.p) {
    int32_t e = 0;
    HIPCHK(hipMemcpy(&e, c->sel1_err.p, 4, hipMemcpyDeviceToHost));
    if (e) sel1_failed(c);
  }
  if (c->sp_check) {
    int32_t t[2] = {0, 0};
    HIPCHK(hipMemcpy(t, c->totals.p + 2, 8, hipMemcpyDeviceToHost));
    check_sp_totals(c, t);
  }
  if (c->sel_pending) {
    const int k = c->sel_k ^ 1;  // the last round's pair
    float ms = 0.f;
    HIPCHK(hipEventElapsedTime(&ms, c->ev_sel[k][0], c->ev_sel[k][1]));
    c->sel_pending->select_ms += ms;
    add_walk_ms(c, k);
    c->sel_pending = nullptr;
  }
}

int64_t allgather_i64(dlg_ctx* c, int64_t v, std::vector<int64_t>* all) {
  const int W = c->comm->world();
  all->assign(W, 0);
  if (W == 1) {
    (*all)[0] = v;
    return v;
  }
  c->gath64.ensure(W + 1);
  c->h_g64.ensure(W + 1);
  c->h_g64.p[0] = v;
  HIPCHK(hipMemcpyAsync(c->gath64.p + W, c->h_g64.p, 8, hipMemcpyHostToDevice, c->stream));
  c->comm->allgather(c->gath64.p + W, c->gath64.p, 1, DType::I64, c->stream);
  HIPCHK(hipMemcpyAsync(c->h_g64.p, c->gath64.p, 8 * W, hipMemcpyDeviceToHost, c->stream));
  sync(c);
  int64_t s = 0;
  for (int r = 0; r < W; ++r) {
    (*all)[r] = c->h_g64.p[r];
    s += c->h_g64.p[r];
  }
  return s;
}

// gather every rank's device list (count_r items of `width` int32 each) into host `out`, rank order
void gather_lists(dlg_ctx* c, const int32_t* dev_local, int64_t n_local, int width,
                  std::vector<int32_t>* out) {
  const int W = c->comm->world();
  std::vector<int64_t> cnt;
  int64_t total = allgather_i64(c, n_local, &cnt);
  out->resize((size_t)(total * width));
  if (W == 1) {
    if (total)
      HIPCHK(hipMemcpyAsync(out->data(), dev_local, (size_t)total * width * 4, hipMemcpyDeviceToHost,
                            c->stream));
    sync(c);
    return;
  }
  int64_t mx = *std::max_element(cnt.begin(), cnt.end());
  if (mx == 0) return;
  const size_t per = (size_t)mx * width;
  c->gath32.ensure(per * (W + 1));
  int32_t* send = c->gath32.p + per * W;
  if (n_local)
    HIPCHK(hipMemcpyAsync(send, dev_local, (size_t)n_local * width * 4, hipMemcpyDeviceToDevice,
                          c->stream));
  c->comm->allgather(send, c->gath32.p, per, DType::I32, c->stream);
  std::vector<int32_t> tmp(per * W);
  HIPCHK(hipMemcpyAsync(tmp.data(), c->gath32.p, per * W * 4, hipMemcpyDeviceToHost, c->stream));
  sync(c);
  size_t w = 0;
  for (int r = 0; r < W; ++r) {
    std::memcpy(out->data() + w, tmp.data() + per * r, (size_t)cnt[r] * width * 4);
    w += (size_t)cnt[r] * width;
  }
}

float event_ms(dlg_ctx* c, int a, int b) {
  float ms = 0.f;
  HIPCHK(hipEventElapsedTime(&ms, c->ev[a], c->ev[b]));
  return ms;
}

void drain_pending(dlg_ctx* c) {
  if (!c->pending_dst) return;
  if (!c->stage_ready) HIPCHK(hipEventSynchronize(c->ev_stage));
  std::memcpy(c->pending_dst + c->pending_off, c->h_stage.p + c->pending_off,
              (size_t)(c->pending_n - c->pending_off) * 4);
  c->pending_dst = nullptr;
  c->pending_n = c->pending_off = 0;
}

// part of the staged ids to the caller, once the copy has landed (called while the host spins
// on a round's results, so the copy costs the rounds nothing)
void pump_pending(dlg_ctx* c, int64_t ids) {
  if (!c->pending_dst) return;
  if (!c->stage_ready) {
    const hipError_t e = hipEventQuery(c->ev_stage);
    if (e == hipErrorNotReady) return;
    HIPCHK(e);
    c->stage_ready = true;
  }
  const int64_t n = std::min<int64_t>(ids, c->pending_n - c->pending_off);
  std::memcpy(c->pending_dst + c->pending_off, c->h_stage.p + c->pending_off, (size_t)n * 4);
  c->pending_off += n;
  if (c->pending_off == c->pending_n) {
    c->pending_dst = nullptr;
    c->pending_n = c->pending_off = 0;
  }
}

// the requested inlier copy: device -> pinned stage on the copy stream, behind the select that
// wrote inl_gid (ev_inl); enqueued after the next round's launches, off the host's critical path
void flush_emit(dlg_ctx* c) {
  if (!c->emit_dst) return;
  drain_pending(c);  // (the stage is reused)
  c->h_stage.ensure((size_t)c->emit_n);
  if (!c->ev_stage) HIPCHK(hipEventCreateWithFlags(&c->ev_stage, hipEventDisableTiming));
  HIPCHK(hipStreamWaitEvent(c->cstream, c->ev_inl_cur, 0));
  HIPCHK(hipMemcpyAsync(c->h_stage.p, c->inl_gid.p, (size_t)c->emit_n * 4, hipMemcpyDeviceToHost,
                        c->cstream));
  HIPCHK(hipEventRecord(c->ev_stage, c->cstream));
  c->stage_inflight = true;  // inl_gid is read until ev_stage
  c->pending_dst = c->emit_dst;
  c->pending_n = c->emit_n;
  c->pending_off = 0;
  c->stage_ready = false;
  c->emit_dst = nullptr;
  c->emit_n = 0;
}

struct SegOut {
  bool has_model = false;
  float coeff[4] = {0, 0, 0, 0};
  int64_t n_in_local = 0;   // refined inliers on this rank (ids in ctx->inl_gid)
  int64_t n_out_local = 0;  // survivors on this rank (compacted into the spare buffer if remove)
  int64_t n_in_global = 0;
  bool sp_compacted = false;  // the spatial copy's survivors are in its spare buffer
  int64_t sp_n_out = 0;
  bool lean = false;  // lean-list round: the spare list buffer holds pristine indices only
  // every rank's refined inliers / survivors (device allgather folded into the round's sync)
  std::vector<int64_t> in_ranks, out_ranks;
};

// pruned scoring (spatial.hpp): by default clouds of >= kPruneMinPoints points get a Morton copy
constexpr int64_t kPruneMinPoints = 131072;

// the pruned kernel's work counters (DLG_OPT_PRUNE_STATS), accumulated over its launches
// the list lengths + the scorers' work area (spatial.hpp); a new allocation starts with zeroed
// counters (afterwards the scorer's last workgroup leaves them zero)
void ensure_prune_work(dlg_ctx* c, int64_t ns) {
  int32_t* old = c->lp_n.p;
  c->lp_n.ensure((size_t)prune_work_words(ns));
  if (c->lp_n.p != old) HIPCHK(hipMemsetAsync(c->lp_n.p, 0, sizeof(int32_t) * c->lp_n.cap, c->stream));
}

unsigned long long* prune_stats_ptr(dlg_ctx* c) {
  return c->opt.prune_stats ? c->pstats.p : nullptr;
}

void build_spatial(dlg_ctx* c, dlg_cloud* cl) {
  const int64_t n = cl->n_total;
  DevBuf<uint32_t>& k0 = c->mk0;
  DevBuf<uint32_t>& k1 = c->mk1;
  DevBuf<int32_t>& i0 = c->mi0;
  DevBuf<int32_t>& i1 = c->mi1;
  DevBuf<uint8_t>& tmp = c->msort;
  {
    k0.ensure(n); k1.ensure(n); i0.ensure(n); i1.ensure(n);
    const size_t tb = morton_sort_temp_bytes(n);
    tmp.ensure(std::max<size_t>(tb, 16));
    c->totals.ensure(8);
    HIPCHK(hipMemsetAsync(c->totals.p, 0, 4, c->stream));
    c->mxyz.ensure((size_t)std::max<int64_t>(n, 1));
    launch_morton_keys(cl->pristine.view(n), cl->amax[0], cl->amax[1], cl->amax[2], k0.p, i0.p,
                       c->totals.p, c->mxyz.p, c->stream, c->opt.spatial_curve == 1);
    HIPCHK(morton_sort(tmp.p, tb, k0.p, k1.p, i0.p, i1.p, n, c->stream));
    int32_t nonfinite = 0;
    HIPCHK(hipMemcpyAsync(&nonfinite, c->totals.p, 4, hipMemcpyDeviceToHost, c->stream));
    sync(c);
    const int64_t m = n - nonfinite;
    cl->sp_pristine.ensure((size_t)std::max<int64_t>(m, 1));
    launch_gather_order(c->mxyz.p, i1.p, m, cl->sp_pristine.out(), c->stream);
    cl->sp_order.ensure((size_t)std::max<int64_t>(m, 1));
    if (m > 0)
      HIPCHK(hipMemcpyAsync(cl->sp_order.p, i1.p, (size_t)m * 4, hipMemcpyDeviceToDevice, c->stream));
    if (cl->has_normals) {
      cl->sp_pristine.ensure_nrm((size_t)std::max<int64_t>(m, 1));
      launch_gather_nrm(cl->pristine.nrm.p, cl->sp_order.p, m, cl->sp_pristine.nrm.p, c->stream);
    }
    cl->sp_tiles_pr.ensure((size_t)std::max<int64_t>(sp_tiles(m), 1));
    cl->sp_supers_pr.ensure((size_t)std::max<int64_t>(sp_supers(m), 1));
    launch_sphere_bounds(cl->sp_pristine.x.p, cl->sp_pristine.y.p, cl->sp_pristine.z.p, m, nullptr,
                         cl->sp_tiles_pr.p, cl->sp_supers_pr.p, c->stream);
    HIPCHK(hipGetLastError());
    // (no synchronisation: everything that reads the copy is queued behind it on the stream;
    // the scratch above is only rewritten by the next build, on the same stream)
    cl->sp_n_pristine = cl->sp_n = m;
    cl->sp_built = cl->sp_valid = true;
    cl->sp_cur = -1;
    cl->sp_dirty = false;
  }
}

SpatialView spatial_view(const dlg_cloud* cl) {
  const SoA& s = cl->sp_soa();
  const bool pr = cl->sp_cur < 0;
  return SpatialView{s.x.p, s.y.p, s.z.p, cl->sp_n, pr ? cl->sp_tiles_pr.p : cl->sp_tb[cl->sp_cur].p,
                     pr ? cl->sp_supers_pr.p : cl->sp_sb[cl->sp_cur].p};
}

// (re)compute the sphere bounds of the working spatial copy when they are stale
void ensure_sphere_bounds(dlg_ctx* c, dlg_cloud* cl) {
  if (cl->sp_dirty && cl->sp_cur >= 0 && cl->sp_n > 0) {
    const int b = cl->sp_cur;
    cl->sp_tb[b].ensure((size_t)std::max<int64_t>(sp_tiles(cl->sp_n), 1));
    cl->sp_sb[b].ensure((size_t)std::max<int64_t>(sp_supers(cl->sp_n), 1));
    const SoA& s = cl->sp_soa();
    launch_sphere_bounds(s.x.p, s.y.p, s.z.p, cl->sp_n, nullptr, cl->sp_tb[b].p, cl->sp_sb[b].p,
                         c->stream);
  }
  cl->sp_dirty = false;
}

// a lean list's coordinates (and ids, normals) from the pristine copy, before any path that
// reads them
void ensure_list_xyz(dlg_ctx* c, dlg_cloud* cl) {
  if (!cl->list_lean()) return;
  SoA& b = cl->buf[cl->cur];
  if (cl->pristine.with_nrm) b.ensure_nrm((size_t)std::max<int64_t>(cl->n_active, 1));
  PointsOut io = b.out();
  if (!cl->pristine.with_nrm) io.nrm = nullptr;
  launch_list_materialize(cl->pristine.view(cl->n_total), cl->n_active, io, c->stream);
  HIPCHK(hipGetLastError());
  cl->buf_lean[cl->cur] = false;
}

void ensure_sel1(dlg_ctx* c, int64_t n, int64_t min_tiles = 0) {
  const size_t nt = (size_t)std::max<int64_t>(sel1_tiles(n), min_tiles) + 1;
  if (nt > c->sel1_status.cap) {
    c->sel1_status.ensure(nt);
    HIPCHK(hipMemsetAsync(c->sel1_status.p, 0, sizeof(uint64_t) * c->sel1_status.cap, c->stream));
  }
  if (!c->sel1_err.p) {
    c->sel1_err.ensure(1);
    HIPCHK(hipMemsetAsync(c->sel1_err.p, 0, sizeof(int32_t), c->stream));
  }
  if (!c->sel1_tk.p) {
    c->sel1_tk.ensure(1);
    HIPCHK(hipMemsetAsync(c->sel1_tk.p, 0, sizeof(uint64_t), c->stream));
    c->sel1.issued = 0;
  }
  c->sel1.status = c->sel1_status.p;
  c->sel1.err = c->sel1_err.p;
  // (tickets whenever another context of this process may run its selects on the same device
  // at once: with the device to itself a launch's tiles complete in workgroup-index order)
  const bool tk = c->opt.sel1_ticket == 1 || (c->opt.sel1_ticket == -1 && ctx_shared(c->device));
  c->sel1.ticket = tk ? reinterpret_cast<unsigned long long*>(c->sel1_tk.p) : nullptr;
}

void ensure_mom_done(dlg_ctx* c) {
  if (c->mom_done.p) return;
  c->mom_done.ensure(1);
  HIPCHK(hipMemsetAsync(c->mom_done.p, 0, sizeof(unsigned), c->stream));
}

// one SACSegmentation::segment() over the cloud's active list (all ranks)
// active_ranks: every rank's active count when the caller already knows it (the extract loop
// carries it from the previous round's survivors), else allgathered here
SegOut segment_impl(dlg_ctx* c, dlg_cloud* cl, const dlg_sac_params& prm, bool compact,
                    dlg_sac_stats* st, dlg_extract_stats* xs,
                    const std::vector<int64_t>* active_ranks = nullptr) {
  SegOut out;
  std::memset(st, 0, sizeof(*st));
  const bool np = prm.model == DLG_SACMODEL_NORMAL_PLANE;
  if (prm.model != DLG_SACMODEL_PLANE && !np)
    throw DlgError(DLG_ERR_INVALID, "model must be SACMODEL_PLANE or SACMODEL_NORMAL_PLANE");
  if (np && !cl->has_normals)  // PCL: "No input dataset containing normals was given!"
    throw DlgError(DLG_ERR_INVALID, "SACMODEL_NORMAL_PLANE needs normals (dlg_cloud_set_normals)");
  if (!(prm.threshold == prm.threshold)) throw DlgError(DLG_ERR_INVALID, "threshold is NaN");
  const int cap_h = prm.hypotheses_per_launch > 0
                        ? std::min(prm.hypotheses_per_launch, kMaxHypPerLaunch)
                        : kMaxHypPerLaunch;
  std::vector<int64_t> per_rank;
  int64_t N = 0;
  if (active_ranks && (int)active_ranks->size() == c->comm->world() &&
      (*active_ranks)[c->comm->rank()] == cl->n_active) {
    per_rank = *active_ranks;
    for (int64_t v : per_rank) N += v;
  } else {
    N = allgather_i64(c, cl->n_active, &per_rank);
  }
  int64_t offset = 0;
  for (int r = 0; r < c->comm->rank(); ++r) offset += per_rank[r];
  st->n_active = N;
  if (N > INT32_MAX) throw DlgError(DLG_ERR_INVALID, "more than 2^31-1 active points");
  if (prm.threshold == DBL_MAX) return out;  // PCL: "No threshold set!" -> computeModel false
  if (N < 3) return out;                      // getSamples: cannot select 3 unique points

  // lean-list round: plane model over the Morton copy, device refit, a list that is pristine or
  // already lean (a list compacted with coordinates stays on the full path); any rank count
  // (below)
  const bool pcl_refit = prm.optimize && prm.refit_mode != DLG_REFIT_FAST;
  // PCL's float sums on the device (fsum.hip; several ranks: each walks its segment of the list
  // from the previous rank's end values); lean rounds take the unrefined inliers in list order
  // from a bitmap over pristine indices instead of list coordinates
  const bool pcl_dev = pcl_refit && c->opt.pcl_dev != 0;
  // (any rank count: the fast refit's moments are exact integers, so summing them over the
  // Morton copies of the shards gives the list's bits.  Every rank decides alike: whether all
  // ranks hold a spatial copy is agreed once per extraction (c->sp_all), and the other inputs
  // -- the list lean, NORMAL_PLANE rounds dropping the copy -- evolve identically on every rank)
  // NORMAL_PLANE over the Morton copy: the prefilter d_euclid < lim(w) holds for the cloud's
  // largest w = lambda (1 - min curvature) when every w lies in [0, 1) (then lim is finite and
  // monotone in w); NaN curvatures never pass PCL's test.  Otherwise the exhaustive kernel.
  float np_lim = INFINITY;
  if (np && cl->curv_known) {
    const double w_max = prm.normal_distance_weight * (1.0 - (double)cl->curv_min);
    const double w_min = prm.normal_distance_weight * (1.0 - (double)cl->curv_max);
    if (w_min >= 0.0 && w_max < 1.0) np_lim = np_lim_max(w_max, prm.threshold);
  }
  // (NORMAL_PLANE: only with the pruned NP scorer -- every w in [0, 1), the copy carrying normals)
  const bool np_lean_ok = !np || (cl->sp_valid && cl->sp_soa().with_nrm && c->opt.prune_np &&
                                  np_lim < INFINITY);
  const bool lean = compact && np_lean_ok && (!pcl_refit || pcl_dev) && c->opt.lean && cl->sp_valid &&
                    c->sp_all &&
                    cl->n_total < (int64_t(1) << 30) && c->opt.prune != 0 &&
                    (cl->cur < 0 || cl->buf_lean[cl->cur]);
  if (!lean) ensure_list_xyz(c, cl);
  const PointsView src = cl->view();
  // the lean list's pristine indices (null while the list is the pristine one)
  const int32_t* lidx = lean && cl->cur >= 0 ? cl->buf[cl->cur].gid.p : nullptr;
  const float cthr = thr_ceil(prm.threshold);
  ModelTest mt;
  mt.cthr = cthr;
  mt.normal_plane = np ? 1 : 0;
  mt.thr = prm.threshold;
  mt.lambda = prm.normal_distance_weight;
  const double t_ctl0 = trace_on() ? now_ms() : 0.0;
  RansacControl ctl(prm, N, cap_h, &c->replay);
  if (trace_on()) std::fprintf(stderr, "[dlg] segment start %.3fms ctl %.3fms\n", t_ctl0 - c->t_tot, now_ms() - t_ctl0);
  // pruned scoring over the spatial copy (plane model, default kernel, spatial copy in step)
  const bool pruned = !np && cl->sp_valid && c->opt.prune != 0;
  const bool pruned_np = np && cl->sp_valid && cl->sp_soa().with_nrm && c->opt.prune != 0 &&
                         c->opt.prune_np && np_lim < INFINITY;
  const float pmargin = pruned ? prune_margin(cthr, cl->amax)
                               : pruned_np ? prune_margin(np_lim, cl->amax) : 0.0f;
  if (pruned || pruned_np) ensure_sphere_bounds(c, cl);
  // device slots: winning HypRec (its first float4 is the plane), its 3 samples, refined plane
  c->small.ensure(16);
  c->h_small.ensure(16);
  HypRec* best_dev = reinterpret_cast<HypRec*>(c->small.p);
  SampleRec* best_smp_dev = reinterpret_cast<SampleRec*>(c->small.p + 2);
  float4* rc_dev = c->small.p + 5;
  const float4* bc_dev = c->small.p;
  int launches = 0;
  // Speculative pick (probability 1): the first batch holds all max_iterations + 1 draws, so
  // k_pick_p1 can take computeModel's decision on the device and the refit + select follow
  // without a host round trip (one sync per round in fast-refit mode, one less in PCL mode).
  // The counts still come back with the round's sync and the host replays them
  // (RansacControl::consume); on any disagreement, or when the loop needs more draws (bad
  // samples), the round continues on the exact host path and the refit + select are redone.
  const bool spec = c->opt.spec_pick && prm.probability == 1.0 && prm.max_iterations >= 0 &&
                    (int64_t)prm.max_iterations + 1 <= cap_h;
  c->pick.ensure(4);
  c->h_pick.ensure(4);
  int spec_D = 0, spec_Dp = 0;
  bool spec_pending = false;

  // one batch of draws: replay, gather, build, score; then either the host replay (sync) or,
  // for the first batch of a speculative round, the device pick
  auto one_batch = [&](bool speculate) {
    const int D = ctl.next_size();
    // ---- host: drawIndexSample over positions
    const double t_draw0 = trace_on() ? now_ms() : 0.0;
    c->h_pos.ensure(3 * (size_t)D);
    int32_t* hp = c->h_pos.p;
    ctl.next_batch(hp);
    const double t_draw1 = trace_on() ? now_ms() : 0.0;
    // ---- device: gather, build, score
    c->pos.ensure(3 * (size_t)D);
    c->samples.ensure(3 * (size_t)D);
    c->hyps.ensure(kHypScratchBytes / sizeof(HypRec) + 1);
    c->res.ensure(2 * (size_t)kMaxHypPerLaunch + 64);
    // res = counts[Dp] | good[D]  (Dp = D rounded up to the 64-hypothesis groups of k_score)
    const int Dp = (D + 63) / 64 * 64;
    if (c->comm->world() == 1) {
      // one launch: positions read from the pinned host buffer (the next round's draw rewrites
      // it only after this round's results were published, i.e. after this kernel ran)
      if (lean)
        launch_gather_build(hp, D, cl->pristine.view(cl->n_total), c->samples.p, cthr,
                            cl->amax[0], cl->amax[1], cl->amax[2], c->hyps.p, c->res.p, c->stream,
                            lidx, src.n);
      else
        launch_gather_build(hp, D, src, c->samples.p, cthr, cl->amax[0], cl->amax[1],
                            cl->amax[2], c->hyps.p, c->res.p, c->stream);
    } else {
      HIPCHK(hipMemcpyAsync(c->pos.p, hp, 12 * (size_t)D, hipMemcpyHostToDevice, c->stream));
      if (lean)
        launch_gather_samples(c->pos.p, 3 * D, offset, cl->pristine.view(cl->n_total),
                              c->samples.p, c->stream, lidx, src.n);
      else
        launch_gather_samples(c->pos.p, 3 * D, offset, src, c->samples.p, c->stream);
      c->comm->allreduce_sum(c->samples.p, 12 * (size_t)D, DType::I32, c->stream);
      launch_build_hyps(c->samples.p, D, cthr, cl->amax[0], cl->amax[1], cl->amax[2], c->hyps.p,
                        c->res.p + Dp, c->stream);
      HIPCHK(hipMemsetAsync(c->res.p, 0, 4 * (size_t)Dp, c->stream));
    }
    // hypothesis sharding: this rank scores hypotheses [h_lo, h_hi) only (slices in whole
    // 64-hypothesis groups, so an exhaustive kernel's padded group never reaches into another
    // rank's slice), the other counts stay zero until the allreduce below
    int h_lo = 0, h_hi = D;
    if (c->hcomm) {
      const int64_t U = Dp / 64, R = c->hcomm->world(), r = c->hcomm->rank();
      h_lo = (int)std::min<int64_t>(D, 64 * (U * r / R));
      h_hi = (int)std::min<int64_t>(D, 64 * (U * (r + 1) / R));
    }
    const int Ds = h_hi - h_lo;
    const HypRec* hyps_s = c->hyps.p + h_lo;
    int32_t* counts_s = c->res.p + h_lo;
    // the pruned scorer records its timing events on its own dispatches (no marker packets)
    const bool ext_ev = c->profiling && (pruned_np || (!np && pruned));
    if (c->profiling && !ext_ev) HIPCHK(hipEventRecord(c->ev[0], c->stream));
    // the speculative pick: fused into the pruned scoring's last workgroup on one rank (at N > 1
    // it needs the allreduced counts: its own launch after the collective)
    PickArgs pk;
    if (speculate) {
      pk.res = c->res.p;
      pk.Dp = Dp;
      pk.D = D;
      pk.need_good = prm.max_iterations + 1;
      pk.hyps = c->hyps.p;
      pk.samples = c->samples.p;
      pk.best = best_dev;
      pk.best_smp = best_smp_dev;
      pk.out = c->pick.p;
    }
    const bool fuse_pick = speculate && (pruned_np || (!np && pruned)) && c->comm->world() == 1 &&
                           !c->hcomm;
    if (fuse_pick) {
      if (!c->pick_done.p) {
        c->pick_done.ensure(1);
        HIPCHK(hipMemsetAsync(c->pick_done.p, 0, sizeof(unsigned), c->stream));
      }
      pk.done = c->pick_done.p;
    }
    if (pruned_np) {
      c->lp.ensure((size_t)sp_supers(cl->sp_n) * prune_list_stride(D) + 1);
      ensure_prune_work(c, sp_supers(cl->sp_n));
      c->np_cn.ensure(kMaxHypPerLaunch);
      const PrunedNp npp{cl->sp_soa().nrm.p, prm.normal_distance_weight, prm.threshold, c->np_cn.p};
      launch_score_pruned(spatial_view(cl), hyps_s, Ds, cthr, pmargin, cl->amax, counts_s,
                          c->lp.p, c->lp_n.p + kPwHeader, c->num_cus, c->stream, prune_stats_ptr(c), &npp,
                          fuse_pick ? &pk : nullptr, ext_ev ? c->ev[0] : nullptr,
                          ext_ev ? c->ev[1] : nullptr, c->opt.tile_scorer);
    } else if (np) {
      if (Ds > 0) launch_score_np(src, hyps_s, Ds, mt, counts_s, c->num_cus, c->stream);
    } else if (pruned) {
      c->lp.ensure((size_t)sp_supers(cl->sp_n) * prune_list_stride(D) + 1);
      ensure_prune_work(c, sp_supers(cl->sp_n));
      launch_score_pruned(spatial_view(cl), hyps_s, Ds, cthr, pmargin, cl->amax, counts_s,
                          c->lp.p, c->lp_n.p + kPwHeader, c->num_cus, c->stream, prune_stats_ptr(c), nullptr,
                          fuse_pick ? &pk : nullptr, ext_ev ? c->ev[0] : nullptr,
                          ext_ev ? c->ev[1] : nullptr, c->opt.tile_scorer);
    } else if (Ds > 0) {
      launch_score(src, hyps_s, Ds, cthr, counts_s, c->opt.score_kernel, c->num_cus, c->stream);
    }
    HIPCHK(hipGetLastError());
    if (c->profiling && !ext_ev) HIPCHK(hipEventRecord(c->ev[1], c->stream));
    if (c->comm->world() > 1) c->comm->allreduce_sum(c->res.p, D, DType::I32, c->stream);
    if (c->hcomm) c->hcomm->allreduce_sum(c->res.p, D, DType::I32, c->stream);
    c->h_res.ensure((size_t)Dp + D);
    ++launches;
    st->tests_scored += (int64_t)D * N;
    if (speculate) {
      // (the counts and the pick come back with the round's totals: a copy here would sit
      // between the scoring and the pick on the stream)
      if (!fuse_pick) launch_pick_p1(pk, c->stream);
      HIPCHK(hipGetLastError());
      spec_pending = true;
      spec_D = D;
      spec_Dp = Dp;
      flush_emit(c);  // the previous round's inlier copy, behind this round's launches
      if (trace_on())
        std::fprintf(stderr, "[dlg] N=%lld D=%d totals->draw=%.3fms draw=%.3fms enqueue=%.3fms (speculative pick)\n",
                     (long long)N, D, c->t_tot > 0 ? t_draw0 - c->t_tot : 0.0, t_draw1 - t_draw0,
                     now_ms() - t_draw1);
      return;
    }
    HIPCHK(hipMemcpyAsync(c->h_res.p, c->res.p, 4 * ((size_t)Dp + D), hipMemcpyDeviceToHost, c->stream));
    const double t_launch = trace_on() ? now_ms() : 0.0;
    flush_emit(c);  // the previous round's inlier copy, behind this round's launches
    sync(c);
    if (trace_on())
      std::fprintf(stderr, "[dlg] N=%lld D=%d totals->draw=%.3fms draw=%.3fms launch=%.3fms score+wait=%.3fms\n",
                   (long long)N, D, c->t_tot > 0 ? t_draw0 - c->t_tot : 0.0, t_draw1 - t_draw0,
                   t_launch - t_draw1, now_ms() - t_launch);
    if (c->profiling) st->score_ms += event_ms(c, 0, 1);
    // ---- host: computeModel replay over the batch
    const int best_d = ctl.consume(c->h_res.p, c->h_res.p + Dp, D);
    if (best_d >= 0) {  // keep the winner on the device (the next batch overwrites hyps)
      HIPCHK(hipMemcpyAsync(best_dev, c->hyps.p + best_d, sizeof(HypRec), hipMemcpyDeviceToDevice,
                            c->stream));
      HIPCHK(hipMemcpyAsync(best_smp_dev, c->samples.p + 3 * best_d, 3 * sizeof(SampleRec),
                            hipMemcpyDeviceToDevice, c->stream));
    }
  };

  // refit + final select (+ compaction of both copies, sphere bounds of the survivors); ends
  // with the round's sync
  const double t_ref0 = trace_on() ? now_ms() : 0.0;
  const int nt = select_tiles(src.n);
  c->tile_in.ensure(nt + 1);
  c->tile_off_in.ensure(nt + 1);
  c->tile_off_out.ensure(nt + 1);
  c->totals.ensure(8);
  c->h_tot.ensure(4);
  c->h_small.ensure(8);
  c->inl_gid.ensure((size_t)std::max<int64_t>(src.n, 1));
  c->moments.ensure(kMomDigits);
  if (!cl->qexp_known && prm.optimize && !pcl_refit) {
    // the fast refit's quantum comes from the largest finite |coordinate| of the whole cloud
    // (all ranks: one max-allreduce per cloud)
    double f = (double)cl->fmax;
    if (c->comm->world() > 1) {
      c->scratch_f64.ensure(1);
      HIPCHK(hipMemcpyAsync(c->scratch_f64.p, &f, 8, hipMemcpyHostToDevice, c->stream));
      c->comm->allreduce_max_f64(c->scratch_f64.p, 1, c->stream);
      HIPCHK(hipMemcpyAsync(&f, c->scratch_f64.p, 8, hipMemcpyDeviceToHost, c->stream));
      sync(c);
    }
    cl->qexp = fast_qexp((float)f);
    cl->qexp_known = true;
  }
  PointsOut dst{};
  if (compact) {
    SoA& sp = cl->buf[cl->spare()];
    sp.ensure((size_t)std::max<int64_t>(src.n, 1));
    if (src.nrm) sp.ensure_nrm((size_t)std::max<int64_t>(src.n, 1));
    dst = sp.out();
  }
  const bool sp_compact = compact && cl->sp_valid && (!np || cl->sp_soa().with_nrm);
  auto sp_cur_view = [&]() {
    const SoA& ss = cl->sp_soa();
    return PointsView{ss.x.p, ss.y.p, ss.z.p, ss.gid.p, cl->sp_n,
                      np && ss.with_nrm ? ss.nrm.p : nullptr};
  };
  if (lean && cl->tag.cap < (size_t)cl->n_total) {
    cl->tag.ensure((size_t)std::max<int64_t>(cl->n_total, 1));
    HIPCHK(hipMemsetAsync(cl->tag.p, 0, cl->tag.cap, c->stream));
    cl->tagv = 0;
  }
  // before the first launch of a round that writes inl_gid: the previous round's inlier copy
  // (copy stream) may still read it.  A stream wait only when the copy is still running (it
  // has almost always landed by then); placed at the writer, not at the round's start, so a
  // wait never sits between the scoring and the refit on the critical path.
  auto stage_wait = [&]() {
    if (!c->stage_inflight) return;
    const hipError_t q = hipEventQuery(c->ev_stage);
    if (q == hipErrorNotReady) HIPCHK(hipStreamWaitEvent(c->stream, c->ev_stage, 0));
    else HIPCHK(q);
    c->stage_inflight = false;
  };
  std::function<void(int)> select_round;
  auto refit_select = [&]() {
    // Fast mode (and no optimisation) never leave the device: moments of the unrefined plane's
    // inliers (k_moments, centred on the winning sample), the double eigen33 refit in a
    // one-thread kernel, then the select with the refined plane read from device memory.  PCL
    // mode needs the host's sequential float sums in between.
    // (tests: DLG_OPT_FAULT_INJECT -- this rank fails here, after the round's scoring
    // collectives, while its peers go on into the refit's and the select's)
    if (xs && c->opt.fault_round > 0 && xs->rounds == c->opt.fault_round - 1)
      throw DlgError(DLG_ERR_INTERNAL, "injected fault (DLG_OPT_FAULT_INJECT) in extract round " +
                                           std::to_string(xs->rounds));
    const int sk = c->sel_k;  // this round's pair of select timing events
    c->walk_rec[sk] = false;
    // the PCL refit walk's timing events (profiling only)
    // (e = 2, 3: k_fs_repair's, which runs on ranks > 0 of a group only)
    c->rep_rec[sk] = false;
    c->mid_rec[sk] = false;
    // (e = 4, 5: the first walk's end and the second's start, ranks > 0 under protocols 0, 2)
    auto walk_ev = [&](int e) -> hipEvent_t {
      if (!c->profiling || !c->walk_events) return nullptr;
      if (e >= 2 && (c->comm->world() == 1 || c->comm->rank() == 0)) return nullptr;
      if (e >= 4 && c->opt.fs_protocol == 1) return nullptr;
      if (!c->ev_walk[sk][e]) HIPCHK(hipEventCreate(&c->ev_walk[sk][e]));
      (e >= 4 ? c->mid_rec : e >= 2 ? c->rep_rec : c->walk_rec)[sk] = true;
      return c->ev_walk[sk][e];
    };
    if (c->profiling) {
      for (auto& ev : c->ev_sel[sk])
        if (!ev) HIPCHK(hipEventCreate(&ev));
      if (spec_pending) {
        // the scoring's end event (just recorded) opens the select phase: no second marker
        std::swap(c->ev[1], c->ev_sel[sk][0]);
        c->ev_score_end = c->ev_sel[sk][0];
      } else {
        HIPCHK(hipEventRecord(c->ev_sel[sk][0], c->stream));
      }
    }
    if (!pcl_refit) {
      const bool one = c->comm->world() == 1;
      if (prm.optimize) {
        // (lean: the moments of the Morton copy -- the same finite inliers -- over the tiles
        // whose sphere may hold one; one rank: the refit in the same launch)
        const PointsView mv = lean ? sp_cur_view() : src;
        const int nb = lean ? moments_sp_blocks(mv.n) : moments_blocks(mv.n);
        c->partials.ensure((size_t)nb * kMomDigits);
        ensure_mom_done(c);
        if (lean) {
          const SpatialView sv = spatial_view(cl);
          launch_moments_sp(mv, sv.tiles, sv.supers, pmargin, bc_dev, mt, cl->qexp, c->partials.p,
                            c->mom_done.p, nb, c->moments.p, one ? rc_dev : nullptr, c->stream);
        } else if (one) {
          launch_moments_refit(mv, bc_dev, mt, cl->qexp, c->partials.p, c->mom_done.p, nb,
                               c->moments.p, rc_dev, c->stream);
        } else {
          launch_moments(mv, bc_dev, mt, cl->qexp, c->partials.p, c->mom_done.p, nb,
                         c->moments.p, c->stream);
        }
      }
      if (!(prm.optimize && one)) {
        // exact integers: the rank sum is the one-rank result, whatever the sharding
        if (prm.optimize) c->comm->allreduce_sum(c->moments.p, kMomDigits, DType::I64, c->stream);
        launch_refit_moments(c->moments.p, cl->qexp, bc_dev, prm.optimize, rc_dev, c->stream);
      }
    } else if (pcl_dev) {
      // PCL float refit on the device: the unrefined plane's inliers in list order, PCL's nine
      // sequential float sums evaluated exactly in parallel (fsum.hip), the float eigen33; the
      // refined plane stays on the device (no host round trip)
      if (c->fs_cap < src.n) {
        const int64_t cap = std::max<int64_t>(src.n, 1);
        c->fs_scr.ensure(fs_scratch_bytes(cap, c->comm->world()));
        c->fs_b = fs_carve(c->fs_scr.p, cap, c->comm->world());
        HIPCHK(fs_reset(c->fs_b, c->stream, c->opt.fs_poison));
        c->fs_cap = cap;
      }
      int32_t* fs_res = reinterpret_cast<int32_t*>(c->small.p + 8);
      int repairs = 0;
      if (lean) {
        // the unrefined plane's inliers' x, y, z in list order (= ascending pristine order):
        // one pass over the active list (k_ulist), or (DLG_OPT_UNREFINED_LIST 0) stamped into a
        // bitmap over pristine indices from the Morton copy's near tiles and compacted from it
        const int64_t nw = (cl->n_total + 31) / 32;
        c->fs_x.ensure((size_t)std::max<int64_t>(src.n, 1));
        c->fs_y.ensure((size_t)std::max<int64_t>(src.n, 1));
        c->fs_z.ensure((size_t)std::max<int64_t>(src.n, 1));
        c->fs_n.ensure(1);
        if (c->opt.unrefined_list) {
          ensure_sel1(c, std::max<int64_t>(src.n, cl->sp_n));
          launch_ulist(lidx, src.n, cl->pristine.view(cl->n_total), bc_dev, mt, c->sel1,
                       c->fs_x.p, c->fs_y.p, c->fs_z.p, c->fs_n.p, c->stream);
          HIPCHK(hipGetLastError());
        } else {
          if (cl->ubits.cap < (size_t)nw + 16 || cl->ubits_dirty) {
            // (new, or left stamped by an extraction that failed between the stamp and the
            // compaction, which clears every word it reads)
            cl->ubits.ensure((size_t)nw + 16);
            HIPCHK(hipMemsetAsync(cl->ubits.p, 0, cl->ubits.cap * sizeof(uint32_t), c->stream));
            cl->ubits_dirty = false;
          }
          ensure_sel1(c, std::max<int64_t>(src.n, cl->sp_n), ucompact_tiles(nw));
          const SpatialView sv = spatial_view(cl);
          cl->ubits_dirty = true;
          launch_ustamp(sp_cur_view(), sv.tiles, sv.supers, pmargin, bc_dev, mt, cl->ubits.p,
                        c->stream);
          launch_ucompact(cl->ubits.p, nw, cl->pristine.view(cl->n_total), c->sel1, c->fs_x.p,
                          c->fs_y.p, c->fs_z.p, c->fs_n.p, c->stream);
          HIPCHK(hipGetLastError());
          cl->ubits_dirty = false;
        }
        launch_fs_refit(c->fs_x.p, c->fs_y.p, c->fs_z.p, 1, c->fs_n.p, src.n, c->fs_b, bc_dev,
                        rc_dev, fs_res, c->num_cus, c->stream, c->comm.get(), walk_ev(0),
                        walk_ev(1), walk_ev(2), walk_ev(3), c->opt.fs_protocol, &repairs,
                        c->opt.fs_segments, walk_ev(4), walk_ev(5), c->opt.fs_join);
      } else {
        c->inl_xyz.ensure(3 * (size_t)std::max<int64_t>(src.n, 1));
        stage_wait();
        launch_select(src, bc_dev, mt, c->tile_in.p, c->tile_off_in.p, c->tile_off_out.p,
                      c->totals.p, c->inl_gid.p, c->inl_xyz.p, nullptr, c->stream);
        launch_fs_refit(c->inl_xyz.p, c->inl_xyz.p + 1, c->inl_xyz.p + 2, 3, c->totals.p, src.n,
                        c->fs_b, bc_dev, rc_dev, fs_res, c->num_cus, c->stream, c->comm.get(),
                        walk_ev(0), walk_ev(1), walk_ev(2), walk_ev(3), c->opt.fs_protocol,
                        &repairs, c->opt.fs_segments, walk_ev(4), walk_ev(5), c->opt.fs_join);
      }
      HIPCHK(hipGetLastError());
      if (xs) xs->refit_repairs += repairs;
    } else {
      // PCL float refit: inlier xyz in global list order -> sequential float sums on the host
      c->inl_xyz.ensure(3 * (size_t)std::max<int64_t>(src.n, 1));
      stage_wait();
      launch_select(src, bc_dev, mt, c->tile_in.p, c->tile_off_in.p, c->tile_off_out.p, c->totals.p,
                    c->inl_gid.p, c->inl_xyz.p, nullptr, c->stream);
      HIPCHK(hipMemcpyAsync(c->h_tot.p, c->totals.p, 8, hipMemcpyDeviceToHost, c->stream));
      HIPCHK(hipMemcpyAsync(c->h_small.p, c->small.p, 5 * sizeof(float4), hipMemcpyDeviceToHost,
                            c->stream));
      sync(c);
      const HypRec* bh = reinterpret_cast<const HypRec*>(c->h_small.p);
      const float bc[4] = {bh->a, bh->b, bh->c, bh->d};
      std::vector<int32_t> xyz_bits;
      gather_lists(c, reinterpret_cast<const int32_t*>(c->inl_xyz.p), c->h_tot.p[0], 3, &xyz_bits);
      float rc[4];
      refit_pcl_float(reinterpret_cast<const float*>(xyz_bits.data()), (int64_t)xyz_bits.size() / 3,
                      bc, rc);
      c->h_small.p[5] = make_float4(rc[0], rc[1], rc[2], rc[3]);
      HIPCHK(hipMemcpyAsync(rc_dev, c->h_small.p + 5, sizeof(float4), hipMemcpyHostToDevice,
                            c->stream));
    }
    select_round(sk);
    if (pcl_dev) {
      // an eigen33 transcendental the device could not round for certain (a double result within
      // 2^-46 of a float rounding boundary): the host's value from the published sums decides,
      // and the select is redone when it differs (DLG_OPT_PCL_REFIT_DEVICE 2 / 3: every round)
      const int32_t* fr = reinterpret_cast<const int32_t*>(c->h_small.p + 8);
      if (fr[0] != 0 || c->opt.pcl_dev >= 2) {
        ++c->fs_checks;
        if (xs) xs->pcl_host_checks++;
        float a9[9], rh[4];
        std::memcpy(a9, fr + 2, sizeof(a9));
        const HypRec* bh = reinterpret_cast<const HypRec*>(c->h_small.p);
        const float cin[4] = {bh->a, bh->b, bh->c, bh->d};
        fs_refit_tail_plain(a9, fr[1], cin, rh);
        const float4 rd = c->h_small.p[5];
        if (std::memcmp(rh, &rd, sizeof(rh)) != 0 || c->opt.pcl_dev == 3) {
          ++c->fs_fixes;
          c->h_small.p[15] = make_float4(rh[0], rh[1], rh[2], rh[3]);
          HIPCHK(hipMemcpyAsync(rc_dev, c->h_small.p + 15, sizeof(float4), hipMemcpyHostToDevice,
                                c->stream));
          // (the first select wrote only spare buffers and stamps under its own tag: redone
          // outright; its timing is not kept)
          const bool prof = c->profiling;
          c->profiling = false;
          select_round(c->sel_k);
          c->profiling = prof;
        }
      }
    }
  };
  // final selectWithinDistance with the refined plane at rc_dev (+ compaction, publish, wait)
  select_round = [&](int sk) {
    // final selectWithinDistance with the refined model: the head (counts + scan) makes the
    // round's totals final, they are published right away, and the scatters (inlier ids,
    // survivors of both copies) and the sphere bounds run while the host reads them and draws
    // the next round
    // (lean: the Morton copy's single-pass select makes the totals final and stamps the inliers;
    // on one rank its last tile publishes the round too)
    const int W = c->comm->world();
    // the round's results into the coherent pinned buffer + a sequence number the host spins on
    // (totals[2..3] still hold the previous compaction's Morton-copy totals: checked below)
    const bool with_counts = spec_pending;
    const int nres = with_counts ? spec_Dp + spec_D : 0;
    const size_t need = (size_t)kPubRk + (W > 1 ? 2 * (size_t)W : 0) + (size_t)nres;
    if (need > c->pub_cap) {
      if (c->pub) HIPCHK(hipHostFree(c->pub));
      c->pub = nullptr;
      c->pub_cap = 0;
      HIPCHK(hipHostMalloc(reinterpret_cast<void**>(&c->pub), std::max<size_t>(need, 16384) * 4,
                           hipHostMallocCoherent));
      c->pub_cap = std::max<size_t>(need, 16384);
      c->pub[0] = 0;
    }
    if (W > 1) {
      c->rk.ensure(2 * (size_t)W + 2);
      c->h_rk.ensure(2 * (size_t)W + 2);
    }
    const int32_t seq = ++c->pub_seq == 0 ? ++c->pub_seq : c->pub_seq;
    PubArgs pa;
    pa.totals = c->totals.p;
    pa.ntot = 4;
    pa.small = c->small.p;
    pa.nsmall = pcl_dev ? 12 : 6;  // (+ the device PCL refit's flag, count and sums: small[8..11])
    pa.rk = W > 1 ? c->rk.p : nullptr;
    pa.nrk = W > 1 ? 2 * W : 0;
    pa.pick = with_counts ? c->pick.p : nullptr;
    pa.npick = with_counts ? 2 : 0;
    pa.res = with_counts ? c->res.p : nullptr;
    pa.nres = nres;
    pa.err = c->sel1_err.p;
    pa.pub = c->pub;
    pa.seq = seq;
    const bool fused_pub = lean && W == 1;
    if (lean) {
      if (++cl->tagv > 255) {
        HIPCHK(hipMemsetAsync(cl->tag.p, 0, (size_t)cl->n_total, c->stream));
        cl->tagv = 1;
      }
      ensure_sel1(c, std::max<int64_t>(src.n, cl->sp_n));
      pa.err = c->sel1_err.p;
      SoA& sd = cl->sp_buf[cl->sp_spare()];
      sd.ensure((size_t)std::max<int64_t>(cl->sp_n, 1));
      const SoA& ss = cl->sp_soa();
      if (ss.with_nrm) sd.ensure_nrm((size_t)std::max<int64_t>(cl->sp_n, 1));
      PointsOut spo = sd.out();
      PointsView spv = sp_cur_view();
      if (ss.with_nrm) spv.nrm = ss.nrm.p;  // (a later NORMAL_PLANE round reads them)
      else spo.nrm = nullptr;
      launch_sel1_morton(spv, rc_dev, mt, c->sel1, cl->tag.p, (uint8_t)cl->tagv, spo, src.n,
                         c->totals.p, c->stream, fused_pub ? &pa : nullptr, c->opt.sel1_tile);
    } else {
      launch_select_head(src, rc_dev, mt, c->tile_in.p, c->tile_off_in.p, c->tile_off_out.p,
                         c->totals.p, c->stream);
    }
    HIPCHK(hipGetLastError());
    if (W > 1)  // every rank's (in, out): the extract loop needs no host-synced allgather
      c->comm->allgather(c->totals.p, c->rk.p, 2, DType::I32, c->stream);
    if (!fused_pub) launch_publish(pa, c->stream);
    HIPCHK(hipGetLastError());
    spec_pending = false;
    if (lean) {
      // the list from the stamps (ids in list order; survivors' pristine indices), then the
      // sphere bounds of the Morton survivors (count in totals[4]).  DLG_OPT_BOUNDS_STREAM: the
      // bounds on a second stream beside the list pass (independent passes over different
      // buffers; forked after the Morton select, joined before anything later on the stream).
      // (Round 5 dropped it after an 8-context loopback run hung; the cause was the single-pass
      // selects' look-back, not the stream: DESIGN.md §6.)
      const int b = cl->sp_spare();
      SoA& sd = cl->sp_buf[b];
      cl->sp_tb[b].ensure((size_t)std::max<int64_t>(sp_tiles(cl->sp_n), 1));
      cl->sp_sb[b].ensure((size_t)std::max<int64_t>(sp_supers(cl->sp_n), 1));
      const bool side = c->opt.bounds_stream;
      if (side) {
        if (!c->sstream) {
          HIPCHK(hipStreamCreateWithFlags(&c->sstream, hipStreamNonBlocking));
          HIPCHK(hipEventCreateWithFlags(&c->ev_fork, hipEventDisableTiming));
          HIPCHK(hipEventCreateWithFlags(&c->ev_join, hipEventDisableTiming));
        }
        HIPCHK(hipEventRecord(c->ev_fork, c->stream));
        HIPCHK(hipStreamWaitEvent(c->sstream, c->ev_fork, 0));
        launch_sphere_bounds(sd.x.p, sd.y.p, sd.z.p, cl->sp_n, c->totals.p + 4, cl->sp_tb[b].p,
                             cl->sp_sb[b].p, c->sstream);
        HIPCHK(hipEventRecord(c->ev_join, c->sstream));
      }
      stage_wait();
      launch_sel1_list(lidx, src.n, cl->tag.p, (uint8_t)cl->tagv,
                       cl->gid_ident ? nullptr : cl->pristine.gid.p, cl->id_base, c->sel1,
                       c->inl_gid.p, dst.gid, c->totals.p + 2, c->stream, c->opt.sel1_tile);
      if (side) HIPCHK(hipStreamWaitEvent(c->stream, c->ev_join, 0));
      else
        launch_sphere_bounds(sd.x.p, sd.y.p, sd.z.p, cl->sp_n, c->totals.p + 4, cl->sp_tb[b].p,
                             cl->sp_sb[b].p, c->stream);
    } else {
      stage_wait();
      launch_select_tail(src, rc_dev, mt, c->tile_off_in.p, c->tile_off_out.p, c->inl_gid.p,
                         nullptr, compact ? &dst : nullptr, c->stream);
    }
    // the Morton copy loses the same points (same predicate, same float inputs): its totals
    // land in totals[2..3], checked at the next publish / the end of the extraction
    if (sp_compact && !lean) {
      SoA& sd = cl->sp_buf[cl->sp_spare()];
      sd.ensure((size_t)std::max<int64_t>(cl->sp_n, 1));
      const SoA& ss = cl->sp_soa();
      if (ss.with_nrm) sd.ensure_nrm((size_t)std::max<int64_t>(cl->sp_n, 1));
      PointsOut spo = sd.out();
      if (!ss.with_nrm) spo.nrm = nullptr;  // (normals travel only when the source has them)
      const PointsView spv{ss.x.p, ss.y.p, ss.z.p, ss.gid.p, cl->sp_n,
                           ss.with_nrm ? ss.nrm.p : nullptr};
      launch_select(spv, rc_dev, mt, c->tile_in.p, c->tile_off_in.p, c->tile_off_out.p,
                    c->totals.p + 2, nullptr, nullptr, &spo, c->stream);
      // sphere bounds of the survivors, into the spare buffer's own bound arrays (sized for
      // the current count, an upper bound; the kernel reads the survivor count from
      // totals[3]), so a round whose plane is rejected leaves the current bounds intact
      const int b = cl->sp_spare();
      cl->sp_tb[b].ensure((size_t)std::max<int64_t>(sp_tiles(cl->sp_n), 1));
      cl->sp_sb[b].ensure((size_t)std::max<int64_t>(sp_supers(cl->sp_n), 1));
      launch_sphere_bounds(sd.x.p, sd.y.p, sd.z.p, cl->sp_n, c->totals.p + 3, cl->sp_tb[b].p,
                           cl->sp_sb[b].p, c->stream);
    }
    HIPCHK(hipGetLastError());
    // one marker at the end of the round's work: inl_gid is final there (flush_emit's copy waits
    // for it) and, when profiling, it closes the select phase.  (The GPU then waits for the
    // host's next draw anyway.)
    c->ev_inl_cur = c->profiling ? c->ev_sel[sk][1] : c->ev_inl;
    HIPCHK(hipEventRecord(c->ev_inl_cur, c->stream));
    const double t_wait0 = trace_on() ? now_ms() : 0.0;
    wait_published(c, seq);
    if (trace_on())
      std::fprintf(stderr, "[dlg] select enqueue=%.3fms wait=%.3fms\n", t_wait0 - t_ref0, now_ms() - t_wait0);
    if (trace_on()) c->t_tot = now_ms();
    std::memcpy(c->h_tot.p, c->pub + kPubTot, 16);
    if (c->pub[kPubErr] != 0) sel1_failed(c);  // (this round's or the last list pass's look-back)
    std::memcpy(c->h_small.p, c->pub + kPubSmall, (size_t)pa.nsmall * sizeof(float4));
    if (W > 1) std::memcpy(c->h_rk.p, c->pub + kPubRk, 8 * (size_t)W);
    check_sp_totals(c, c->h_tot.p + 2);
    if (with_counts) {
      std::memcpy(c->h_pick.p, c->pub + kPubPick, 8);
      std::memcpy(c->h_res.p, c->pub + kPubRk + (W > 1 ? 2 * W : 0), 4 * (size_t)nres);
    }
    // the previous round's select events precede this publish on the stream: complete now
    if (c->sel_pending) {
      float ms = 0.f;
      HIPCHK(hipEventElapsedTime(&ms, c->ev_sel[sk ^ 1][0], c->ev_sel[sk ^ 1][1]));
      c->sel_pending->select_ms += ms;
      add_walk_ms(c, sk ^ 1);
      c->sel_pending = nullptr;
    }
    if (c->profiling && xs) c->sel_pending = xs;  // this round's: read at the next publish / end
    c->sel_k = sk ^ 1;
  };

  bool selected = false;
  if (spec && !ctl.done()) {
    one_batch(true);
    refit_select();  // on the device's pick
    selected = true;
    // the exact host replay of the same counts
    if (c->profiling) {
      float ms = 0.f;
      HIPCHK(hipEventElapsedTime(&ms, c->ev[0], c->ev_score_end));
      st->score_ms += ms;
    }
    const int best_d = ctl.consume(c->h_res.p, c->h_res.p + spec_Dp, spec_D);
    if (!(ctl.done() && best_d == c->h_pick.p[0] && c->h_pick.p[1] == 1)) {
      ++c->spec_misses;
      if (xs) xs->spec_misses++;
      if (trace_on())
        std::fprintf(stderr, "[dlg] speculative pick overturned: host %d done %d, device %d complete %d\n",
                     best_d, ctl.done() ? 1 : 0, c->h_pick.p[0], c->h_pick.p[1]);
      selected = false;
      if (best_d >= 0) {
        HIPCHK(hipMemcpyAsync(best_dev, c->hyps.p + best_d, sizeof(HypRec), hipMemcpyDeviceToDevice,
                              c->stream));
        HIPCHK(hipMemcpyAsync(best_smp_dev, c->samples.p + 3 * best_d, 3 * sizeof(SampleRec),
                              hipMemcpyDeviceToDevice, c->stream));
      }
    }
  }
  while (!ctl.done()) one_batch(false);
  const int iterations = ctl.iterations();
  const bool have = ctl.have_model();
  const int best = ctl.best_count();
  st->draws = ctl.draws();
  st->tests = ctl.tests();
  st->iterations = iterations;
  st->launches = launches;
  if (xs) {
    xs->tests += st->tests;
    xs->tests_scored += st->tests_scored;
    xs->score_launches += launches;
    xs->score_ms += st->score_ms;
  }
  if (!have) return out;

  st->has_model = 1;
  st->n_unrefined = best;
  if (!selected) refit_select();
  const HypRec* bh = reinterpret_cast<const HypRec*>(c->h_small.p);
  const SampleRec* bs = reinterpret_cast<const SampleRec*>(c->h_small.p + 2);
  const float4 rc = c->h_small.p[5];
  st->coeff_unrefined[0] = bh->a; st->coeff_unrefined[1] = bh->b;
  st->coeff_unrefined[2] = bh->c; st->coeff_unrefined[3] = bh->d;
  for (int i = 0; i < 3; ++i) st->best_sample[i] = bs[i].gid;
  out.coeff[0] = rc.x; out.coeff[1] = rc.y; out.coeff[2] = rc.z; out.coeff[3] = rc.w;
  out.has_model = true;
  out.n_in_local = c->h_tot.p[0];
  out.n_out_local = src.n == 0 ? 0 : c->h_tot.p[1];
  {
    const int W = c->comm->world();
    out.in_ranks.assign(W, 0);
    out.out_ranks.assign(W, 0);
    for (int r = 0; r < W; ++r) {
      // (a rank with no active points skips its select kernels: its totals are zero)
      const bool empty = per_rank[r] == 0;
      out.in_ranks[r] = W == 1 ? out.n_in_local : (empty ? 0 : c->h_rk.p[2 * r]);
      out.out_ranks[r] = W == 1 ? out.n_out_local : (empty ? 0 : c->h_rk.p[2 * r + 1]);
    }
    out.n_in_global = 0;
    for (int64_t v : out.in_ranks) out.n_in_global += v;
  }
  if (lean) {
    // the Morton copy decided the inliers; the list pass's own totals (totals[2..3]) must agree
    // with them (checked at the next publish, check_sp_totals)
    out.lean = true;
    out.sp_compacted = true;
    out.sp_n_out = cl->sp_n - out.n_in_local;
    c->sp_expect_in = out.n_in_local;
    c->sp_expect_out = out.n_out_local;
    c->sp_check = out.n_in_local != 0 || out.n_out_local != 0;
  } else if (sp_compact) {
    // non-finite points are never inliers: the Morton copy loses exactly the list's inliers
    // (its own totals are checked at the next publish, check_sp_totals)
    out.sp_compacted = true;
    out.sp_n_out = cl->sp_n - out.n_in_local;
    c->sp_expect_in = cl->sp_n == 0 ? 0 : out.n_in_local;
    c->sp_expect_out = out.sp_n_out;
    c->sp_check = true;
  }
  if (trace_on())
    std::fprintf(stderr, "[dlg] refit+select=%.3fms n_in=%lld\n", now_ms() - t_ref0,
                 (long long)out.n_in_local);
  return out;
}

// DLG_OPT_SYNC_CHECK: every rank's view of the round just run -- (round, model, global inliers,
// coefficient bits, collectives issued so far) -- allgathered and compared; the first rank that
// differs from rank 0 fails the call on every rank (and, through guarded_group, nothing waits)
void check_in_step(dlg_ctx* c, int round, const SegOut& so) {
  Comm* g = c->group();
  const int W = g->world();
  if (W == 1) return;
  constexpr int K = 5;
  int64_t mine[K];
  uint32_t cb[4];
  std::memcpy(cb, so.coeff, sizeof(cb));
  mine[0] = round;
  mine[1] = so.has_model ? so.n_in_global : -1;
  mine[2] = (int64_t)(((uint64_t)cb[0] << 32) | cb[1]);
  mine[3] = (int64_t)(((uint64_t)cb[2] << 32) | cb[3]);
  mine[4] = (int64_t)g->ops();
  c->gath64.ensure((size_t)K * (W + 1));
  c->h_g64.ensure((size_t)K * W);
  HIPCHK(hipMemcpyAsync(c->gath64.p + (size_t)K * W, mine, sizeof(mine), hipMemcpyHostToDevice,
                        c->stream));
  g->allgather(c->gath64.p + (size_t)K * W, c->gath64.p, K, DType::I64, c->stream);
  HIPCHK(hipMemcpyAsync(c->h_g64.p, c->gath64.p, sizeof(mine) * W, hipMemcpyDeviceToHost,
                        c->stream));
  sync(c);
  static const char* what[K] = {"round", "inliers", "coefficients", "coefficients", "collectives"};
  for (int r = 1; r < W; ++r)
    for (int k = 0; k < K; ++k)
      if (c->h_g64.p[(size_t)K * r + k] != c->h_g64.p[k])
        throw DlgError(DLG_ERR_INTERNAL,
                       "ranks diverged in extract round " + std::to_string(round) + ": rank " +
                           std::to_string(r) + "'s " + what[k] + " " +
                           std::to_string(c->h_g64.p[(size_t)K * r + k]) + " vs rank 0's " +
                           std::to_string(c->h_g64.p[k]));
}

// copy this rank's (or every rank's) refined inliers to the caller buffer
int64_t emit_inliers(dlg_ctx* c, const SegOut& so, bool gather, int32_t* dst, int64_t cap,
                     int64_t* global_count, bool deferred = false, bool counts_known = false) {
  if (gather && c->comm->world() > 1) {
    gather_lists(c, c->inl_gid.p, so.n_in_local, 1, &c->h_inl);
    int64_t n = (int64_t)c->h_inl.size();
    *global_count = n;
    if (n > cap) throw DlgError(DLG_ERR_CAPACITY, "inlier buffer too small: need " + std::to_string(n));
    if (n) std::memcpy(dst, c->h_inl.data(), (size_t)n * 4);
    return n;
  }
  if (counts_known) {
    *global_count = so.n_in_global;
  } else {
    std::vector<int64_t> all;
    *global_count = allgather_i64(c, so.n_in_local, &all);
  }
  if (so.n_in_local > cap)
    throw DlgError(DLG_ERR_CAPACITY, "inlier buffer too small: need " + std::to_string(so.n_in_local));
  if (so.n_in_local) {
    if (deferred) {
      // (copied by flush_emit after the next round's launches, or at the end of the loop)
      flush_emit(c);
      c->emit_dst = dst;
      c->emit_n = so.n_in_local;
    } else {
      HIPCHK(hipMemcpyAsync(dst, c->inl_gid.p, (size_t)so.n_in_local * 4, hipMemcpyDeviceToHost,
                            c->stream));
      sync(c);
    }
  }
  return so.n_in_local;
}

std::string g_last_create_error;

std::mutex g_ctx_mu;
std::map<int, int> g_ctx_count;  // live contexts per device

dlg_status init_ctx(dlg_ctx* c, int device) {
  int n = 0;
  hipError_t e = hipGetDeviceCount(&n);
  if (e != hipSuccess || n <= 0)
    return fail(c, DLG_ERR_NO_DEVICE, std::string("no HIP device: ") + hipGetErrorString(e));
  if (device < 0 || device >= n) return fail(c, DLG_ERR_NO_DEVICE, "device index out of range");
  hipDeviceProp_t p;
  if (hipGetDeviceProperties(&p, device) != hipSuccess)
    return fail(c, DLG_ERR_NO_DEVICE, "hipGetDeviceProperties failed");
  if (std::strncmp(p.gcnArchName, "gfx950", 6) != 0)
    return fail(c, DLG_ERR_NO_DEVICE, std::string("built for gfx950, device is ") + p.gcnArchName);
  c->device = device;
  c->num_cus = p.multiProcessorCount;
  return guarded(c, [&] {
    HIPCHK(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
    HIPCHK(hipStreamCreateWithFlags(&c->cstream, hipStreamNonBlocking));
    HIPCHK(hipEventCreateWithFlags(&c->ev_inl, hipEventDisableTiming));
    for (auto& ev : c->ev) HIPCHK(hipEventCreate(&ev));
    ctx_count_add(device, 1);  // (last: a failed init is not counted)
    c->counted = true;
  });
}

}  // namespace

void dlg::ctx_count_add(int device, int delta) {
  std::lock_guard<std::mutex> lk(g_ctx_mu);
  g_ctx_count[device] += delta;
}
bool dlg::ctx_shared(int device) {
  std::lock_guard<std::mutex> lk(g_ctx_mu);
  auto it = g_ctx_count.find(device);
  return it != g_ctx_count.end() && it->second > 1;
}

// normals records on the device (raw_dev: stride_f floats per record, curvature at curv_off,
// indexed by uploaded point (by_pos false) or by pristine position) -> the cloud's normal
// buffers (normalized, + curvature), the Morton copy's, the curvature range; the cloud is reset
void dlg::attach_normals(dlg_ctx* c, dlg_cloud* cl, const float* raw_dev, int64_t stride_f,
                    int curv_off, bool by_pos) {
  {
    cl->cur = -1;  // normals attach to the pristine list: the cloud is reset
    cl->n_active = cl->n_total;
    cl->pristine.ensure_nrm((size_t)std::max<int64_t>(cl->n_total, 1));
    cl->raw_nrm.ensure((size_t)std::max<int64_t>(cl->n_total, 1));
    if (raw_dev && cl->n_total > 0) {
      PointsView pv = cl->pristine.view(cl->n_total);
      if (by_pos) pv.gid = nullptr;
      // the records as given, in pristine order (unless they are that buffer already), then the
      // normalised copy the NORMAL_PLANE model reads
      if (raw_dev != reinterpret_cast<const float*>(cl->raw_nrm.p))
        launch_pack_point_normals(raw_dev, stride_f, curv_off, pv, cl->id_base, cl->raw_nrm.p,
                                  c->stream, false);
      pv.gid = nullptr;
      launch_pack_point_normals(reinterpret_cast<const float*>(cl->raw_nrm.p), 4, 3, pv,
                                cl->id_base, cl->pristine.nrm.p, c->stream, true);
      HIPCHK(hipGetLastError());
      // the Morton copy carries the normals too (pruned NORMAL_PLANE scoring)
      if (cl->sp_built) {
        cl->sp_pristine.ensure_nrm((size_t)std::max<int64_t>(cl->sp_n_pristine, 1));
        launch_gather_nrm(cl->pristine.nrm.p, cl->sp_order.p, cl->sp_n_pristine,
                          cl->sp_pristine.nrm.p, c->stream);
      }
      // curvature range -> the largest w = lambda (1 - curvature) of the cloud
      c->small.ensure(8);
      uint32_t* cr = reinterpret_cast<uint32_t*>(c->small.p + 7);
      launch_curv_range(cl->pristine.nrm.p, cl->n_total, cr, c->stream);
      uint32_t h[2] = {0u, 0u};
      HIPCHK(hipMemcpyAsync(h, cr, 8, hipMemcpyDeviceToHost, c->stream));
      HIPCHK(hipGetLastError());
      sync(c);
      auto ord2f = [](uint32_t o) {
        const uint32_t u = (o & 0x80000000u) ? (o & 0x7FFFFFFFu) : ~o;
        float f;
        std::memcpy(&f, &u, 4);
        return f;
      };
      cl->curv_known = h[0] <= h[1];  // (all NaN: no finite curvature)
      if (cl->curv_known) {
        cl->curv_min = ord2f(h[0]);
        cl->curv_max = ord2f(h[1]);
      }
    }
    cl->has_normals = true;
    cl->sp_cur = -1;  // (the reset above also resets the Morton copy)
    cl->sp_n = cl->sp_n_pristine;
    cl->sp_valid = cl->sp_built;
    cl->sp_dirty = false;
  }
}

// ================================================================================================
// C ABI
// ================================================================================================
extern "C" {

int dlg_abi_version(void) { return DLG_ABI_VERSION; }

int64_t dlg_abi_struct_size(int which) {
  switch (which) {
    case 0: return (int64_t)sizeof(dlg_points);
    case 1: return (int64_t)sizeof(dlg_sac_params);
    case 2: return (int64_t)sizeof(dlg_sac_stats);
    case 3: return (int64_t)sizeof(dlg_extract_stats);
    case 4: return (int64_t)sizeof(dlg_planes);
    case 5: return (int64_t)sizeof(dlg_postprocess_params);
  }
  return -1;
}

const char* dlg_status_string(dlg_status s) {
  switch (s) {
    case DLG_OK: return "ok";
    case DLG_ERR_INVALID: return "invalid argument";
    case DLG_ERR_HIP: return "HIP error";
    case DLG_ERR_NO_DEVICE: return "no usable gfx950 device";
    case DLG_ERR_COMM: return "communicator error";
    case DLG_ERR_CAPACITY: return "output buffer too small";
    case DLG_ERR_INTERNAL: return "internal error";
  }
  return "unknown status";
}

void dlg_sac_params_default(dlg_sac_params* p) {
  if (!p) return;
  std::memset(p, 0, sizeof(*p));
  p->threshold = 0.0;  // SACSegmentation::threshold_ default
  p->max_iterations = 50;
  p->probability = 0.99;
  p->optimize = 1;
  p->seed = 12345u;
  p->model = DLG_SACMODEL_PLANE;
  p->normal_distance_weight = 0.1;
  p->refit_mode = DLG_REFIT_PCL;
  p->hypotheses_per_launch = 0;
  p->gather_inliers = 1;
}

dlg_status dlg_ctx_create(dlg_ctx** out, int device) {
  if (!out) return DLG_ERR_INVALID;
  *out = nullptr;
  auto c = std::make_unique<dlg_ctx>();
  dlg_status s = init_ctx(c.get(), device);
  if (s != DLG_OK) {
    g_last_create_error = c->err;
    return s;
  }
  c->comm = make_single_comm();
  *out = c.release();
  return DLG_OK;
}

dlg_status dlg_get_unique_id(void* uid) {
  if (!uid) return DLG_ERR_INVALID;
  std::string err;
  if (!rccl_get_unique_id(uid, &err)) {
    g_last_create_error = err;
    return DLG_ERR_COMM;
  }
  return DLG_OK;
}

dlg_status dlg_ctx_create_dist(dlg_ctx** out, int device, int rank, int world, const void* uid) {
  if (!out || world < 1 || rank < 0 || rank >= world || (world > 1 && !uid)) return DLG_ERR_INVALID;
  *out = nullptr;
  auto c = std::make_unique<dlg_ctx>();
  dlg_status s = init_ctx(c.get(), device);
  if (s != DLG_OK) {
    g_last_create_error = c->err;
    return s;
  }
  if (world == 1 && !uid) {  // (world 1 with an id: a 1-rank RCCL communicator)
    c->comm = make_single_comm();
  } else {
    std::string err;
    (void)hipSetDevice(device);
    c->comm = make_rccl_comm(rank, world, uid, &err);
    if (!c->comm) {
      g_last_create_error = err;
      dlg_ctx_destroy(c.release());  // (its streams, events and device count)
      return DLG_ERR_COMM;
    }
  }
  *out = c.release();
  return DLG_OK;
}

dlg_status dlg_ctx_create_loopback_group(dlg_ctx** out_array, int world, int device) {
  if (!out_array || world < 1) return DLG_ERR_INVALID;
  auto g = make_loopback_group(world);
  std::vector<dlg_ctx*> made;
  for (int r = 0; r < world; ++r) {
    auto c = std::make_unique<dlg_ctx>();
    dlg_status s = init_ctx(c.get(), device);
    if (s != DLG_OK) {
      g_last_create_error = c->err;
      for (auto* m : made) dlg_ctx_destroy(m);
      return s;
    }
    c->comm = make_loopback_comm(g, r);
    made.push_back(c.release());
  }
  for (int r = 0; r < world; ++r) out_array[r] = made[r];
  return DLG_OK;
}

dlg_status dlg_ctx_destroy(dlg_ctx* c) {
  if (!c) return DLG_OK;
  if (c->counted) ctx_count_add(c->device, -1);
  (void)hipSetDevice(c->device);
  if (c->stream) (void)hipStreamSynchronize(c->stream);
  c->comm.reset();
  c->pos.release(); c->samples.release(); c->hyps.release(); c->res.release();
  c->tile_in.release(); c->tile_off_in.release(); c->tile_off_out.release(); c->totals.release();
  c->partials.release(); c->moments.release(); c->scratch_f64.release(); c->inl_gid.release(); c->inl_xyz.release();
  c->small.release(); c->h_small.release();
  c->gath64.release(); c->gath32.release();
  c->h_pos.release(); c->h_res.release(); c->h_tot.release(); c->h_mom.release(); c->h_g64.release();
  c->h_stage.release();
  c->pick.release(); c->h_pick.release(); c->rk.release(); c->h_rk.release();
  if (c->pub) (void)hipHostFree(c->pub);
  c->pub = nullptr;
  c->pub_cap = 0;
  c->nw.release();
  c->pw.release();
  c->pstats.release();
  c->sel1_status.release();
  c->sel1_err.release();
  c->sel1_tk.release();
  c->lp.release();
  c->lp_n.release();
  c->fs_scr.release();
  c->fs_x.release(); c->fs_y.release(); c->fs_z.release(); c->fs_n.release();
  c->mk0.release(); c->mk1.release(); c->mi0.release(); c->mi1.release(); c->msort.release(); c->mxyz.release();
  c->mom_done.release(); c->pick_done.release();
  if (c->ev_stage) (void)hipEventDestroy(c->ev_stage);
  if (c->ev_inl) (void)hipEventDestroy(c->ev_inl);
  if (c->cstream) {
    (void)hipStreamSynchronize(c->cstream);
    (void)hipStreamDestroy(c->cstream);
  }
  if (c->sstream) {
    (void)hipStreamSynchronize(c->sstream);
    (void)hipStreamDestroy(c->sstream);
  }
  if (c->ev_fork) (void)hipEventDestroy(c->ev_fork);
  if (c->ev_join) (void)hipEventDestroy(c->ev_join);
  for (auto& pr : c->ev_sel)
    for (auto& ev : pr)
      if (ev) (void)hipEventDestroy(ev);
  for (auto& pr : c->ev_walk)
    for (auto& ev : pr)
      if (ev) (void)hipEventDestroy(ev);
  for (auto& ev : c->ev)
    if (ev) (void)hipEventDestroy(ev);
  if (c->stream) (void)hipStreamDestroy(c->stream);
  delete c;
  return DLG_OK;
}

const char* dlg_last_error(const dlg_ctx* c) {
  return c ? c->err.c_str() : g_last_create_error.c_str();
}

dlg_status dlg_ctx_info(const dlg_ctx* c, int* rank, int* world, int* device) {
  if (!c) return DLG_ERR_INVALID;
  if (rank) *rank = c->comm->rank();
  if (world) *world = c->comm->world();
  if (device) *device = c->device;
  return DLG_OK;
}

dlg_status dlg_cloud_upload(dlg_ctx* c, const dlg_points* pts, const int32_t* indices,
                            int64_t n_indices, int32_t id_base, dlg_cloud** out) {
  if (!c || !pts || !out || (pts->n > 0 && !pts->xyz) || pts->n < 0) return DLG_ERR_INVALID;
  if (pts->stride_bytes < 12 || pts->stride_bytes % 4) return fail(c, DLG_ERR_INVALID, "stride_bytes must be >= 12 and a multiple of 4");
  if (indices && n_indices < 0) return fail(c, DLG_ERR_INVALID, "negative n_indices");
  *out = nullptr;
  auto cl = std::make_unique<dlg_cloud>();
  dlg_status s = guarded(c, [&] {
    const int64_t n = indices ? n_indices : pts->n;
    if (n > INT32_MAX) throw DlgError(DLG_ERR_INVALID, "more than 2^31-1 points");
    const int64_t sf = pts->stride_bytes / 4;
    cl->ctx = c;
    cl->n_total = n;
    cl->n_points = pts->n;
    cl->id_base = id_base;
    cl->gid_ident = indices == nullptr;
    cl->n_active = n;
    cl->pristine.ensure((size_t)std::max<int64_t>(n, 1));
    if (indices)
      for (int64_t i = 0; i < n; ++i)
        if (indices[i] < 0 || indices[i] >= pts->n) throw DlgError(DLG_ERR_INVALID, "index out of range");
    if (n && (!indices || 4 * n >= pts->n)) {
      // the caller's records go up as they are (one DMA), the SoA split and ids on the device
      DevBuf<uint8_t>& raw = c->nw.raw;
      const size_t bytes = (size_t)pts->n * (size_t)pts->stride_bytes;
      raw.ensure(bytes + (indices ? 4 * (size_t)n : 0));
      HIPCHK(hipMemcpyAsync(raw.p, pts->xyz, bytes, hipMemcpyHostToDevice, c->stream));
      const int32_t* didx = nullptr;
      if (indices) {
        HIPCHK(hipMemcpyAsync(raw.p + bytes, indices, 4 * (size_t)n, hipMemcpyHostToDevice,
                              c->stream));
        didx = reinterpret_cast<const int32_t*>(raw.p + bytes);
      }
      launch_upload_gather(reinterpret_cast<const float*>(raw.p), sf, didx, n, id_base,
                           cl->pristine.out(), c->stream);
      HIPCHK(hipGetLastError());
    } else if (n) {
      // a small subset of a large cloud: gather on the host
      std::vector<float> x(n), y(n), z(n);
      std::vector<int32_t> g(n);
      for (int64_t i = 0; i < n; ++i) {
        const int64_t k = indices[i];
        const float* p = pts->xyz + k * sf;
        x[i] = p[0]; y[i] = p[1]; z[i] = p[2];
        g[i] = (int32_t)(id_base + k);
      }
      HIPCHK(hipMemcpyAsync(cl->pristine.x.p, x.data(), 4 * n, hipMemcpyHostToDevice, c->stream));
      HIPCHK(hipMemcpyAsync(cl->pristine.y.p, y.data(), 4 * n, hipMemcpyHostToDevice, c->stream));
      HIPCHK(hipMemcpyAsync(cl->pristine.z.p, z.data(), 4 * n, hipMemcpyHostToDevice, c->stream));
      HIPCHK(hipMemcpyAsync(cl->pristine.gid.p, g.data(), 4 * n, hipMemcpyHostToDevice, c->stream));
      sync(c);  // the host vectors go out of scope
    }
    c->totals.ensure(8);
    launch_absmax(cl->pristine.view(n), reinterpret_cast<uint32_t*>(c->totals.p), c->stream);
    uint32_t bits[4];
    HIPCHK(hipMemcpyAsync(bits, c->totals.p, 16, hipMemcpyDeviceToHost, c->stream));
    sync(c);
    for (int k = 0; k < 3; ++k) std::memcpy(&cl->amax[k], &bits[k], 4);
    std::memcpy(&cl->fmax, &bits[3], 4);
    if (c->opt.prune != 0 && n >= 3 && (n >= kPruneMinPoints || c->opt.prune == 1))
      build_spatial(c, cl.get());
  });
  if (s != DLG_OK) {
    cl->pristine.release();
    cl->sp_pristine.release();
    cl->sp_tiles_pr.release();
    cl->sp_supers_pr.release();
    return s;
  }
  *out = cl.release();
  return DLG_OK;
}

dlg_status dlg_cloud_destroy(dlg_cloud* cl) {
  if (!cl) return DLG_OK;
  if (cl->ctx) (void)hipSetDevice(cl->ctx->device);
  if (cl->ctx && cl->ctx->stream) (void)hipStreamSynchronize(cl->ctx->stream);
  cl->pristine.release();
  cl->raw_nrm.release();
  cl->buf[0].release();
  cl->buf[1].release();
  cl->sp_pristine.release();
  cl->sp_buf[0].release();
  cl->sp_buf[1].release();
  cl->sp_tiles_pr.release();
  cl->sp_supers_pr.release();
  cl->sp_order.release();
  for (int b = 0; b < 2; ++b) {
    cl->sp_tb[b].release();
    cl->sp_sb[b].release();
  }
  cl->ubits.release();
  cl->tag.release();
  delete cl;
  return DLG_OK;
}

dlg_status dlg_cloud_build_spatial(dlg_ctx* c, dlg_cloud* cl) {
  if (!c || !cl || cl->ctx != c) return DLG_ERR_INVALID;
  return guarded(c, [&] {
    if (cl->n_total < 3 || cl->sp_built) return;
    if (cl->cur >= 0) throw DlgError(DLG_ERR_INVALID, "build the spatial copy before extracting (or after dlg_cloud_reset)");
    build_spatial(c, cl);
  });
}

dlg_status dlg_cloud_drop_spatial(dlg_cloud* cl) {
  if (!cl) return DLG_ERR_INVALID;
  // (the copy's device buffers stay allocated for the next build -- hipFree synchronises the
  // device and a rebuild would allocate them again; dlg_cloud_destroy frees them)
  cl->sp_built = cl->sp_valid = false;
  cl->sp_n = cl->sp_n_pristine = 0;
  cl->cur = -1;  // (a lean list needs the Morton copy: back to the pristine list)
  cl->n_active = cl->n_total;
  cl->sp_cur = -1;
  cl->sp_dirty = false;
  return DLG_OK;
}

dlg_status dlg_cloud_reset(dlg_cloud* cl) {
  if (!cl) return DLG_ERR_INVALID;
  cl->cur = -1;
  cl->n_active = cl->n_total;
  cl->sp_cur = -1;
  cl->sp_n = cl->sp_n_pristine;
  cl->sp_valid = cl->sp_built;
  cl->sp_dirty = false;
  return DLG_OK;
}

dlg_status dlg_cloud_active(const dlg_cloud* cl, int64_t* n) {
  if (!cl || !n) return DLG_ERR_INVALID;
  *n = cl->n_active;
  return DLG_OK;
}

dlg_status dlg_cloud_set_normals(dlg_ctx* c, dlg_cloud* cl, const float* normals, int64_t n,
                                 int64_t stride_bytes) {
  if (!c || !cl || cl->ctx != c || (n > 0 && !normals)) return DLG_ERR_INVALID;
  if (n != cl->n_points)
    return fail(c, DLG_ERR_INVALID, "normals must have one record per uploaded point");
  if (stride_bytes != 16 && (stride_bytes < 32 || stride_bytes % 4))
    return fail(c, DLG_ERR_INVALID, "stride_bytes must be 16 (nx, ny, nz, curvature) or >= 32 (pcl::Normal)");
  return guarded(c, [&] {
    const float* raw_dev = nullptr;
    if (n > 0) {
      DevBuf<uint8_t>& raw = c->nw.raw;  // scratch shared with the normals path
      raw.ensure((size_t)n * (size_t)stride_bytes);
      HIPCHK(hipMemcpyAsync(raw.p, normals, (size_t)n * (size_t)stride_bytes,
                            hipMemcpyHostToDevice, c->stream));
      raw_dev = reinterpret_cast<const float*>(raw.p);
    }
    attach_normals(c, cl, raw_dev, stride_bytes / 4, stride_bytes == 16 ? 3 : 4, false);
  });
}

namespace {
// DLG_OPT_HYP_SHARD on a multi-rank context: for the call, the context runs as one rank (every
// rank holds the whole cloud and computes the same round) and only the scoring is split by
// hypotheses over the real communicator (one_batch: slices + an allreduce of the counts)
struct HypShardScope {
  dlg_ctx* c;
  bool on;
  HypShardScope(dlg_ctx* ctx, bool enable) : c(ctx), on(enable) {
    if (!on) return;
    if (!c->solo) c->solo = make_single_comm();
    std::swap(c->comm, c->solo);
    c->hcomm = c->solo.get();
  }
  ~HypShardScope() {
    if (!on) return;
    std::swap(c->comm, c->solo);
    c->hcomm = nullptr;
  }
};

// whether a call on this cloud runs hypothesis-sharded.  DLG_OPT_HYP_SHARD -1 (default): when
// every rank holds the same cloud -- the same ids (id_base, count, identity) and the same extent --
// which is how SURVEY 8(e)'s small-N fallback is set up (dlg_shard_range hands every rank the
// whole cloud when point shards would fall below the Morton-copy cut-off); point-sharding such a
// replicated cloud would count every point once per rank.  Decided once per cloud (one allgather
// of a signature; every rank decides alike).
bool hyp_shard_on(dlg_ctx* c, dlg_cloud* cl) {
  if (c->comm->world() == 1) return false;
  if (c->opt.hyp_shard >= 0) return c->opt.hyp_shard == 1;
  if (!cl->repl_known) {
    uint64_t h = 1469598103934665603ull;
    auto mix = [&](uint64_t v) {
      for (int k = 0; k < 8; ++k) h = (h ^ ((v >> (8 * k)) & 0xFFu)) * 1099511628211ull;
    };
    mix((uint64_t)cl->n_points);
    mix((uint64_t)cl->n_total);
    mix((uint64_t)(uint32_t)cl->id_base);
    mix(cl->gid_ident ? 1u : 0u);
    uint32_t b[4];
    std::memcpy(b, cl->amax, 12);
    std::memcpy(b + 3, &cl->fmax, 4);
    for (uint32_t v : b) mix(v);
    std::vector<int64_t> all;
    allgather_i64(c, (int64_t)(h >> 1), &all);
    cl->repl = std::all_of(all.begin(), all.end(), [&](int64_t v) { return v == all[0]; });
    cl->repl_known = true;
  }
  return cl->repl;
}
}  // namespace

dlg_status dlg_sac_segment(dlg_ctx* c, dlg_cloud* cl, const dlg_sac_params* prm, float coeff_out[4],
                           int32_t* inliers_out, int64_t cap, int64_t* n_inliers,
                           dlg_sac_stats* stats) {
  if (!c || !cl || !prm || !coeff_out || !n_inliers || cl->ctx != c) return DLG_ERR_INVALID;
  if (!inliers_out && cap > 0) return DLG_ERR_INVALID;
  dlg_sac_stats local;
  dlg_sac_stats* st = stats ? stats : &local;
  return guarded_group(c, [&] {
    HypShardScope hs(c, hyp_shard_on(c, cl));
    std::memset(coeff_out, 0, 4 * sizeof(float));
    *n_inliers = 0;
    SegOut so = segment_impl(c, cl, *prm, false, st, nullptr);
    if (!so.has_model) return;
    std::memcpy(coeff_out, so.coeff, sizeof(so.coeff));
    int64_t g = 0;
    *n_inliers = emit_inliers(c, so, prm->gather_inliers != 0, inliers_out, cap, &g);
  });
}

dlg_status dlg_sac_segment_host(dlg_ctx* c, const dlg_points* pts, const int32_t* indices,
                                int64_t n_indices, const dlg_sac_params* prm, float coeff_out[4],
                                int32_t* inliers_out, int64_t cap, int64_t* n_inliers,
                                dlg_sac_stats* stats) {
  dlg_cloud* cl = nullptr;
  dlg_status s = dlg_cloud_upload(c, pts, indices, n_indices, 0, &cl);
  if (s != DLG_OK) return s;
  s = dlg_sac_segment(c, cl, prm, coeff_out, inliers_out, cap, n_inliers, stats);
  dlg_cloud_destroy(cl);
  return s;
}

dlg_status dlg_extract_planes(dlg_ctx* c, dlg_cloud* cl, const dlg_sac_params* prm, int max_planes,
                              int64_t min_inliers, float* coeffs_out, int64_t* offsets_out,
                              int32_t* inliers_out, int64_t cap, int* n_planes,
                              dlg_extract_stats* stats) {
  if (!c || !cl || !prm || max_planes < 0 || !n_planes || cl->ctx != c) return DLG_ERR_INVALID;
  if (max_planes > 0 && (!coeffs_out || !offsets_out)) return DLG_ERR_INVALID;
  if (!inliers_out && cap > 0) return DLG_ERR_INVALID;
  dlg_extract_stats local;
  dlg_extract_stats* xs = stats ? stats : &local;
  std::memset(xs, 0, sizeof(*xs));
  auto t0 = std::chrono::steady_clock::now();
  dlg_status s = guarded_group(c, [&] {
    HypShardScope hs(c, hyp_shard_on(c, cl));
    *n_planes = 0;
    if (max_planes > 0) offsets_out[0] = 0;
    int64_t written = 0;
    const int64_t floor_n = std::max<int64_t>(3, min_inliers);
    // every rank's active count: gathered once, then carried from each round's survivors
    std::vector<int64_t> active;
    // (bit 40: this rank holds a valid spatial copy.  Lean rounds change the round's collective
    // sequence, so they run only when every rank can take them: one agreed decision per call)
    constexpr int64_t kSpBit = int64_t(1) << 40;
    int64_t N = allgather_i64(c, cl->n_active | (cl->sp_valid ? kSpBit : 0), &active);
    c->sp_all = true;
    N = 0;
    for (int64_t& v : active) {
      c->sp_all = c->sp_all && (v & kSpBit) != 0;
      v &= kSpBit - 1;
      N += v;
    }
    for (int p = 0; p < max_planes; ++p) {
      if (N < floor_n) break;
      dlg_sac_stats st;
      SegOut so = segment_impl(c, cl, *prm, true, &st, xs, &active);
      if (c->opt.sync_check) check_in_step(c, p, so);
      xs->rounds++;
      if (!so.has_model) break;
      if (so.lean) xs->lean_rounds++;
      const int64_t n_in = so.n_in_global;
      if (n_in == 0 || n_in < min_inliers) break;  // plane rejected: active list unchanged
      int64_t g = 0;
      const double t_e0 = trace_on() ? now_ms() : 0.0;
      int64_t n = emit_inliers(c, so, prm->gather_inliers != 0, inliers_out + written,
                               cap - written, &g, /*deferred=*/true, /*counts_known=*/true);
      if (trace_on())
        std::fprintf(stderr, "[dlg] after-round: segment-return %.3fms emit %.3fms\n",
                     t_e0 - c->t_tot, now_ms() - t_e0);
      std::memcpy(coeffs_out + 4 * p, so.coeff, sizeof(so.coeff));
      written += n;
      offsets_out[p + 1] = written;
      *n_planes = p + 1;
      cl->buf_lean[cl->spare()] = so.lean;
      cl->cur = cl->spare();  // commit the removal
      cl->n_active = so.n_out_local;
      active = so.out_ranks;
      N = 0;
      for (int64_t v : active) N += v;
      if (so.sp_compacted) {
        cl->sp_cur = cl->sp_spare();
        cl->sp_n = so.sp_n_out;
        cl->sp_dirty = false;  // bounds queued by segment_impl behind the compaction
      } else {
        cl->sp_valid = false;  // (SACMODEL_NORMAL_PLANE rounds do not carry the spatial copy)
      }
    }
    flush_emit(c);
    drain_pending(c);
    // A stream synchronisation lets the HIP runtime reclaim the per-command resources of the
    // rounds: with event waits alone they pile up until a D2H copy blocks the host for ~10 ms
    // (measured: every ~55 rounds).  The stream only holds the last round's tails here.
    sync(c);
    settle_round(c);
  });
  c->pending_dst = nullptr;  // (error path: never write into the caller's buffer later)
  c->pending_n = c->pending_off = 0;
  c->emit_dst = nullptr;
  c->emit_n = 0;
  c->sel_pending = nullptr;  // (never read into the caller's stats after the call)
  c->sp_check = false;
  xs->wall_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  return s;
}

dlg_status dlg_float_sums(dlg_ctx* c, const float* xyz, int64_t n, const float cin[4], int reps,
                          float sums_out[9], float coeff_out[4], int* uncertain,
                          double* ms_per_call, int64_t* walk_stats) {
  if (!c || n < 0 || n > INT32_MAX || (n > 0 && !xyz) || !cin || reps < 1 || !sums_out ||
      !coeff_out || !uncertain || !ms_per_call)
    return DLG_ERR_INVALID;
  return guarded(c, [&] {
    DevBuf<float> dx;
    DevBuf<float4> dc;
    DevBuf<int32_t> dn, dres;
    DevBuf<uint8_t> scr;
    dx.ensure(3 * (size_t)std::max<int64_t>(n, 1));
    dc.ensure(2);
    dn.ensure(1);
    dres.ensure(16);
    scr.ensure(fs_scratch_bytes(std::max<int64_t>(n, 1), 1));
    FsBuffers b = fs_carve(scr.p, std::max<int64_t>(n, 1), 1);
    DevBuf<int64_t> wst;
    if (walk_stats) {
      wst.ensure(72);
      HIPCHK(hipMemsetAsync(wst.p, 0, 72 * 8, c->stream));
      b.wst = wst.p;
    }
    HIPCHK(fs_reset(b, c->stream, c->opt.fs_poison));
    if (n) HIPCHK(hipMemcpyAsync(dx.p, xyz, 12 * (size_t)n, hipMemcpyHostToDevice, c->stream));
    const int32_t n32 = (int32_t)n;
    const float4 ci = make_float4(cin[0], cin[1], cin[2], cin[3]);
    HIPCHK(hipMemcpyAsync(dn.p, &n32, 4, hipMemcpyHostToDevice, c->stream));
    HIPCHK(hipMemcpyAsync(dc.p, &ci, 16, hipMemcpyHostToDevice, c->stream));
    double total = 0.0;
    for (int r = 0; r < reps; ++r) {
      if (walk_stats) HIPCHK(hipMemsetAsync(wst.p, 0, 72 * 8, c->stream));  // (the last call's)
      HIPCHK(hipEventRecord(c->ev[0], c->stream));
      launch_fs_refit(dx.p, dx.p + 1, dx.p + 2, 3, dn.p, std::max<int64_t>(n, 1), b, dc.p,
                      dc.p + 1, dres.p, c->num_cus, c->stream, nullptr, nullptr, nullptr, nullptr,
                      nullptr, 0, nullptr, c->opt.fs_segments, nullptr, nullptr,
                      c->opt.fs_join);
      HIPCHK(hipGetLastError());
      HIPCHK(hipEventRecord(c->ev[1], c->stream));
      sync(c);
      total += event_ms(c, 0, 1);
    }
    int32_t h[16];
    float4 co;
    HIPCHK(hipMemcpy(h, dres.p, sizeof(h), hipMemcpyDeviceToHost));
    HIPCHK(hipMemcpy(&co, dc.p + 1, 16, hipMemcpyDeviceToHost));
    std::memcpy(sums_out, h + 2, 9 * sizeof(float));
    coeff_out[0] = co.x; coeff_out[1] = co.y; coeff_out[2] = co.z; coeff_out[3] = co.w;
    *uncertain = h[0];
    *ms_per_call = total / reps;
    if (walk_stats) HIPCHK(hipMemcpy(walk_stats, wst.p, 72 * 8, hipMemcpyDeviceToHost));
  });
}

dlg_status dlg_score_benchmark(dlg_ctx* c, dlg_cloud* cl, int D, int kernel, int reps,
                               double threshold, double* ms_per_launch, int32_t* counts_out) {
  if (!c || !cl || D < 1 || D > kMaxHypPerLaunch || reps < 1 || !ms_per_launch) return DLG_ERR_INVALID;
  if (kernel != kScoreExact && kernel != kScoreBf16 && kernel != kScorePruned) return DLG_ERR_INVALID;
  const int variant = kernel;
  return guarded(c, [&] {
    ensure_list_xyz(c, cl);
    const PointsView src = cl->view();
    if (src.n < 3) throw DlgError(DLG_ERR_INVALID, "need >= 3 active points");
    Mt19937 rng(777u);
    c->h_pos.ensure(3 * (size_t)D);
    for (int i = 0; i < 3 * D; ++i) c->h_pos.p[i] = (int32_t)((uint32_t)rng.rnd() % (uint64_t)src.n);
    c->pos.ensure(3 * (size_t)D);
    c->samples.ensure(3 * (size_t)D);
    c->hyps.ensure(kHypScratchBytes / sizeof(HypRec) + 1);
    c->res.ensure(2 * (size_t)kMaxHypPerLaunch + 64);
    const float cthr = thr_ceil(threshold);
    if (variant == kScorePruned && cl->sp_valid) ensure_sphere_bounds(c, cl);
    HIPCHK(hipMemcpyAsync(c->pos.p, c->h_pos.p, 12 * (size_t)D, hipMemcpyHostToDevice, c->stream));
    launch_gather_samples(c->pos.p, 3 * D, 0, src, c->samples.p, c->stream);
    const int Dp = (D + 63) / 64 * 64;
    launch_build_hyps(c->samples.p, D, cthr, cl->amax[0], cl->amax[1], cl->amax[2], c->hyps.p,
                      c->res.p + Dp, c->stream);
    double total = 0.0;
    for (int r = 0; r < reps; ++r) {
      HIPCHK(hipMemsetAsync(c->res.p, 0, 4 * (size_t)Dp, c->stream));
      HIPCHK(hipEventRecord(c->ev[0], c->stream));
      if (variant == kScorePruned) {
        if (!cl->sp_valid) throw DlgError(DLG_ERR_INVALID, "cloud has no spatial copy");
        c->lp.ensure((size_t)sp_supers(cl->sp_n) * prune_list_stride(D) + 1);
        ensure_prune_work(c, sp_supers(cl->sp_n));
        unsigned long long* stp = prune_stats_ptr(c);
        launch_score_pruned(spatial_view(cl), c->hyps.p, D, cthr, prune_margin(cthr, cl->amax),
                            cl->amax, c->res.p, c->lp.p, c->lp_n.p + kPwHeader, c->num_cus, c->stream, stp,
                            nullptr, nullptr, nullptr, nullptr, c->opt.tile_scorer);
      } else {
        launch_score(src, c->hyps.p, D, cthr, c->res.p, variant, c->num_cus, c->stream);
      }
      HIPCHK(hipGetLastError());
      HIPCHK(hipEventRecord(c->ev[1], c->stream));
      sync(c);
      total += event_ms(c, 0, 1);
    }
    *ms_per_launch = total / reps;
    if (counts_out) {
      HIPCHK(hipMemcpyAsync(counts_out, c->res.p, 4 * (size_t)D, hipMemcpyDeviceToHost, c->stream));
      sync(c);
    }
  });
}

dlg_status dlg_ctx_set_option(dlg_ctx* c, int option, int64_t value) {
  if (!c) return DLG_ERR_INVALID;
  return guarded(c, [&] {
    PathOptions& o = c->opt;
    switch (option) {
      case DLG_OPT_PRUNE:
        if (value < -1 || value > 1) throw DlgError(DLG_ERR_INVALID, "DLG_OPT_PRUNE: -1, 0 or 1");
        o.prune = (int)value;
        break;
      case DLG_OPT_LEAN_ROUNDS: o.lean = value != 0; break;
      case DLG_OPT_SPEC_PICK: o.spec_pick = value != 0; break;
      case DLG_OPT_PRUNE_NP: o.prune_np = value != 0; break;
      case DLG_OPT_SCORE_KERNEL:
        if (value != DLG_SCORE_BF16 && value != DLG_SCORE_EXACT)
          throw DlgError(DLG_ERR_INVALID, "DLG_OPT_SCORE_KERNEL: DLG_SCORE_BF16 or DLG_SCORE_EXACT");
        o.score_kernel = value == DLG_SCORE_EXACT ? kScoreExact : kScoreBf16;
        break;
      case DLG_OPT_PRUNE_STATS:
        o.prune_stats = value != 0;
        if (o.prune_stats) {
          c->pstats.ensure(8);
          HIPCHK(hipMemsetAsync(c->pstats.p, 0, 8 * sizeof(unsigned long long), c->stream));
        }
        break;
      case DLG_OPT_SELECT_TILE:
        if (value != kSel1Points[0] && value != kSel1Points[1] && value != kSel1Points[2])
          throw DlgError(DLG_ERR_INVALID, "DLG_OPT_SELECT_TILE: 4096, 8192 or 16384");
        o.sel1_tile = (int)value;
        break;
      case DLG_OPT_PCL_REFIT_DEVICE:
        if (value < 0 || value > 3) throw DlgError(DLG_ERR_INVALID, "DLG_OPT_PCL_REFIT_DEVICE: 0..3");
        o.pcl_dev = (int)value;
        break;
      case DLG_OPT_NORMALS_FUSED: o.nbr_fused = value != 0; break;
      case DLG_OPT_REGULATE_WAVE: o.bfs_wave = value != 0; break;
      case DLG_OPT_FS_POISON: o.fs_poison = value != 0; break;
      case DLG_OPT_HYP_SHARD:
        if (value < -1 || value > 1) throw DlgError(DLG_ERR_INVALID, "DLG_OPT_HYP_SHARD: -1, 0 or 1");
        o.hyp_shard = (int)value;
        break;
      case DLG_OPT_FAULT_INJECT:
        if (value < 0) throw DlgError(DLG_ERR_INVALID, "DLG_OPT_FAULT_INJECT: >= 0");
        o.fault_round = (int)value;
        break;
      case DLG_OPT_SYNC_CHECK: o.sync_check = value != 0; break;
      case DLG_OPT_COMM_TIMEOUT_MS:
        if (value < 0) throw DlgError(DLG_ERR_INVALID, "DLG_OPT_COMM_TIMEOUT_MS: >= 0");
        c->comm->timeout_ms = value;
        if (c->solo) c->solo->timeout_ms = value;
        break;
      case DLG_OPT_SEL1_TICKET:
        if (value < -1 || value > 1) throw DlgError(DLG_ERR_INVALID, "DLG_OPT_SEL1_TICKET: -1, 0 or 1");
        o.sel1_ticket = (int)value;
        break;
      case DLG_OPT_BOUNDS_STREAM: o.bounds_stream = value != 0; break;
      case DLG_OPT_SPATIAL_CURVE:
        if (value < 0 || value > 1) throw DlgError(DLG_ERR_INVALID, "DLG_OPT_SPATIAL_CURVE: 0 or 1");
        o.spatial_curve = (int)value;
        break;
      case DLG_OPT_FS_JOIN: o.fs_join = value != 0; break;
      case DLG_OPT_UNREFINED_LIST: o.unrefined_list = value != 0; break;
      case DLG_OPT_FS_SEGMENTS:
        if (value < 1 || value > kFsSegMax) throw DlgError(DLG_ERR_INVALID, "DLG_OPT_FS_SEGMENTS: 1..16");
        o.fs_segments = (int)value;
        break;
      case DLG_OPT_FS_ONE_WALK:
        if (value < 0 || value > 2) throw DlgError(DLG_ERR_INVALID, "DLG_OPT_FS_ONE_WALK: 0..2");
        o.fs_protocol = (int)value;
        break;
      case DLG_OPT_PRUNE_TILE_SCORER:
        // (DLG_TILE_* values, and the A/B-only kernel variants kTileScorerExK1/ExK4/ExPk and
        // claim variants 15..17)
        if (value != DLG_TILE_EXACT && value != DLG_TILE_BF16 && value != DLG_TILE_MFMA &&
            value != kTileScorerExK1 && value != kTileScorerMfmaX && value != kTileScorerMfmaW &&
            value != kTileScorerExK4 && value != kTileScorerExPk &&
            !(value >= kTileScorerClaimR4 && value <= kTileScorerClaimTail))
          throw DlgError(DLG_ERR_INVALID, "DLG_OPT_PRUNE_TILE_SCORER: DLG_TILE_EXACT or DLG_TILE_BF16");
        o.tile_scorer = (int)value;
        break;
      default: throw DlgError(DLG_ERR_INVALID, "unknown option");
    }
  });
}

dlg_status dlg_ctx_get_option(const dlg_ctx* c, int option, int64_t* value) {
  if (!c || !value) return DLG_ERR_INVALID;
  const PathOptions& o = c->opt;
  switch (option) {
    case DLG_OPT_PRUNE: *value = o.prune; break;
    case DLG_OPT_LEAN_ROUNDS: *value = o.lean; break;
    case DLG_OPT_SPEC_PICK: *value = o.spec_pick; break;
    case DLG_OPT_PRUNE_NP: *value = o.prune_np; break;
    case DLG_OPT_SCORE_KERNEL: *value = o.score_kernel == kScoreExact ? DLG_SCORE_EXACT : DLG_SCORE_BF16; break;
    case DLG_OPT_PRUNE_STATS: *value = o.prune_stats; break;
    case DLG_OPT_SELECT_TILE: *value = o.sel1_tile; break;
    case DLG_OPT_PCL_REFIT_DEVICE: *value = o.pcl_dev; break;
    case DLG_OPT_NORMALS_FUSED: *value = o.nbr_fused; break;
    case DLG_OPT_REGULATE_WAVE: *value = o.bfs_wave; break;
    case DLG_OPT_FS_POISON: *value = o.fs_poison; break;
    case DLG_OPT_HYP_SHARD: *value = o.hyp_shard; break;
    case DLG_OPT_FAULT_INJECT: *value = o.fault_round; break;
    case DLG_OPT_SYNC_CHECK: *value = o.sync_check; break;
    case DLG_OPT_COMM_TIMEOUT_MS: *value = c->comm->timeout_ms; break;
    case DLG_OPT_SEL1_TICKET: *value = o.sel1_ticket; break;
    case DLG_OPT_BOUNDS_STREAM: *value = o.bounds_stream; break;
    case DLG_OPT_SPATIAL_CURVE: *value = o.spatial_curve; break;
    case DLG_OPT_FS_JOIN: *value = o.fs_join; break;
    case DLG_OPT_UNREFINED_LIST: *value = o.unrefined_list; break;
    case DLG_OPT_FS_ONE_WALK: *value = o.fs_protocol; break;
    case DLG_OPT_FS_SEGMENTS: *value = o.fs_segments; break;
    case DLG_OPT_PRUNE_TILE_SCORER: *value = o.tile_scorer; break;
    default: return DLG_ERR_INVALID;
  }
  return DLG_OK;
}

dlg_status dlg_prune_stats(dlg_ctx* c, uint64_t out[8], int reset) {
  if (!c || !out) return DLG_ERR_INVALID;
  return guarded(c, [&] {
    std::memset(out, 0, 8 * sizeof(uint64_t));
    if (!c->opt.prune_stats) return;
    HIPCHK(hipMemcpyAsync(out, c->pstats.p, 8 * sizeof(uint64_t), hipMemcpyDeviceToHost, c->stream));
    if (reset) HIPCHK(hipMemsetAsync(c->pstats.p, 0, 8 * sizeof(unsigned long long), c->stream));
    sync(c);
  });
}

dlg_status dlg_set_profiling(dlg_ctx* c, int enable) {
  if (!c) return DLG_ERR_INVALID;
  if (enable < 0 || enable > 2) return DLG_ERR_INVALID;
  c->profiling = enable != 0;
  c->walk_events = enable == 1;
  return DLG_OK;
}

dlg_status dlg_synchronize(dlg_ctx* c) {
  if (!c) return DLG_ERR_INVALID;
  return guarded(c, [&] { HIPCHK(hipDeviceSynchronize()); });
}

dlg_status dlg_allreduce_max_f64(dlg_ctx* c, double* v) {
  if (!c || !v) return DLG_ERR_INVALID;
  if (c->comm->world() == 1) return DLG_OK;
  return guarded_group(c, [&] {
    c->scratch_f64.ensure(1);
    HIPCHK(hipMemcpyAsync(c->scratch_f64.p, v, 8, hipMemcpyHostToDevice, c->stream));
    c->comm->allreduce_max_f64(c->scratch_f64.p, 1, c->stream);
    HIPCHK(hipMemcpyAsync(v, c->scratch_f64.p, 8, hipMemcpyDeviceToHost, c->stream));
    sync(c);
  });
}

dlg_status dlg_shard_range(int64_t n_global, int rank, int world, int64_t* lo, int64_t* hi,
                           int* replicated) {
  if (n_global < 0 || world < 1 || rank < 0 || rank >= world || !lo || !hi) return DLG_ERR_INVALID;
  const bool repl = world > 1 && n_global / world < kPruneMinPoints;
  if (replicated) *replicated = repl ? 1 : 0;
  if (repl) {
    *lo = 0;
    *hi = n_global;
  } else {
    *lo = n_global * rank / world;
    *hi = n_global * (rank + 1) / world;
  }
  return DLG_OK;
}

dlg_status dlg_barrier(dlg_ctx* c) {
  double v = 0.0;
  return dlg_allreduce_max_f64(c, &v);
}

}  // extern "C"
