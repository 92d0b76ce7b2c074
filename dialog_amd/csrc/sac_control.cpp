// sac_control.cpp -- RansacControl (sac_control.hpp) and its C ABI (dlg_sac_control_*).
// Restates RandomSampleConsensus<PointT>::computeModel and SampleConsensusModel::getSamples /
// drawIndexSample of PCL 1.8 [PCL-1.8 ext; SURVEY.md §8(a) a6, a7]; reference call site
// Dialog/SimplifyVerticesSize.cpp:62-67.
#include "sac_control.hpp"

#include <algorithm>
#include <climits>
#include <cmath>
#include <limits>
#include <new>

namespace dlg {

void Overlay::reset(size_t expect) {
  size_t cap = 64;
  while (cap < expect * 4) cap <<= 1;
  if (slots_.size() < cap || ++gen_ == 0) {  // (a wrapped generation counter clears the table)
    slots_.assign(std::max(cap, slots_.size()), Slot{0, 0, 0});
    gen_ = 1;
  }
  mask_ = slots_.size() - 1;
  size_ = 0;
}

void Overlay::grow() {
  std::vector<Slot> old;
  old.swap(slots_);
  const uint32_t g = gen_;
  slots_.assign(old.size() * 2, Slot{0, 0, 0});
  gen_ = 1;
  mask_ = slots_.size() - 1;
  size_ = 0;
  for (const Slot& s : old)
    if (s.gen == g) (void)exchange(s.key, s.val);
}

namespace {
// the rnd() stream of one seed, generated once per thread and extended on demand: every
// segment() restarts PCL's generator at the same seed, so successive extraction rounds replay
// the same prefix
struct RndCache {
  uint32_t seed = 0;
  bool valid = false;
  Mt19937 gen;
  std::vector<uint32_t> v;
  const uint32_t* get(uint32_t s, int64_t upto) {
    if (!valid || s != seed) {
      seed = s;
      valid = true;
      gen = Mt19937(s);
      v.clear();
    }
    if ((int64_t)v.size() < upto) {
      v.reserve((size_t)upto);
      while ((int64_t)v.size() < upto) v.push_back((uint32_t)gen.rnd());
    }
    return v.data();
  }
};
thread_local RndCache t_rnd;
}  // namespace

RansacControl::RansacControl(const dlg_sac_params& prm, int64_t N, int cap_h,
                             ShuffleReplay* replay)
    : prm_(prm), N_(N), cap_h_(std::max(cap_h, 1)), seed_(prm.seed),
      own_(replay ? nullptr : new ShuffleReplay()), ov_(replay ? replay : own_.get()) {
  log_probability_ = std::log(1.0 - prm.probability);
  one_over_indices_ = 1.0 / (double)N;
  // getSamples cannot select 3 unique points -> computeModel fails without an iteration
  if (N < 3) done_ = true;
  // while (iterations_ < k && skipped_count < max_skip), max_skip = (unsigned)(max_iterations * 10):
  // with max_iterations = 0 the loop never runs (no draw, no model).  skipped_count itself stays
  // 0: computeModelCoefficients repeats isSampleGood's test, which getSamples already passed.
  if ((uint32_t)((int64_t)prm.max_iterations * 10) == 0u) done_ = true;
  ov_->reset(3 * (size_t)std::min<int64_t>((int64_t)prm.max_iterations + 1, cap_h_) + 16);
}

int RansacControl::next_size() const {
  if (done_) return 0;
  // the hypotheses PCL can still evaluate (+ a little slack for bad draws); before the first
  // count k is still 1.0, so the first batch is sized by the iteration cap
  int64_t remaining = (int64_t)prm_.max_iterations + 1 - iterations_;
  if (have_ && std::isfinite(k_) && k_ < 1e18)
    remaining = std::min<int64_t>(remaining, (int64_t)std::ceil(k_) - iterations_);
  remaining = std::max<int64_t>(remaining, 1);
  return (int)std::min<int64_t>(cap_h_, remaining + (iterations_ ? 8 : 0));
}

int RansacControl::next_batch(int32_t* pos) {
  const int D = next_size();
  if (D <= 0) return 0;
  const uint32_t* r = t_rnd.get(seed_, rnd_pos_ + 3 * (int64_t)D) + rnd_pos_;
  rnd_pos_ += 3 * (int64_t)D;
  // rnd() % (N - i): rnd() < 2^31 and N <= INT32_MAX, so 32-bit remainders are exact
  const FastMod32 m0((uint32_t)N_), m1((uint32_t)(N_ - 1)), m2((uint32_t)(N_ - 2));
  ShuffleReplay& ov = *ov_;
  for (int d = 0; d < D; ++d, r += 3) {
    ov.swap(0, (int64_t)m0.mod(r[0]));
    ov.swap(1, 1 + (int64_t)m1.mod(r[1]));
    ov.swap(2, 2 + (int64_t)m2.mod(r[2]));
    pos[3 * d] = ov.at(0);
    pos[3 * d + 1] = ov.at(1);
    pos[3 * d + 2] = ov.at(2);
  }
  batch_base_ = drawn_;
  drawn_ += D;
  pending_ = D;
  return D;
}

int RansacControl::consume(const int32_t* cnt, const int32_t* good, int D) {
  D = std::min(D, pending_);
  pending_ = 0;
  int best_d = -1;
  for (int d = 0; d < D && !done_; ++d) {
    ++draws_;
    if (!good[d]) {
      if (++consec_bad_ >= 1000) done_ = true;  // getSamples: no valid sample in 1000 tries
      continue;
    }
    consec_bad_ = 0;
    const int n = cnt[d];
    if (n > best_) {
      best_ = n;
      best_d = d;
      best_draw_ = batch_base_ + d;
      have_ = true;
      const double w = (double)best_ * one_over_indices_;
      double p_no_outliers = 1.0 - std::pow(w, 3.0);
      p_no_outliers = std::max(std::numeric_limits<double>::epsilon(), p_no_outliers);
      p_no_outliers = std::min(1.0 - std::numeric_limits<double>::epsilon(), p_no_outliers);
      k_ = log_probability_ / std::log(p_no_outliers);
    }
    ++iterations_;
    tests_ += N_;
    if (iterations_ > prm_.max_iterations) done_ = true;
    else if (!(iterations_ < k_)) done_ = true;
  }
  return best_d;
}

}  // namespace dlg

// ---- C ABI ------------------------------------------------------------------------------------

struct dlg_sac_control {
  dlg::RansacControl ctl;
  dlg_sac_control(const dlg_sac_params& p, int64_t n, int cap) : ctl(p, n, cap) {}
};

extern "C" {

dlg_status dlg_sac_control_create(dlg_sac_control** out, const dlg_sac_params* prm,
                                  int64_t n_active_global, int max_batch) {
  if (!out || !prm || n_active_global < 0 || n_active_global > INT32_MAX || max_batch < 0)
    return DLG_ERR_INVALID;
  *out = nullptr;
  if (!(prm->probability == prm->probability)) return DLG_ERR_INVALID;
  dlg_sac_control* c = new (std::nothrow) dlg_sac_control(*prm, n_active_global,
                                                          max_batch > 0 ? max_batch : 4096);
  if (!c) return DLG_ERR_INTERNAL;
  *out = c;
  return DLG_OK;
}

dlg_status dlg_sac_control_destroy(dlg_sac_control* c) {
  delete c;
  return DLG_OK;
}

dlg_status dlg_sac_control_next(dlg_sac_control* c, int32_t* positions_out, int64_t cap,
                                int* n_draws) {
  if (!c || !n_draws) return DLG_ERR_INVALID;
  const int D = c->ctl.next_size();
  *n_draws = D;
  if (3 * (int64_t)D > cap) return DLG_ERR_CAPACITY;
  if (D > 0 && !positions_out) return DLG_ERR_INVALID;
  c->ctl.next_batch(positions_out);
  return DLG_OK;
}

dlg_status dlg_sac_control_consume(dlg_sac_control* c, const int32_t* counts, const int32_t* good,
                                   int n_draws, int* best_in_batch, int* finished) {
  if (!c || (n_draws > 0 && (!counts || !good)) || n_draws < 0) return DLG_ERR_INVALID;
  const int b = c->ctl.consume(counts, good, n_draws);
  if (best_in_batch) *best_in_batch = b;
  if (finished) *finished = c->ctl.done() ? 1 : 0;
  return DLG_OK;
}

dlg_status dlg_sac_control_result(const dlg_sac_control* c, dlg_sac_stats* st,
                                  int64_t* best_draw) {
  if (!c || !st) return DLG_ERR_INVALID;
  *st = dlg_sac_stats{};
  st->iterations = c->ctl.iterations();
  st->has_model = c->ctl.have_model() ? 1 : 0;
  st->draws = c->ctl.draws();
  st->n_unrefined = c->ctl.have_model() ? c->ctl.best_count() : 0;
  st->tests = c->ctl.tests();
  st->n_active = c->ctl.n();
  if (best_draw) *best_draw = c->ctl.best_draw();
  return DLG_OK;
}

}  // extern "C"
