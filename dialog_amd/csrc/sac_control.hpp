// sac_control.hpp -- the host-sequential half of PCL 1.8's RANSAC, separated from the device work.
//
// RandomSampleConsensus<PointXYZ>::computeModel [PCL-1.8 ext; SURVEY.md §8(a) a6] interleaves
// three things per iteration: getSamples / drawIndexSample (RNG + swaps on a persistent shuffled
// copy of the indices, a7), countWithinDistance (a9) and the best/k bookkeeping.  Only the count
// touches the point data, and which list *positions* drawIndexSample swaps depends on the RNG
// stream and N_active alone.  RansacControl owns the two data-independent parts:
//
//   next_batch()  replays D draws over list positions (mt19937(seed) >> 1, the three swaps
//                 swap(shuf[i], shuf[i + rnd() % (N - i)]) kept in a sparse overlay) -> 3*D
//                 global list positions;
//   consume()     replays computeModel's loop over the D (good, count) pairs in draw order:
//                 a bad draw consumes a getSamples try (1000 in a row end the loop), strict '>'
//                 keeps the first best, k = log(1-p)/log(clamp(1-w^3)), iteration cap.
//
// The caller maps positions to points and counts inliers -- the device kernels in driver.cpp, or
// (tests) any other scorer.  With point shards every rank runs an identical controller on the
// global N and the summed counts, so all ranks take identical decisions.
// No HIP here: the controller is plain C++ and is exported through the dlg_sac_control_* C ABI.
#pragma once

#include <cstdint>
#include <vector>

#include "../../include/dialog_ransac.h"
#include "host_math.hpp"

namespace dlg {

// sparse overlay of SampleConsensusModel::shuffled_indices_ over list positions: pos -> pos'
class Overlay {
 public:
  void reset(size_t expect);
  int32_t get(int32_t k) const {
    size_t h = hash(k) & mask_;
    while (keys_[h] != -1) {
      if (keys_[h] == k) return vals_[h];
      h = (h + 1) & mask_;
    }
    return k;
  }
  void set(int32_t k, int32_t v) {
    if ((size_ + 1) * 2 > keys_.size()) grow();
    size_t h = hash(k) & mask_;
    while (keys_[h] != -1 && keys_[h] != k) h = (h + 1) & mask_;
    if (keys_[h] == -1) {
      keys_[h] = k;
      ++size_;
    }
    vals_[h] = v;
  }

 private:
  static size_t hash(int32_t k) { return (size_t)((uint32_t)k * 2654435761u); }
  void grow();
  std::vector<int32_t> keys_, vals_;
  size_t mask_ = 0, size_ = 0;
};

// drawIndexSample's swaps over list positions: positions 0..2 (touched by every draw) live in
// registers, the random partners >= 3 in the overlay -- one hash lookup and one insert per swap
class ShuffleReplay {
 public:
  void reset(size_t expect) {
    head_[0] = 0; head_[1] = 1; head_[2] = 2;
    tail_.reset(expect);
  }
  void swap(int i, int64_t j) {
    if (j < 3) {
      const int32_t t = head_[i];
      head_[i] = head_[j];
      head_[j] = t;
      return;
    }
    const int32_t vj = tail_.get((int32_t)j);
    tail_.set((int32_t)j, head_[i]);
    head_[i] = vj;
  }
  int32_t at(int i) const { return head_[i]; }

 private:
  int32_t head_[3] = {0, 1, 2};
  Overlay tail_;
};

class RansacControl {
 public:
  // N = active points over all ranks; cap_h = largest batch the caller can score at once
  RansacControl(const dlg_sac_params& prm, int64_t N, int cap_h);

  bool done() const { return done_; }
  // batch size PCL can still use (0 once the loop has ended)
  int next_size() const;
  // draws the next batch (size next_size()) -> pos[3*D] list positions; returns D
  int next_batch(int32_t* pos);
  // replays computeModel over the batch just drawn; returns the batch index of the best
  // hypothesis found in this batch (-1: the best is unchanged)
  int consume(const int32_t* counts, const int32_t* good, int D);

  bool have_model() const { return have_; }
  int iterations() const { return iterations_; }
  int best_count() const { return best_; }
  int64_t n() const { return N_; }
  int64_t draws() const { return draws_; }
  int64_t tests() const { return tests_; }
  int64_t batch_base() const { return batch_base_; }  // draw index of the current batch's first draw
  int64_t best_draw() const { return best_draw_; }    // global draw index of the best hypothesis

 private:
  dlg_sac_params prm_;
  int64_t N_;
  int cap_h_;
  Mt19937 rng_;
  ShuffleReplay ov_;
  int iterations_ = 0;
  int best_ = -2147483647;
  double k_ = 1.0;
  double log_probability_;
  double one_over_indices_;
  int consec_bad_ = 0;
  bool done_ = false, have_ = false;
  int pending_ = 0;           // size of the drawn batch not yet consumed
  int64_t draws_ = 0, tests_ = 0, batch_base_ = 0, best_draw_ = -1, drawn_ = 0;
};

}  // namespace dlg
