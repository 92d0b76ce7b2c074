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
#include <memory>
#include <vector>

#include "../../include/dialog_ransac.h"
#include "host_math.hpp"

namespace dlg {

// sparse overlay of SampleConsensusModel::shuffled_indices_ over list positions: pos -> pos'.
// Open addressing with interleaved (key, value, generation) slots; reset() bumps the
// generation instead of clearing, so a table reused across segments costs nothing to reset.
class Overlay {
 public:
  void reset(size_t expect);
  // returns the value at k (k itself when absent) and stores v there: one probe sequence
  int32_t exchange(int32_t k, int32_t v) {
    size_t h = hash(k) & mask_;
    for (;;) {
      Slot& s = slots_[h];
      if (s.gen != gen_) {  // empty in this generation: insert
        s.gen = gen_;
        s.key = k;
        s.val = v;
        if (++size_ * 4 > slots_.size()) grow();
        return k;
      }
      if (s.key == k) {
        const int32_t old = s.val;
        s.val = v;
        return old;
      }
      h = (h + 1) & mask_;
    }
  }

 private:
  struct Slot {
    int32_t key, val;
    uint32_t gen;
  };
  static size_t hash(int32_t k) { return (size_t)((uint32_t)k * 2654435761u); }
  void grow();
  std::vector<Slot> slots_;
  size_t mask_ = 0, size_ = 0;
  uint32_t gen_ = 0;
};

// drawIndexSample's swaps over list positions: positions 0..2 (touched by every draw) live in
// registers, the random partners >= 3 in the overlay -- one probe sequence per swap
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
    head_[i] = tail_.exchange((int32_t)j, head_[i]);
  }
  int32_t at(int i) const { return head_[i]; }

 private:
  int32_t head_[3] = {0, 1, 2};
  Overlay tail_;
};

// x mod d for 32-bit x and a fixed 32-bit d >= 1 without a division (Lemire, Kaser & Kurz,
// "Faster remainder by direct computation", 2019): exact for every 32-bit x
class FastMod32 {
 public:
  explicit FastMod32(uint32_t d = 1) : d_(d), m_(UINT64_C(0xFFFFFFFFFFFFFFFF) / d + 1) {}
  uint32_t mod(uint32_t x) const {
    const uint64_t low = m_ * x;
    return (uint32_t)(((__uint128_t)low * d_) >> 64);
  }

 private:
  uint32_t d_;
  uint64_t m_;
};

class RansacControl {
 public:
  // N = active points over all ranks; cap_h = largest batch the caller can score at once;
  // replay: a table to reuse across segments (the context's; nullptr: the controller owns one)
  RansacControl(const dlg_sac_params& prm, int64_t N, int cap_h, ShuffleReplay* replay = nullptr);

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
  uint32_t seed_;
  int64_t rnd_pos_ = 0;  // rnd() values consumed (the stream restarts at the seed every segment)
  std::unique_ptr<ShuffleReplay> own_;
  ShuffleReplay* ov_;
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
