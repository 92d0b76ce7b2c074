// fsum_host.cpp -- host emulation of the device's parallel exact float sums (test harness).
//
// Builds the same chunk records as the kernels of dialog_amd/csrc/fsum.hip (fan runs around the
// guesses refined from the double prefix by the chunks' float increments) and walks them as k_fs_walk does -- windows of W records, speculative
// starts from the prefix of the record increments, verification lane by lane, the first failed
// lane applied or rerun alone -- with the product's header fsum.hpp, so the CPU test suite can
// check the algorithm against the literal sequential loop on inputs too large or too
// adversarial to run through the GPU in every test.  Compiled with g++ -ffp-contract=off
// (tests/test_fsum.py).
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <vector>

#include "../../dialog_amd/csrc/fsum.hpp"

using namespace dlg;

namespace {

FsRun run_chunk(const float* x, const float* y, const float* z, int64_t n, int c, int64_t k,
                float v) {
  FsState st = fs_start(v);
  const int64_t e1 = std::min<int64_t>(n, (k + 1) * kFsChunk);
  for (int64_t j = k * kFsChunk; j < e1; ++j) fs_step(st, fs_term(c, x[j], y[j], z[j]));
  return fs_finish(st);
}

}  // namespace

extern "C" {

// the literal loop (PCL's dense branch of computeMeanAndCovarianceMatrix)
void fs_literal(const float* x, const float* y, const float* z, int64_t n, float out[9]) {
  float a[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
  for (int64_t i = 0; i < n; ++i)
    for (int c = 0; c < 9; ++c) a[c] = a[c] + fs_term(c, x[i], y[i], z[i]);
  std::memcpy(out, a, sizeof(a));
}

// the parallel algorithm, emulated with windows of `width` records (the device: 64);
// guess_noise != 0 perturbs every guess by that many quanta (exercises the failed lanes and the
// reruns); stats[3] = verified lanes, lanes handled alone by their record, reruns
int fs_host(const float* x, const float* y, const float* z, int64_t n, int width,
            int guess_noise, float out[9], int64_t stats[3]) {
  stats[0] = stats[1] = stats[2] = 0;
  const int64_t K = fs_chunks(n);
  for (int c = 0; c < 9; ++c) {
    // first guesses: the double prefix of the terms at every chunk start (k_fs_prep); the
    // chunk's float increment from there (k_fs_inc); refined guesses: the prefix of the
    // increments (k_fs_l1)
    std::vector<FsNode> rec(K);
    std::vector<double> inc(K);
    double pre = 0.0;
    for (int64_t k = 0; k < K; ++k) {
      const float g0 = (float)pre;
      inc[k] = (double)run_chunk(x, y, z, n, c, k, g0).o - (double)g0;
      const int64_t e1 = std::min<int64_t>(n, (k + 1) * kFsChunk);
      double s = 0.0;
      for (int64_t j = k * kFsChunk; j < e1; ++j) s += (double)fs_term(c, x[j], y[j], z[j]);
      pre += s;
    }
    double rpre = 0.0;
    for (int64_t k = 0; k < K; ++k) {
      float gk = (float)rpre;
      rpre += inc[k];
      if (guess_noise && k > 0) {
        const float q = fs_quantum(gk);
        gk = (float)((double)gk + (double)((k * 7919) % (2 * guess_noise + 1) - guess_noise) * q);
      }
      FsNode& nd = rec[k];
      nd.g = gk;
      nd.pad0 = nd.pad1 = nd.pad2 = 0.0f;
      for (int i = 0; i < kFsFan; ++i) {
        float a;
        if (!fs_member_start(gk, i, &a)) {
          nd.o[i] = nd.mu[i] = 0.0f;
          nd.qm[i] = NAN;
          continue;
        }
        const FsRun r = run_chunk(x, y, z, n, c, k, a);
        nd.o[i] = r.o;
        nd.mu[i] = r.mu;
        nd.qm[i] = r.qm;
      }
    }
    // the walk (k_fs_walk)
    float t = 0.0f;
    std::vector<float> res(width);
    std::vector<char> ver(width);
    for (int64_t base = 0; base < K; base += width) {
      const int cnt = (int)std::min<int64_t>(width, K - base);
      int s = 0;
      while (s < cnt) {
        double acc = 0.0;
        int f = -1;
        const double off = (double)t - (double)rec[base + s].g;  // the walk's lead on the guesses
        for (int l = s; l < cnt; ++l) {
          const FsNode& nd = rec[base + l];
          const double tl = (double)t + acc;  // speculated start: t + increments of lanes s..l-1
          acc += fs_increment(nd, off);
          const float tf = (float)tl;
          FsApply a;
          a.out = 0.0f;
          const bool ok = (double)tf == tl && fs_apply(tf, nd, &a);
          res[l] = a.out;
          if (!(ok && (double)a.out == (double)t + acc)) {
            f = l;
            break;
          }
          stats[0]++;
        }
        if (f < 0) {
          t = res[cnt - 1];
          break;
        }
        const float tfx = f == s ? t : res[f - 1];  // exact: lanes s..f-1 verified
        FsApply a2;
        if (fs_apply(tfx, rec[base + f], &a2)) {
          t = a2.out;
          stats[1]++;
        } else {
          t = run_chunk(x, y, z, n, c, base + f, tfx).o;
          stats[2]++;
        }
        s = f + 1;
      }
    }
    out[c] = t;
  }
  return 0;
}
// the refit tail (device arithmetic of fsum.hpp) on the host: cout, *uncertain
void fs_refit_host(const float a[9], int64_t n, const float cin[4], float cout[4], int* uncertain) {
  bool u = false;
  fs_refit_tail(a, n, cin, cout, &u);
  *uncertain = u ? 1 : 0;
}

// the product's host refit (host_math.hpp refit_pcl_float) for comparison
void fs_refit_pcl_host(const float* xyz, int64_t n, const float cin[4], float cout[4]) {
  refit_pcl_float(xyz, n, cin, cout);
}

}  // extern "C"
