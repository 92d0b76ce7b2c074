// fsum_host.cpp -- host emulation of the device's parallel exact float sums (test harness).
//
// Builds the same records as the kernels of dialog_amd/csrc/fsum.hip (level-1 fan runs around
// the double-prefix guesses, level-L walks of 64 children from each member start, the top walk
// from +0 with descents), with the product's header fsum.hpp, so the CPU test suite can check the
// algorithm against the literal sequential loop on inputs too large or too adversarial to run
// through the GPU in every test.  Compiled with g++ -ffp-contract=off (tests/test_fsum.py).
#include <cmath>
#include <cstdint>
#include <cstring>
#include <vector>

#include "../../dialog_amd/csrc/fsum.hpp"

using namespace dlg;

namespace {

struct HostStore {
  const float *x, *y, *z;
  int64_t n;
  int chain;
  std::vector<std::vector<FsNode>> lv;  // lv[L] for L >= 1
  const FsNode& node(int L, int64_t k) const { return lv[L][k]; }
  int64_t nodes(int L) const { return (int64_t)lv[L].size(); }
  FsRun rerun(int64_t k, float v) const {
    FsState st = fs_start(v);
    const int64_t e1 = std::min<int64_t>(n, (k + 1) * kFsChunk);
    for (int64_t j = k * kFsChunk; j < e1; ++j) fs_step(st, fs_term(chain, x[j], y[j], z[j]));
    return fs_finish(st);
  }
};

// levels until the top holds <= top_max nodes
int fs_levels(int64_t n, int top_max) {
  int L = 1;
  while (fs_nodes(n, L) > top_max) ++L;
  return L;
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

// the parallel algorithm, emulated; guess_noise != 0 perturbs every guess by that many quanta
// (exercises the descent paths); stats[3] = applied, reruns, descents of the top walks
int fs_host(const float* x, const float* y, const float* z, int64_t n, int top_max,
            int guess_noise, float out[9], int64_t stats[3]) {
  stats[0] = stats[1] = stats[2] = 0;
  for (int c = 0; c < 9; ++c) {
    if (n == 0) {
      out[c] = 0.0f;
      continue;
    }
    HostStore st{x, y, z, n, c, {}};
    const int L = fs_levels(n, top_max);
    st.lv.resize(L + 1);
    // guesses: the double prefix of the terms at every chunk start
    const int64_t K = fs_nodes(n, 1);
    std::vector<float> g(K);
    double pre = 0.0;
    for (int64_t k = 0; k < K; ++k) {
      float gk = (float)pre;
      if (guess_noise && k > 0) {
        const float q = fs_quantum(gk);
        gk = (float)((double)gk + (double)((k * 7919) % (2 * guess_noise + 1) - guess_noise) * q);
      }
      g[k] = gk;
      const int64_t e1 = std::min<int64_t>(n, (k + 1) * kFsChunk);
      double s = 0.0;
      for (int64_t j = k * kFsChunk; j < e1; ++j) s += (double)fs_term(c, x[j], y[j], z[j]);
      pre += s;
    }
    // level 1: fan runs
    st.lv[1].resize(K);
    for (int64_t k = 0; k < K; ++k) {
      FsNode& nd = st.lv[1][k];
      nd.g = g[k];
      nd.pad0 = nd.pad1 = nd.pad2 = 0.0f;
      for (int i = 0; i < kFsFan; ++i) {
        float a;
        if (!fs_member_start(g[k], i, &a)) {
          nd.o[i] = nd.mu[i] = 0.0f;
          nd.qm[i] = NAN;
          continue;
        }
        const FsRun r = st.rerun(k, a);
        nd.o[i] = r.o;
        nd.mu[i] = r.mu;
        nd.qm[i] = r.qm;
      }
    }
    // levels 2..L: walks from each member start
    for (int l = 2; l <= L; ++l) {
      const int64_t M = fs_nodes(n, l), Mc = fs_nodes(n, l - 1);
      st.lv[l].resize(M);
      for (int64_t k = 0; k < M; ++k) {
        FsNode& nd = st.lv[l][k];
        const int64_t c0 = k * kFsArity, cnt = std::min<int64_t>(kFsArity, Mc - c0);
        nd.g = st.lv[l - 1][c0].g;  // (the guess at the node's first element)
        nd.pad0 = nd.pad1 = nd.pad2 = 0.0f;
        for (int i = 0; i < kFsFan; ++i) {
          float a;
          if (!fs_member_start(nd.g, i, &a)) {
            nd.o[i] = nd.mu[i] = 0.0f;
            nd.qm[i] = NAN;
            continue;
          }
          float mu = INFINITY, qm = 0.0f;
          nd.o[i] = fs_walk(st, l - 1, c0, cnt, a, &mu, &qm, nullptr);
          nd.mu[i] = mu;
          nd.qm[i] = qm;
        }
      }
    }
    // top walk from +0
    float mu = INFINITY, qm = 0.0f;
    FsWalkStats ws;
    out[c] = fs_walk(st, L, 0, st.nodes(L), 0.0f, &mu, &qm, &ws);
    stats[0] += ws.applied;
    stats[1] += ws.reruns;
    stats[2] += ws.descents;
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
