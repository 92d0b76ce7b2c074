// Host-only sanitizer harness (ASan + UBSan, built by tests/test_sanitizers.py with g++) for the
// product's host-sequential RANSAC code: dialog_amd/csrc/sac_control.cpp (RansacControl: the
// drawIndexSample replay over list positions and computeModel's loop, through its C ABI
// dlg_sac_control_*) and host_math.hpp (Boost mt19937 rnd(), refit_pcl_float, eigen33<float>).
// The scorer here is a brute-force PCL countWithinDistance on the host; the harness prints the
// result so the test can compare it with the oracle.
//   stdin: "n threshold max_iterations probability batch" then n lines "x y z" (hex floats)
//   stdout: "iterations draws has_model best0 best1 best2 n_unrefined c0 c1 c2 c3" (coefficient
//           bits in hex, PCL float refit + re-selection)
#include <cmath>
#include <cstdio>
#include <cstring>
#include <vector>

#include "../../dialog_amd/csrc/host_math.hpp"
#include "../../include/dialog_ransac.h"

namespace {

float pcl_abs(const float c[4], const float* p) {
  return std::fabs((c[0] * p[0] + c[2] * p[2]) + (c[1] * p[1] + c[3] * 1.0f));
}

bool plane_of(const float* p0, const float* p1, const float* p2, float c[4], bool* good) {
  const float a0 = p1[0] - p0[0], a1 = p1[1] - p0[1], a2 = p1[2] - p0[2];
  const float b0 = p2[0] - p0[0], b1 = p2[1] - p0[1], b2 = p2[2] - p0[2];
  const float r0 = a0 / b0, r1 = a1 / b1, r2 = a2 / b2;
  *good = (r0 != r1) || (r2 != r1);
  if (!*good) return false;
  float c0 = a1 * b2 - a2 * b1, c1 = a2 * b0 - a0 * b2, c2 = a0 * b1 - a1 * b0, c3 = 0.0f;
  const float z = (c0 * c0 + c2 * c2) + (c1 * c1 + c3 * c3);
  if (z > 0.0f) {
    const float s = std::sqrt(z);
    c0 /= s; c1 /= s; c2 /= s; c3 /= s;
  }
  const float dot = (c0 * p0[0] + c2 * p0[2]) + (c1 * p0[1] + c3 * 1.0f);
  c[0] = c0; c[1] = c1; c[2] = c2; c[3] = -1.0f * dot;
  return true;
}

}  // namespace

int main() {
  long long n = 0;
  double thr = 0, prob = 0;
  int maxit = 0, batch = 0;
  if (std::scanf("%lld %lf %d %lf %d", &n, &thr, &maxit, &prob, &batch) != 5) return 2;
  std::vector<float> p(3 * (size_t)n);
  for (long long i = 0; i < n; ++i)
    if (std::scanf("%a %a %a", &p[3 * i], &p[3 * i + 1], &p[3 * i + 2]) != 3) return 3;
  dlg_sac_params prm;  // (PCL defaults; dlg_sac_params_default lives in the HIP driver)
  std::memset(&prm, 0, sizeof(prm));
  prm.optimize = 1;
  prm.seed = 12345u;
  prm.model = DLG_SACMODEL_PLANE;
  prm.normal_distance_weight = 0.1;
  prm.threshold = thr;
  prm.max_iterations = maxit;
  prm.probability = prob;
  const float cthr = dlg::thr_ceil(thr);
  dlg_sac_control* ctl = nullptr;
  if (dlg_sac_control_create(&ctl, &prm, n, batch) != DLG_OK) return 4;
  std::vector<int32_t> pos, cnt, good;
  std::vector<float> coef;
  int64_t drawn = 0;
  int32_t bestp[3] = {-1, -1, -1};
  for (;;) {
    int d = 0;
    pos.resize(3 * (size_t)(batch > 0 ? batch : 4096));
    if (dlg_sac_control_next(ctl, pos.data(), (int64_t)pos.size(), &d) != DLG_OK) return 5;
    if (d == 0) break;
    cnt.assign(d, 0);
    good.assign(d, 0);
    coef.resize(4 * (size_t)d);
    for (int k = 0; k < d; ++k) {
      float* c = &coef[4 * k];
      bool g = false;
      if (!plane_of(&p[3 * pos[3 * k]], &p[3 * pos[3 * k + 1]], &p[3 * pos[3 * k + 2]], c, &g)) {
        good[k] = 0;
        continue;
      }
      good[k] = 1;
      int m = 0;
      for (long long i = 0; i < n; ++i) m += pcl_abs(c, &p[3 * i]) < cthr ? 1 : 0;
      cnt[k] = m;
    }
    int best = -1, fin = 0;
    if (dlg_sac_control_consume(ctl, cnt.data(), good.data(), d, &best, &fin) != DLG_OK) return 6;
    if (best >= 0)
      for (int i = 0; i < 3; ++i) bestp[i] = pos[3 * best + i];
    drawn += d;
    if (fin) break;
  }
  dlg_sac_stats st;
  int64_t best_draw = -1;
  if (dlg_sac_control_result(ctl, &st, &best_draw) != DLG_OK) return 7;
  dlg_sac_control_destroy(ctl);
  if (!st.has_model) {
    std::printf("%d %lld 0\n", st.iterations, (long long)st.draws);
    return 0;
  }
  // the winner (list positions = point indices: the list is 0..n-1)
  const float* q[3];
  for (int i = 0; i < 3; ++i) q[i] = &p[3 * (size_t)bestp[i]];
  float c[4];
  bool g = false;
  plane_of(q[0], q[1], q[2], c, &g);
  std::vector<float> inl;
  for (long long i = 0; i < n; ++i)
    if (pcl_abs(c, &p[3 * i]) < cthr) inl.insert(inl.end(), &p[3 * i], &p[3 * i] + 3);
  const long long nu = (long long)(inl.size() / 3);
  float rc[4];
  dlg::refit_pcl_float(inl.data(), nu, c, rc);
  unsigned u[4];
  std::memcpy(u, rc, 16);
  std::printf("%d %lld 1 %d %d %d %lld %08x %08x %08x %08x\n", st.iterations, (long long)st.draws,
              bestp[0], bestp[1], bestp[2], nu, u[0], u[1], u[2], u[3]);
  return 0;
}
