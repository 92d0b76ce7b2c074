// Stand-alone check of the fast-refit moments launch (kernels.hip compiled into this program):
// launch_moments_refit / launch_moments on a synthetic plane, the result against the host's
// refit_exact of the same inliers.  Build:
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fno-slp-vectorize \
//     -fhip-fp32-correctly-rounded-divide-sqrt -mllvm -amdgpu-mfma-vgpr-form \
//     -Idialog_amd/csrc tools/dbg_moments.hip -o tools/dbg_moments
#include "../dialog_amd/csrc/kernels.hip"

#include <cstdio>
#include <vector>

using namespace dlg;

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      std::printf("HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
      return 1;                                                                 \
    }                                                                           \
  } while (0)

int main() {
  const int n = 1000000;
  std::vector<float> x(n), y(n), z(n);
  unsigned s = 99;
  for (int i = 0; i < n; ++i) {
    s = s * 1664525u + 1013904223u;
    const float u = (s >> 8) * 0x1p-24f * 4.f - 2.f;
    s = s * 1664525u + 1013904223u;
    const float v = (s >> 8) * 0x1p-24f * 4.f - 2.f;
    s = s * 1664525u + 1013904223u;
    const float w = ((s >> 8) * 0x1p-24f - 0.5f) * (i % 3 == 0 ? 2.0f : 0.01f);
    x[i] = u; y[i] = v; z[i] = 0.3f * u - 0.2f * v + 1.0f + w;
  }
  const int qexp = 3;
  float *dx, *dy, *dz;
  CK(hipMalloc(&dx, 4 * n)); CK(hipMalloc(&dy, 4 * n)); CK(hipMalloc(&dz, 4 * n));
  CK(hipMemcpy(dx, x.data(), 4 * n, hipMemcpyHostToDevice));
  CK(hipMemcpy(dy, y.data(), 4 * n, hipMemcpyHostToDevice));
  CK(hipMemcpy(dz, z.data(), 4 * n, hipMemcpyHostToDevice));
  // plane z = 0.3x - 0.2y + 1 normalised (PCL-style coefficients)
  const double nn = std::sqrt(0.09 + 0.04 + 1.0);
  const float4 pl = make_float4((float)(0.3 / nn), (float)(-0.2 / nn), (float)(-1.0 / nn), (float)(1.0 / nn));
  float4* dpl;
  CK(hipMalloc(&dpl, 2 * sizeof(float4)));
  CK(hipMemcpy(dpl, &pl, sizeof(float4), hipMemcpyHostToDevice));
  ModelTest mt{};
  mt.thr = 0.02;
  mt.cthr = 0.02f;
  mt.normal_plane = 0;
  const int nb = moments_blocks(n);
  int64_t *part, *out;
  unsigned* done;
  CK(hipMalloc(&part, 8 * (size_t)nb * kMomDigits));
  CK(hipMalloc(&out, 8 * kMomDigits));
  CK(hipMalloc(&done, 4));
  CK(hipMemset(done, 0, 4));
  CK(hipMemset(dpl + 1, 0, sizeof(float4)));
  PointsView v{dx, dy, dz, nullptr, n, nullptr};
  launch_moments_refit(v, dpl, mt, qexp, part, done, nb, out, dpl + 1, 0);
  CK(hipGetLastError());
  CK(hipDeviceSynchronize());
  std::vector<int64_t> dg(kMomDigits);
  float4 rc;
  unsigned dn = 7;
  CK(hipMemcpy(dg.data(), out, 8 * kMomDigits, hipMemcpyDeviceToHost));
  CK(hipMemcpy(&rc, dpl + 1, sizeof(float4), hipMemcpyDeviceToHost));
  CK(hipMemcpy(&dn, done, 4, hipMemcpyDeviceToHost));
  // host: the same inliers (PCL's test in double as model_in)
  std::vector<int64_t> hd(kMomDigits, 0);
  MomAcc m;
  mom_zero(m);
  const double qs = pow2d(kFastBits - qexp);
  for (int i = 0; i < n; ++i) {
    const float d = std::fabs((pl.x * x[i] + pl.z * z[i]) + (pl.y * y[i] + pl.w * 1.0f));
    if ((double)d < mt.thr) {
      mom_point(m, fast_q(x[i], qs), fast_q(y[i], qs), fast_q(z[i], qs));
      mom_flush(hd.data(), m);
    }
  }
  const float cin[4] = {pl.x, pl.y, pl.z, pl.w};
  float hc[4];
  refit_exact(hd.data(), qexp, cin, hc);
  std::printf("nb %d done %u  device n %lld host n %lld\n", nb, dn, (long long)dg[0], (long long)hd[0]);
  std::printf("device %a %a %a %a\nhost   %a %a %a %a\n", rc.x, rc.y, rc.z, rc.w, hc[0], hc[1], hc[2], hc[3]);
  return 0;
}
