// Micro-benchmark of the fast refit's device arithmetic (exact_refit.hpp) on one workgroup:
// entries (big integer -> double) and the Jacobi finish, timed with HIP events over many launches.
// Build: hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -std=c++17 tools/ubench_refit.hip -o tools/ubench_refit
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

#include "../dialog_amd/csrc/exact_refit.hpp"

using namespace dlg;

__global__ void k_entries(const int64_t* dig, double* out) {
  if (threadIdx.x < 9) out[threadIdx.x] = refit_entry(dig, threadIdx.x);
}

__global__ void k_finish(const double* e, const int64_t* dig, float* out) {
  if (threadIdx.x != 0) return;
  double ee[9];
  for (int k = 0; k < 9; ++k) ee[k] = e[k];
  const float cin[4] = {0.f, 0.f, 1.f, 0.f};
  refit_finish(ee, dig[0], 3, cin, out);
}

__global__ void k_jacobi(const double* e, double* out, int* sweeps) {
  if (threadIdx.x != 0) return;
  double A[9] = {e[0], e[1], e[2], e[1], e[3], e[4], e[2], e[4], e[5]}, V[9];
  jacobi3(A, V);
  for (int k = 0; k < 9; ++k) out[k] = V[k];
}

__global__ void k_empty() {}

// the device accumulation path: 64 lanes, each a strided share of the points, flushed every
// kMomFlush points, digits summed over the lanes; then the nine entries and the finish
__global__ void k_acc(const float* xyz, int n, double qs, int64_t* dig_out, float* out) {
  int64_t acc[kMomDigits];
  for (int k = 0; k < kMomDigits; ++k) acc[k] = 0;
  MomAcc m;
  mom_zero(m);
  int since = 0;
  for (int i = threadIdx.x; i < n; i += 64) {
    mom_point(m, fast_q(xyz[3 * i], qs), fast_q(xyz[3 * i + 1], qs), fast_q(xyz[3 * i + 2], qs));
    if (++since == kMomFlush) { mom_flush(acc, m); since = 0; }
  }
  mom_flush(acc, m);
  for (int k = 0; k < kMomDigits; ++k) {
    int64_t v = acc[k];
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    acc[k] = v;
  }
  if (threadIdx.x == 0) {
    for (int k = 0; k < kMomDigits; ++k) dig_out[k] = acc[k];
    const float cin[4] = {0.f, 0.f, 1.f, 0.f};
    refit_exact(acc, 3, cin, out);
  }
}

int main() {
  // digits of ~500k points on a tilted plane (host accumulation)
  std::vector<int64_t> dig(kMomDigits, 0);
  std::vector<float> pts;
  const double qs = pow2d(kFastBits - 3);
  unsigned s = 12345;
  MomAcc ma;
  mom_zero(ma);
  for (int i = 0; i < 500000; ++i) {
    s = s * 1664525u + 1013904223u;
    const float u = (s >> 8) * 0x1p-24f * 4.f - 2.f;
    s = s * 1664525u + 1013904223u;
    const float v = (s >> 8) * 0x1p-24f * 4.f - 2.f;
    s = s * 1664525u + 1013904223u;
    const float w = ((s >> 8) * 0x1p-24f - 0.5f) * 0.01f;
    const float x = u, y = v, z = 0.3f * u - 0.2f * v + 1.0f + w;
    mom_point(ma, fast_q(x, qs), fast_q(y, qs), fast_q(z, qs));
    mom_flush(dig.data(), ma);
    pts.push_back(x); pts.push_back(y); pts.push_back(z);
  }
  int64_t* d_dig;
  double *d_e, *d_o;
  float* d_f;
  int* d_s;
  hipMalloc(&d_dig, 8 * kMomDigits);
  hipMalloc(&d_e, 8 * 16);
  hipMalloc(&d_o, 8 * 16);
  hipMalloc(&d_f, 16);
  hipMalloc(&d_s, 4);
  hipMemcpy(d_dig, dig.data(), 8 * kMomDigits, hipMemcpyHostToDevice);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  auto time = [&](const char* name, auto launch) {
    for (int i = 0; i < 10; ++i) launch();
    hipDeviceSynchronize();
    hipEventRecord(a);
    const int R = 200;
    for (int i = 0; i < R; ++i) launch();
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms = 0;
    hipEventElapsedTime(&ms, a, b);
    std::printf("%-10s %8.2f us/launch\n", name, 1000.0 * ms / R);
  };
  time("empty", [&] { hipLaunchKernelGGL(k_empty, dim3(1), dim3(64), 0, 0); });
  time("entries", [&] { hipLaunchKernelGGL(k_entries, dim3(1), dim3(64), 0, 0, d_dig, d_e); });
  time("jacobi", [&] { hipLaunchKernelGGL(k_jacobi, dim3(1), dim3(64), 0, 0, d_e, d_o, d_s); });
  time("finish", [&] { hipLaunchKernelGGL(k_finish, dim3(1), dim3(64), 0, 0, d_e, d_dig, d_f); });
  float f[4];
  hipMemcpy(f, d_f, 16, hipMemcpyDeviceToHost);
  {
    float* d_p;
    int64_t* d_dg;
    float* d_f2;
    hipMalloc(&d_p, 4 * pts.size());
    hipMalloc(&d_dg, 8 * kMomDigits);
    hipMalloc(&d_f2, 16);
    hipMemcpy(d_p, pts.data(), 4 * pts.size(), hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k_acc, dim3(1), dim3(64), 0, 0, d_p, (int)(pts.size() / 3), qs, d_dg, d_f2);
    std::vector<int64_t> dg(kMomDigits);
    float f2[4];
    hipMemcpy(dg.data(), d_dg, 8 * kMomDigits, hipMemcpyDeviceToHost);
    hipMemcpy(f2, d_f2, 16, hipMemcpyDeviceToHost);
    std::printf("device-accumulated refit %a %a %a %a  n=%lld\n", f2[0], f2[1], f2[2], f2[3], (long long)dg[0]);
    double e1[9], e2[9];
    for (int k = 0; k < 9; ++k) { e1[k] = refit_entry(dig.data(), k); e2[k] = refit_entry(dg.data(), k); }
    for (int k = 0; k < 9; ++k) std::printf("entry %d host %a devdigits %a\n", k, e1[k], e2[k]);
  }
  float h[4];
  const float cin[4] = {0.f, 0.f, 1.f, 0.f};
  refit_exact(dig.data(), 3, cin, h);
  std::printf("device %a %a %a %a\nhost   %a %a %a %a\n", f[0], f[1], f[2], f[3], h[0], h[1], h[2], h[3]);
  return 0;
}
