// mfma_f32_probe.hip -- checks v_mfma_f32_16x16x4_f32's operand / result lane maps on gfx950 and
// which f32 evaluation order it matches, for the MFMA tile scorer (spatial.hip, DLG_TILE_MFMA):
//   lane l supplies A[l & 15][l >> 4] and B[l >> 4][l & 15]; lane l receives D[4 (l >> 4) + r][l & 15].
// Prints the first mismatching element (exact-integer data), then over random f32 data how many
// results equal each candidate evaluation order (fmaf chains k = 0..3 and 3..0, the plain sum).
//   hipcc --offload-arch=gfx950 -O2 tools/mfma_f32_probe.hip -o /tmp/mfma_probe && /tmp/mfma_probe
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>

typedef float f32x4 __attribute__((ext_vector_type(4)));

__global__ void k_probe(const float* A, const float* B, float* D) {  // A [16][4], B [4][16], D [16][16]
  const int l = threadIdx.x;
  const float a = A[(l & 15) * 4 + (l >> 4)];
  const float b = B[(l >> 4) * 16 + (l & 15)];
  f32x4 z = {0.f, 0.f, 0.f, 0.f};
  f32x4 d = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, z, 0, 0, 0);
  for (int r = 0; r < 4; ++r) D[(4 * (l >> 4) + r) * 16 + (l & 15)] = d[r];
}

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      std::printf("%s: %s\n", #x, hipGetErrorString(e_));                      \
      return 1;                                                                 \
    }                                                                           \
  } while (0)

int main() {
  float hA[64], hB[64], hD[256];
  float *dA, *dB, *dD;
  CK(hipMalloc(&dA, sizeof(hA)));
  CK(hipMalloc(&dB, sizeof(hB)));
  CK(hipMalloc(&dD, sizeof(hD)));
  // exact integers, asymmetric: the maps
  for (int i = 0; i < 16; ++i)
    for (int k = 0; k < 4; ++k) hA[i * 4 + k] = (float)(i + 1) * (k == 0 ? 1 : k == 1 ? 32 : k == 2 ? 1024 : 32768);
  for (int k = 0; k < 4; ++k)
    for (int j = 0; j < 16; ++j) hB[k * 16 + j] = (float)((k + 1) * (j + 3) % 7 + 1);  // < 32: exact sums
  CK(hipMemcpy(dA, hA, sizeof(hA), hipMemcpyHostToDevice));
  CK(hipMemcpy(dB, hB, sizeof(hB), hipMemcpyHostToDevice));
  hipLaunchKernelGGL(k_probe, dim3(1), dim3(64), 0, 0, dA, dB, dD);
  CK(hipMemcpy(hD, dD, sizeof(hD), hipMemcpyDeviceToHost));
  int bad = 0;
  for (int i = 0; i < 16; ++i)
    for (int j = 0; j < 16; ++j) {
      double s = 0;
      for (int k = 0; k < 4; ++k) s += (double)hA[i * 4 + k] * hB[k * 16 + j];
      if ((double)hD[i * 16 + j] != s && !bad++) std::printf("map mismatch at D[%d][%d]: %g vs %g\n", i, j, hD[i * 16 + j], s);
    }
  std::printf("lane maps: %s\n", bad ? "WRONG" : "ok");
  // random data: which order
  std::mt19937 g(7);
  std::uniform_real_distribution<float> u(-10.f, 10.f);
  long n = 0, m_fwd = 0, m_bwd = 0, m_plain = 0, m_fwd_c0 = 0, maxulp = 0;
  for (int rep = 0; rep < 2000; ++rep) {
    for (float& v : hA) v = u(g);
    for (float& v : hB) v = u(g) * 0.1f;
    CK(hipMemcpy(dA, hA, sizeof(hA), hipMemcpyHostToDevice));
    CK(hipMemcpy(dB, hB, sizeof(hB), hipMemcpyHostToDevice));
    hipLaunchKernelGGL(k_probe, dim3(1), dim3(64), 0, 0, dA, dB, dD);
    CK(hipMemcpy(hD, dD, sizeof(hD), hipMemcpyDeviceToHost));
    for (int i = 0; i < 16; ++i)
      for (int j = 0; j < 16; ++j) {
        float a[4], b[4];
        for (int k = 0; k < 4; ++k) { a[k] = hA[i * 4 + k]; b[k] = hB[k * 16 + j]; }
        float f = 0.f;
        for (int k = 0; k < 4; ++k) f = std::fmaf(a[k], b[k], f);
        float r = 0.f;
        for (int k = 3; k >= 0; --k) r = std::fmaf(a[k], b[k], r);
        float p = ((a[0] * b[0] + a[1] * b[1]) + a[2] * b[2]) + a[3] * b[3];
        float c0 = a[0] * b[0];
        for (int k = 1; k < 4; ++k) c0 = std::fmaf(a[k], b[k], c0);
        const float d = hD[i * 16 + j];
        ++n;
        m_fwd += d == f;
        m_bwd += d == r;
        m_plain += d == p;
        m_fwd_c0 += d == c0;
        double ex = 0;
        for (int k = 0; k < 4; ++k) ex += (double)a[k] * b[k];
        int32_t ia, ib;
        float exf = (float)ex;
        std::memcpy(&ia, &d, 4);
        std::memcpy(&ib, &exf, 4);
        long ul = std::labs((long)ia - (long)ib);
        if (ul > maxulp) maxulp = ul;
      }
  }
  std::printf("random: %ld results; equal to fmaf chain k=0..3: %ld, k=3..0: %ld, plain sum: %ld, "
              "product then fmaf: %ld; max ulps from the exact sum rounded once: %ld\n",
              n, m_fwd, m_bwd, m_plain, m_fwd_c0, maxulp);
  return 0;
}
