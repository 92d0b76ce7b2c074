// ubench_valu.hip -- issue cost of the instruction classes the scoring kernel uses (gfx950).
// Every body is a fully unrolled block of independent instructions on 16 accumulators whose
// operands are all VGPRs loaded at run time (nothing for the compiler to hoist).  Prints the
// device time per wave-instruction per SIMD and the shader clock measured in-kernel
// (s_memtime / s_memrealtime, 100 MHz) so cycles per instruction are exact.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s\n", hipGetErrorString(e)); exit(1); } } while (0)

constexpr int ITER = 2048;
constexpr int NA = 16;
typedef float v2f __attribute__((ext_vector_type(2)));

__device__ __forceinline__ void stamp(unsigned long long* clk, int which) {
  if (threadIdx.x == 0 && blockIdx.x == 0) {
    clk[2 * which] = __builtin_amdgcn_s_memtime();
    clk[2 * which + 1] = __builtin_amdgcn_s_memrealtime();
  }
}

template <int OP>
__global__ __launch_bounds__(256) void k_body(const float* in, float* out, int* iout,
                                              unsigned long long* clk) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  float a[NA], b = in[t & 255], c = in[(t + 7) & 255], thr = in[(t + 3) & 255];
#pragma unroll
  for (int k = 0; k < NA; ++k) a[k] = in[(t + k) & 255];
  int cnt = 0;
  stamp(clk, 0);
  for (int i = 0; i < ITER; ++i) {
#pragma unroll
    for (int k = 0; k < NA; ++k) {
      if (OP == 0) a[k] = __builtin_fmaf(a[k], b, c);            // v_fma_f32
      if (OP == 1) a[k] = a[k] * b;                               // v_mul_f32
      if (OP == 2) a[k] = a[k] + b;                               // v_add_f32
      if (OP == 3) {                                              // v_add + v_cmp(sgpr) + s_bcnt1 + s_add
        a[k] = a[k] + b;
        cnt += __popcll(__builtin_amdgcn_ballot_w64(fabsf(a[k]) < thr));
      }
      if (OP == 4) {                                              // v_add + v_cmp(vcc) + v_addc
        a[k] = a[k] + b;
        cnt += fabsf(a[k]) < thr ? 1 : 0;
      }
    }
    if (OP >= 5) {  // packed f32 on register pairs (a[2i], a[2i+1])
#pragma unroll
      for (int k = 0; k < NA; k += 2) {
        v2f x = {a[k], a[k + 1]};
        v2f y = {b, c};
        if (OP == 5) asm volatile("v_pk_mul_f32 %0, %1, %2" : "=v"(x) : "v"(x), "v"(y));
        if (OP == 6) asm volatile("v_pk_add_f32 %0, %1, %2" : "=v"(x) : "v"(x), "v"(y));
        if (OP == 7) asm volatile("v_pk_fma_f32 %0, %1, %2, %3" : "=v"(x) : "v"(x), "v"(y), "v"(y));
        a[k] = x.x;
        a[k + 1] = x.y;
      }
    }
    asm volatile("" ::: "memory");
  }
  stamp(clk, 1);
  float s = 0;
#pragma unroll
  for (int k = 0; k < NA; ++k) s += a[k];
  out[t] = s;
  iout[t] = cnt;
}

template <typename F>
float time_kernel(F launch, int reps) {
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a)); CHECK(hipEventCreate(&b));
  launch();
  CHECK(hipDeviceSynchronize());
  CHECK(hipEventRecord(a));
  for (int r = 0; r < reps; ++r) launch();
  CHECK(hipEventRecord(b));
  CHECK(hipEventSynchronize(b));
  float ms; CHECK(hipEventElapsedTime(&ms, a, b));
  return ms / reps;
}

int main(int argc, char** argv) {
  hipDeviceProp_t p; CHECK(hipGetDeviceProperties(&p, 0));
  const int cus = p.multiProcessorCount;
  float* in; float* fo; int* io; unsigned long long* clk;
  CHECK(hipMalloc(&in, 256 * 4));
  float h[256]; for (int i = 0; i < 256; ++i) h[i] = 1.0f + i * 1e-6f;
  CHECK(hipMemcpy(in, h, sizeof(h), hipMemcpyHostToDevice));
  const int maxb = cus * 8;
  CHECK(hipMalloc(&fo, (size_t)maxb * 256 * 4)); CHECK(hipMalloc(&io, (size_t)maxb * 256 * 4));
  CHECK(hipMalloc(&clk, 64));
  const char* names[] = {"fma", "mul", "add", "add+cmp->sgpr+bcnt", "add+cmp->vcc+addc",
                         "pk_mul (2 lanes-ops)", "pk_add (2 lane-ops)", "pk_fma (2 lane-ops)"};
  // VALU instructions per (iteration, accumulator), from the gfx950 asm of each body
  const double valu[] = {1, 1, 1, 2, 3, 0.5, 0.5, 0.5};
  for (int wps = 1; wps <= 8; wps *= 2) {
    const int blocks = cus * wps;  // 256-thread block = 4 waves = 1 wave per SIMD
    printf("== %d wave(s)/SIMD\n", wps);
    for (int op = 0; op < 8; ++op) {
      auto L = [&] {
        switch (op) {
          case 0: hipLaunchKernelGGL(k_body<0>, blocks, 256, 0, 0, in, fo, io, clk); break;
          case 1: hipLaunchKernelGGL(k_body<1>, blocks, 256, 0, 0, in, fo, io, clk); break;
          case 2: hipLaunchKernelGGL(k_body<2>, blocks, 256, 0, 0, in, fo, io, clk); break;
          case 3: hipLaunchKernelGGL(k_body<3>, blocks, 256, 0, 0, in, fo, io, clk); break;
          case 4: hipLaunchKernelGGL(k_body<4>, blocks, 256, 0, 0, in, fo, io, clk); break;
          case 5: hipLaunchKernelGGL(k_body<5>, blocks, 256, 0, 0, in, fo, io, clk); break;
          case 6: hipLaunchKernelGGL(k_body<6>, blocks, 256, 0, 0, in, fo, io, clk); break;
          case 7: hipLaunchKernelGGL(k_body<7>, blocks, 256, 0, 0, in, fo, io, clk); break;
        }
      };
      float ms = time_kernel(L, 5);
      unsigned long long c[4];
      CHECK(hipMemcpy(c, clk, 32, hipMemcpyDeviceToHost));
      double ghz = (double)(c[2] - c[0]) / ((double)(c[3] - c[1]) / 100e6) / 1e9;
      double instr = (double)wps * ITER * NA * valu[op];  // VALU wave-instructions per SIMD
      double cyc = ms * 1e-3 * ghz * 1e9 / instr;
      printf("  %-22s %7.3f ms  clock %.2f GHz  %5.2f cycles per VALU wave-instr\n", names[op], ms,
             ghz, cyc);
    }
  }
  return 0;
}
