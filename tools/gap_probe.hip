// gap_probe.hip -- what sets the ~5 us gaps between some back-to-back dependent kernels of an
// extraction round (tools/host_gaps.py: the host is far ahead, so the gaps are the
// device's).  Launches pairs of trivial kernels that differ in one property (workgroup size,
// static LDS, grid size, a device-scope atomic ticket at the end, hipExtLaunchKernelGGL) on one
// stream, each pair 50 times; run under rocprofv3 --kernel-trace and summarise with
// tools/gap_probe.py.
//   hipcc --offload-arch=gfx950 -O2 tools/gap_probe.hip -o tools/gap_probe
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <cstdio>

template <int BS, int LDS_FLOATS, bool TICKET>
__global__ __launch_bounds__(BS) void k_probe(float* out, unsigned* ticket, int tag) {
  __shared__ float s[LDS_FLOATS > 0 ? LDS_FLOATS : 1];
  float v = (float)(threadIdx.x + tag);
  if constexpr (LDS_FLOATS > 0) {
    s[threadIdx.x % LDS_FLOATS] = v;
    __syncthreads();
    v += s[(threadIdx.x + 1) % LDS_FLOATS];
  }
  if (threadIdx.x == 0) out[blockIdx.x] = v;
  if constexpr (TICKET) {
    if (threadIdx.x == 0) {
      const unsigned t = __hip_atomic_fetch_add(ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (t == gridDim.x - 1) *ticket = 0u;
    }
  }
}

#define CK(x)                                                               \
  do {                                                                      \
    hipError_t e_ = (x);                                                    \
    if (e_ != hipSuccess) {                                                 \
      std::printf("%s: %s\n", #x, hipGetErrorString(e_));                  \
      return 1;                                                             \
    }                                                                       \
  } while (0)

int main() {
  float* out;
  unsigned* ticket;
  CK(hipMalloc(&out, 1 << 20));
  CK(hipMalloc(&ticket, 64));
  CK(hipMemset(ticket, 0, 64));
  hipStream_t s;
  CK(hipStreamCreate(&s));
  auto small = k_probe<256, 0, false>;
  auto big = k_probe<1024, 0, false>;
  auto lds = k_probe<256, 16384, false>;     // 64 KB static LDS
  auto lds132 = k_probe<1024, 33792, false>; // 132 KB static LDS, 1024 threads (the scorer's shape)
  auto tick = k_probe<256, 0, true>;
  auto w64 = k_probe<64, 0, false>;
  // pair p: (first, first grid, second, second grid, ext launch of the second); tag = 100 p + k
  struct P { void (*a)(float*, unsigned*, int); int ga; void (*b)(float*, unsigned*, int); int gb; int bsb; int bsa; bool ext; };
  const P pairs[] = {
      {small, 1, small, 1, 256, 256, false},      // 0 baseline
      {small, 1, big, 1, 1024, 256, false},       // 1 -> 1024-thread workgroup
      {small, 1, lds, 1, 256, 256, false},        // 2 -> 64 KB LDS
      {small, 1, lds132, 1, 1024, 256, false},    // 3 -> 132 KB LDS, 1024 threads
      {small, 2048, small, 2048, 256, 256, false},// 4 wide -> wide
      {tick, 512, small, 1, 256, 256, false},     // 5 ticket kernel -> small
      {small, 1, small, 1, 256, 256, true},       // 6 -> ext launch
      {small, 1, w64, 1600, 64, 256, false},      // 7 -> 1600 x 64-thread workgroups
      {lds132, 256, small, 1, 256, 1024, false},  // 8 scorer-shaped -> small
      {big, 611, big, 611, 1024, 1024, false},    // 9 select-shaped -> select-shaped
  };
  for (int p = 0; p < (int)(sizeof(pairs) / sizeof(pairs[0])); ++p) {
    for (int k = 0; k < 50; ++k) {
      const P& q = pairs[p];
      hipLaunchKernelGGL(q.a, dim3(q.ga), dim3(q.bsa), 0, s, out, ticket, 100 * p + k);
      if (q.ext)
        hipExtLaunchKernelGGL(q.b, dim3(q.gb), dim3(q.bsb), 0, s, nullptr, nullptr, 0, out, ticket,
                              100 * p + k);
      else
        hipLaunchKernelGGL(q.b, dim3(q.gb), dim3(q.bsb), 0, s, out, ticket, 100 * p + k);
    }
    CK(hipStreamSynchronize(s));
  }
  CK(hipGetLastError());
  // without a profiler: wall time of 2000 dependent dispatches of one kernel (events around)
  {
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const P variants[] = {pairs[0], pairs[1], pairs[3], pairs[9]};
    const char* names[] = {"256 x 1", "1024 x 1", "1024 x 1, 132 KB LDS", "611 x 1024"};
    for (int v = 0; v < 4; ++v) {
      const P& q = variants[v];
      for (int k = 0; k < 50; ++k)
        hipLaunchKernelGGL(q.b, dim3(q.gb), dim3(q.bsb), 0, s, out, ticket, k);
      CK(hipEventRecord(e0, s));
      for (int k = 0; k < 2000; ++k)
        hipLaunchKernelGGL(q.b, dim3(q.gb), dim3(q.bsb), 0, s, out, ticket, k);
      CK(hipEventRecord(e1, s));
      CK(hipEventSynchronize(e1));
      float ms = 0.f;
      CK(hipEventElapsedTime(&ms, e0, e1));
      std::printf("dispatch cycle %-22s %.2f us per kernel (stream)\n", names[v], 1000.0f * ms / 2000);
      // the same from a captured graph of 200 launches (no host launch cost per kernel)
      hipGraph_t g;
      hipGraphExec_t ge;
      CK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
      for (int k = 0; k < 200; ++k)
        hipLaunchKernelGGL(q.b, dim3(q.gb), dim3(q.bsb), 0, s, out, ticket, k);
      CK(hipStreamEndCapture(s, &g));
      CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
      CK(hipGraphLaunch(ge, s));
      CK(hipEventRecord(e0, s));
      for (int k = 0; k < 10; ++k) CK(hipGraphLaunch(ge, s));
      CK(hipEventRecord(e1, s));
      CK(hipEventSynchronize(e1));
      CK(hipEventElapsedTime(&ms, e0, e1));
      std::printf("dispatch cycle %-22s %.2f us per kernel (graph)\n", names[v], 1000.0f * ms / 2000);
      CK(hipGraphExecDestroy(ge));
      CK(hipGraphDestroy(g));
    }
  }
  std::printf("gap_probe done\n");
  return 0;
}
