// ubench_lat.hip -- single-wave dependent-latency micro-benchmarks on gfx950 (walk design aid):
// cycles per iteration of a dependent chain of (a) f32 adds, (b) f64 adds, (c) v_readlane ->
// SALU add, (d) f64 floor+mul, (e) v_cvt_f64_f32, (f) a readlane-driven uniform loop.
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void k(float* out, long long* cyc, int iters) {
  const int lane = threadIdx.x;
  float f = lane * 1e-3f;
  double d = lane * 1e-3;
  long long t0, t1;
  // (a) f32 add chain
  t0 = clock64();
  for (int i = 0; i < iters; ++i) { f = f + 1.0000001f; f = f + 0.9999999f; f = f + 1e-7f; f = f - 1e-7f; }
  t1 = clock64(); if (lane == 0) cyc[0] = (t1 - t0) / (4 * iters);
  // (b) f64 add chain
  t0 = clock64();
  for (int i = 0; i < iters; ++i) { d = d + 1.0000001; d = d + 0.9999999; d = d + 1e-7; d = d - 1e-7; }
  t1 = clock64(); if (lane == 0) cyc[1] = (t1 - t0) / (4 * iters);
  // (c) readlane -> scalar dependency: s = readlane(v, s & 63); v += 1
  int v = lane, s = 0;
  t0 = clock64();
  for (int i = 0; i < iters; ++i) { s = __builtin_amdgcn_readlane(v, s & 63) + s; s = __builtin_amdgcn_readlane(v, s & 63) + s; }
  t1 = clock64(); if (lane == 0) cyc[2] = (t1 - t0) / (2 * iters);
  // (d) f64 floor + mul chain
  double e = 1.5 + lane;
  t0 = clock64();
  for (int i = 0; i < iters; ++i) { e = floor(e * 1.0000001) + 0.5; e = floor(e * 0.9999999) + 0.5; }
  t1 = clock64(); if (lane == 0) cyc[3] = (t1 - t0) / (2 * iters);
  // (e) cvt f32->f64->f32 chain
  float g = lane;
  t0 = clock64();
  for (int i = 0; i < iters; ++i) { g = (float)((double)g * 1.5); g = (float)((double)g / 1.5); }
  t1 = clock64(); if (lane == 0) cyc[4] = (t1 - t0) / (2 * iters);
  // (f) uniform value through readlane of a VGPR float add: t = readlane(t_vec + p, j)
  float tv = 0.0f, p = lane * 1e-3f;
  t0 = clock64();
  for (int i = 0; i < iters; ++i) {
    const float x = tv + p;
    tv = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(x), i & 63));
  }
  t1 = clock64(); if (lane == 0) cyc[5] = (t1 - t0) / iters;
  // (g) ballot -> ctz -> readlane chain
  int q = lane;
  t0 = clock64();
  for (int i = 0; i < iters; ++i) {
    const unsigned long long m = __builtin_amdgcn_ballot_w64(((q + i) & 7) == 0);
    const int f2 = m ? __builtin_ctzll(m) : 0;
    q = __builtin_amdgcn_readlane(q, f2) + lane;
  }
  t1 = clock64(); if (lane == 0) cyc[6] = (t1 - t0) / iters;
  // (h) int add + DPP wave_shr:1 chain; (i) int add + DPP row_shr:1 chain; (j) v_bfi chain;
  // (k) dependent SALU chain (s_add + s_lshr through asm)
  int wv = lane;
  t0 = clock64();
  for (int i = 0; i < iters; ++i) {
    wv = __builtin_amdgcn_update_dpp(wv, wv + 3, 0x138, 0xF, 0xF, false);
    wv = __builtin_amdgcn_update_dpp(wv, wv + 5, 0x138, 0xF, 0xF, false);
  }
  t1 = clock64(); if (lane == 0) cyc[7] = (t1 - t0) / (2 * iters);
  int rv = lane;
  t0 = clock64();
  for (int i = 0; i < iters; ++i) {
    rv = __builtin_amdgcn_update_dpp(rv, rv + 3, 0x111, 0xF, 0xF, false);
    rv = __builtin_amdgcn_update_dpp(rv, rv + 5, 0x111, 0xF, 0xF, false);
  }
  t1 = clock64(); if (lane == 0) cyc[8] = (t1 - t0) / (2 * iters);
  unsigned bv = lane, mk = 0x0F0F0F0Fu + lane;
  t0 = clock64();
  for (int i = 0; i < iters; ++i) {
    bv = (mk & bv) | (~mk & (bv + 7u));
    bv = (mk & (bv + 3u)) | (~mk & bv);
  }
  t1 = clock64(); if (lane == 0) cyc[9] = (t1 - t0) / (2 * iters);
  int sv = iters;
  t0 = clock64();
  for (int i = 0; i < iters; ++i) {
    asm volatile("s_add_u32 %0, %0, 7\n\ts_lshr_b32 %0, %0, 1\n\ts_add_u32 %0, %0, 3\n\ts_lshr_b32 %0, %0, 1"
                 : "+s"(sv));
  }
  t1 = clock64(); if (lane == 0) cyc[10] = (t1 - t0) / (4 * iters);
  out[lane] = f + (float)d + (float)s + (float)e + g + tv + q + (float)wv + (float)rv + (float)bv + (float)sv;
}

int main() {
  float* o; long long* c;
  hipMalloc(&o, 256); hipMalloc(&c, 128);
  k<<<1, 64>>>(o, c, 1000);
  hipDeviceSynchronize();
  k<<<1, 64>>>(o, c, 10000);
  long long h[11];
  hipMemcpy(h, c, 88, hipMemcpyDeviceToHost);
  const char* names[] = {"f32 add", "f64 add", "readlane->salu", "f64 floor+mul+add (x3)",
                         "cvt f32->f64 mul f64->f32", "readlane(float add) uniform", "ballot->ctz->readlane",
                         "int add + dpp wave_shr:1", "int add + dpp row_shr:1", "bfi-style select",
                         "salu add/lshr"};
  for (int i = 0; i < 11; ++i) printf("%-32s %lld clk\n", names[i], h[i]);
  int clk = 0; hipDeviceGetAttribute(&clk, hipDeviceAttributeClockRate, 0);
  printf("clock rate %d kHz\n", clk);
  return 0;
}
