// host_math.hpp -- host-side PCL-1.8 arithmetic of the RANSAC plane path (product code).
//
// Used by the driver for the parts that are sequential by definition in PCL:
//   * Boost mt19937 + uniform_int<>(0, INT_MAX)   (SampleConsensusModel::rnd, seed 12345u)
//   * RandomSampleConsensus::computeModel's best/k bookkeeping
//   * optimizeModelCoefficients' refit: PCL float single-pass sums (parity mode) or double
//     moments from the device (fast mode), then pcl::eigen33
// Op order follows PCL/Eigen as compiled by MSVC x64 (SSE, no FMA): this file must be built with
// -ffp-contract=off.  [PCL-1.8 ext] = third-party source, not vendored in the reference.
#pragma once

#include <cfloat>
#include <cmath>
#include <cstdint>
#include <limits>
#include <utility>

// (host-only builds -- the sanitizer harness tests/cpp/sac_control_san.cpp -- compile without
// HIP: g++ -fsanitize=address,undefined)
#if defined(__HIP__) || defined(__HIPCC__)
#include <hip/hip_runtime.h>
#ifndef DLG_HD
#define DLG_HD __host__ __device__
#endif
#else
#ifndef DLG_HD
#define DLG_HD
#endif
#endif

namespace dlg {

template <typename S>
DLG_HD inline S eps_of();
template <>
DLG_HD inline float eps_of<float>() { return FLT_EPSILON; }
template <>
DLG_HD inline double eps_of<double>() { return DBL_EPSILON; }
template <typename S>
DLG_HD inline S min_of();
template <>
DLG_HD inline float min_of<float>() { return FLT_MIN; }
template <>
DLG_HD inline double min_of<double>() { return DBL_MIN; }
template <typename S>
DLG_HD inline void swap_(S& a, S& b) { S t = a; a = b; b = t; }
// PCL's float eigen33 calls std::sqrt / atan2 / cos / sin on floats.  sqrtf is correctly rounded
// everywhere; the float transcendental functions are platform-specific (MSVC's CRT for the
// reference -- unknowable here), so they are taken as the correctly rounded float values,
// computed as the double function rounded to float: host and device then agree (except in the
// ~2^-29-probable case of a double result within an ulp of a float rounding boundary), and the
// oracle (orc_eigen33) and the numpy twin evaluate them the same way.
DLG_HD inline float m_sqrt(float x) { return sqrtf(x); }
DLG_HD inline double m_sqrt(double x) { return sqrt(x); }
DLG_HD inline float m_fabs(float x) { return fabsf(x); }
DLG_HD inline double m_fabs(double x) { return fabs(x); }
DLG_HD inline float m_atan2(float y, float x) { return (float)atan2((double)y, (double)x); }
DLG_HD inline double m_atan2(double y, double x) { return atan2(y, x); }
DLG_HD inline float m_cos(float x) { return (float)cos((double)x); }
DLG_HD inline double m_cos(double x) { return cos(x); }
DLG_HD inline float m_sin(float x) { return (float)sin((double)x); }
DLG_HD inline double m_sin(double x) { return sin(x); }

class Mt19937 {
 public:
  explicit Mt19937(uint32_t seed = 5489u) { seed_(seed); }
  void seed_(uint32_t s) {
    mt_[0] = s;
    for (int i = 1; i < 624; ++i) mt_[i] = 1812433253u * (mt_[i - 1] ^ (mt_[i - 1] >> 30)) + (uint32_t)i;
    idx_ = 624;
  }
  uint32_t operator()() {
    if (idx_ >= 624) twist();
    uint32_t y = mt_[idx_++];
    y ^= y >> 11;
    y ^= (y << 7) & 0x9d2c5680u;
    y ^= (y << 15) & 0xefc60000u;
    y ^= y >> 18;
    return y;
  }
  // boost::uniform_int<>(0, INT_MAX) over mt19937: bucket_size 2, never rejects [PCL-1.8 ext]
  int rnd() { return (int)((*this)() >> 1); }

 private:
  void twist() {
    for (int i = 0; i < 624; ++i) {
      uint32_t y = (mt_[i] & 0x80000000u) | (mt_[(i + 1) % 624] & 0x7fffffffu);
      mt_[i] = mt_[(i + 397) % 624] ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
    }
    idx_ = 0;
  }
  uint32_t mt_[624];
  int idx_;
};

// smallest float >= thr, so that (double)|d| < thr  <=>  |d| < thr_ceil(thr) for float d
inline float thr_ceil(double thr) {
  float f = (float)thr;
  if ((double)f < thr) f = std::nextafter(f, INFINITY);
  return f;
}

// ---- pcl::computeRoots2 / computeRoots / eigen33 (common/impl/eigen.hpp) [PCL-1.8 ext] ----------
template <typename S>
DLG_HD inline void compute_roots2(S b, S c, S roots[3]) {
  roots[0] = S(0);
  S d = S((double)(b * b) - 4.0 * (double)c);  // Scalar(b * b - 4.0 * c): b*b in S, rest in double
  if (d < S(0)) d = S(0);
  S sd = m_sqrt(d);
  roots[2] = S(0.5f) * (b + sd);
  roots[1] = S(0.5f) * (b - sd);
}

// the transcendental functions of eigen33 (host_math's m_atan2 / m_cos / m_sin by default; the
// device refit of fsum.hpp substitutes a variant that flags results it cannot round for certain)
struct PlainTx {
  template <typename S>
  DLG_HD S atan2(S y, S x) const { return m_atan2(y, x); }
  template <typename S>
  DLG_HD S cos(S x) const { return m_cos(x); }
  template <typename S>
  DLG_HD S sin(S x) const { return m_sin(x); }
};

template <typename S, typename TX = PlainTx>
DLG_HD inline void compute_roots(const S m[9], S roots[3], const TX& tx = TX()) {
  auto M = [&](int r, int c) { return m[r * 3 + c]; };
  S c0 = M(0, 0) * M(1, 1) * M(2, 2) + S(2) * M(0, 1) * M(0, 2) * M(1, 2) -
         M(0, 0) * M(1, 2) * M(1, 2) - M(1, 1) * M(0, 2) * M(0, 2) - M(2, 2) * M(0, 1) * M(0, 1);
  S c1 = M(0, 0) * M(1, 1) - M(0, 1) * M(0, 1) + M(0, 0) * M(2, 2) - M(0, 2) * M(0, 2) +
         M(1, 1) * M(2, 2) - M(1, 2) * M(1, 2);
  S c2 = M(0, 0) + M(1, 1) + M(2, 2);
  const S eps = eps_of<S>();
  if (m_fabs(c0) < eps) {
    compute_roots2(c2, c1, roots);
    return;
  }
  const S s_inv3 = S(1.0 / 3.0);
  const S s_sqrt3 = m_sqrt(S(3.0));
  S c2_over_3 = c2 * s_inv3;
  S a_over_3 = (c1 - c2 * c2_over_3) * s_inv3;
  if (a_over_3 > S(0)) a_over_3 = S(0);
  S half_b = S(0.5) * (c0 + c2_over_3 * (S(2) * c2_over_3 * c2_over_3 - c1));
  S q = half_b * half_b + a_over_3 * a_over_3 * a_over_3;
  if (q > S(0)) q = S(0);
  S rho = m_sqrt(-a_over_3);
  S theta = tx.atan2(m_sqrt(-q), half_b) * s_inv3;
  S ct = tx.cos(theta), st = tx.sin(theta);
  roots[0] = c2_over_3 + S(2) * rho * ct;
  roots[1] = c2_over_3 - rho * (ct + s_sqrt3 * st);
  roots[2] = c2_over_3 - rho * (ct - s_sqrt3 * st);
  if (roots[0] >= roots[1]) swap_(roots[0], roots[1]);
  if (roots[1] >= roots[2]) {
    swap_(roots[1], roots[2]);
    if (roots[0] >= roots[1]) swap_(roots[0], roots[1]);
  }
  if (roots[0] <= S(0)) compute_roots2(c2, c1, roots);
}

template <typename S, typename TX>
DLG_HD inline void eigen33_tx(const S mat[9], S* eval, S evec[3], const TX& tx) {
  S scale = S(0);
  for (int k = 0; k < 9; ++k) scale = m_fabs(mat[k]) > scale ? m_fabs(mat[k]) : scale;
  if (scale <= min_of<S>()) scale = S(1);
  S m[9];
  for (int k = 0; k < 9; ++k) m[k] = mat[k] / scale;
  S roots[3];
  compute_roots(m, roots, tx);
  *eval = roots[0] * scale;
  m[0] -= roots[0]; m[4] -= roots[0]; m[8] -= roots[0];
  auto cross = [](const S* a, const S* b, S* o) {
    o[0] = a[1] * b[2] - a[2] * b[1];
    o[1] = a[2] * b[0] - a[0] * b[2];
    o[2] = a[0] * b[1] - a[1] * b[0];
  };
  // Vector3 squaredNorm: Eigen's non-vectorised unroller -> x^2 + (y^2 + z^2)
  auto sqn = [](const S* v) { return v[0] * v[0] + (v[1] * v[1] + v[2] * v[2]); };
  S v1[3], v2[3], v3[3];
  cross(m + 0, m + 3, v1);
  cross(m + 0, m + 6, v2);
  cross(m + 3, m + 6, v3);
  S l1 = sqn(v1), l2 = sqn(v2), l3 = sqn(v3);
  const S* v;
  S l;
  if (l1 >= l2 && l1 >= l3) { v = v1; l = l1; }
  else if (l2 >= l1 && l2 >= l3) { v = v2; l = l2; }
  else { v = v3; l = l3; }
  S s = m_sqrt(l);
  evec[0] = v[0] / s; evec[1] = v[1] / s; evec[2] = v[2] / s;
}

template <typename S>
DLG_HD inline void eigen33(const S mat[9], S* eval, S evec[3]) {
  eigen33_tx(mat, eval, evec, PlainTx());
}

// optimizeModelCoefficients, parity mode: computeMeanAndCovarianceMatrix (float, dense branch,
// single pass in list order) + eigen33 + coeff[3] = -1 * coeff.dot(centroid) (SSE predux order).
// xyz: inliers in list order, AoS 3 floats.
inline void refit_pcl_float(const float* xyz, int64_t n, const float cin[4], float cout[4]) {
  if (n < 4) {
    for (int k = 0; k < 4; ++k) cout[k] = cin[k];
    return;
  }
  float a[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
  for (int64_t i = 0; i < n; ++i) {
    const float x = xyz[3 * i], y = xyz[3 * i + 1], z = xyz[3 * i + 2];
    a[0] += x * x; a[1] += x * y; a[2] += x * z;
    a[3] += y * y; a[4] += y * z; a[5] += z * z;
    a[6] += x;     a[7] += y;     a[8] += z;
  }
  const float cnt = (float)(size_t)n;
  for (int k = 0; k < 9; ++k) a[k] = a[k] / cnt;
  float cov[9];
  cov[0] = a[0] - a[6] * a[6];
  cov[1] = a[1] - a[6] * a[7];
  cov[2] = a[2] - a[6] * a[8];
  cov[4] = a[3] - a[7] * a[7];
  cov[5] = a[4] - a[7] * a[8];
  cov[8] = a[5] - a[8] * a[8];
  cov[3] = cov[1]; cov[6] = cov[2]; cov[7] = cov[5];
  float ev, v[3];
  eigen33(cov, &ev, v);
  const float c3 = 0.0f, cw = 1.0f;
  float dot = (v[0] * a[6] + v[2] * a[8]) + (v[1] * a[7] + c3 * cw);
  cout[0] = v[0]; cout[1] = v[1]; cout[2] = v[2]; cout[3] = -1.0f * dot;
}

// fast mode: moments m[10] = {n, sx, sy, sz, sxx, sxy, sxz, syy, syz, szz} of (p - shift), double.
DLG_HD inline void refit_from_moments(const double m[10], const double shift[3], const float cin[4],
                                      float cout[4]) {
  const double n = m[0];
  if (n < 4.0) {
    for (int k = 0; k < 4; ++k) cout[k] = cin[k];
    return;
  }
  const double mx = m[1] / n, my = m[2] / n, mz = m[3] / n;
  double cov[9];
  cov[0] = m[4] / n - mx * mx;
  cov[1] = m[5] / n - mx * my;
  cov[2] = m[6] / n - mx * mz;
  cov[4] = m[7] / n - my * my;
  cov[5] = m[8] / n - my * mz;
  cov[8] = m[9] / n - mz * mz;
  cov[3] = cov[1]; cov[6] = cov[2]; cov[7] = cov[5];
  double ev, v[3];
  eigen33(cov, &ev, v);
  const double cx = shift[0] + mx, cy = shift[1] + my, cz = shift[2] + mz;
  const double d = -(v[0] * cx + v[1] * cy + v[2] * cz);
  cout[0] = (float)v[0]; cout[1] = (float)v[1]; cout[2] = (float)v[2]; cout[3] = (float)d;
}

}  // namespace dlg
