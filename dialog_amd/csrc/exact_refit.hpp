// exact_refit.hpp -- the fast refit (DLG_REFIT_FAST) of optimizeModelCoefficients: a least-squares
// plane through the inliers whose value depends only on the inlier SET.
//
// PCL's refit (single-pass float sums in list order, host_math.hpp refit_pcl_float) is
// order-dependent and sequential by definition.  The fast refit instead accumulates the moments
// of the inliers EXACTLY, in integers, so that any visiting order -- list or Morton order, any
// number of workgroups, any number of point-sharded ranks (int64 allreduce) -- gives the same
// bits; the plane is then a deterministic function of those integers, evaluated with IEEE double
// +, -, *, / and sqrt only (no transcendental functions: host and device agree bit for bit), and
// restated independently by the oracle (oracle/pcl_oracle.c orc_refit_exact).
//
// Definition, for the inliers p_i (i < n) of the unrefined plane:
//   e      = the binary exponent with F < 2^e, F = max |coordinate| over the cloud's finite points
//            (frexp; F = 0 -> e = 0); all ranks use the global F
//   q(v)   = trunc(v * 2^(48 - e))  as int64, |q| < 2^48 (the product in double is exact)
//   L_a    = sum q(a_i), P_ab = sum q(a_i) q(b_i)            (a, b in x, y, z; exact integers)
//   C_ab   = n P_ab - L_a L_b  (= n^2 2^(2(48-e)) cov_ab, exact, < 2^160 in magnitude)
//   M_ab   = RN(C_ab) as double (correctly rounded), v = unit eigenvector of the smallest
//            eigenvalue of M by cyclic Jacobi (exactly the rotation sequence of jacobi3 below),
//            oriented so that v . (a, b, c)_unrefined >= 0
//   centre = RN(L_a) / n * 2^(e - 48)
//   coeff  = (float(v), float(-((v_x c_x + v_y c_y) + v_z c_z)))
// n < 4 keeps the unrefined plane (as PCL).  The quantisation step 2^(e - 48) is ~2^-48 of the
// cloud's extent: far below float resolution, so this is the LS plane of the inliers to within
// the rounding of its final float coefficients (tests: within 1e-6 of a float64 LS fit).
//
// Moments travel as kMomDigits int64 "digits" (all sums < 2^63 for n < 2^31):
//   [0] n; [1 + 2a, 2 + 2a] L_a = hi 2^32 + lo  (lo = q & 0xFFFFFFFF, hi = q >> 32);
//   [7 + 3k .. 9 + 3k] P_k (k = xx, xy, xz, yy, yz, zz) = d2 2^64 + d1 2^32 + d0 of each
//   128-bit product (d0, d1 its two low 32-bit halves, d2 its signed high 64 bits).
#pragma once

#include <cmath>
#include <cstdint>
#include <cstring>

// (host-only translation units -- tests/cpp/exact_refit_host.cpp -- build without HIP)
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

constexpr int kMomDigits = 25;
constexpr int kFastBits = 48;

DLG_HD inline double pow2d(int k) {  // 2^k exactly (normal range)
  const uint64_t bits = (uint64_t)(1023 + k) << 52;
  double d;
  std::memcpy(&d, &bits, 8);
  return d;
}

// the quantisation exponent of a cloud from its largest finite |coordinate|
inline int fast_qexp(float fmax) {
  if (!(fmax > 0.0f) || !(fmax < INFINITY)) return 0;
  int e = 0;
  (void)std::frexp((double)fmax, &e);  // fmax = f 2^e, f in [0.5, 1)
  return e;
}

DLG_HD inline int64_t fast_q(float v, double scale) { return (int64_t)((double)v * scale); }

// one inlier's contribution to the digits
DLG_HD inline void mom_add(int64_t* acc, int64_t qx, int64_t qy, int64_t qz) {
  acc[0] += 1;
  const int64_t q[3] = {qx, qy, qz};
#pragma unroll
  for (int a = 0; a < 3; ++a) {
    acc[1 + 2 * a] += q[a] & 0xFFFFFFFFll;
    acc[2 + 2 * a] += q[a] >> 32;
  }
  const int ia[6] = {0, 0, 0, 1, 1, 2}, ib[6] = {0, 1, 2, 1, 2, 2};
#pragma unroll
  for (int k = 0; k < 6; ++k) {
    const int64_t u = q[ia[k]], w = q[ib[k]];
    const uint64_t lo = (uint64_t)u * (uint64_t)w;
#if defined(__HIP_DEVICE_COMPILE__)
    const int64_t hi = __mul64hi(u, w);
#else
    const int64_t hi = (int64_t)(((__int128)u * (__int128)w) >> 64);
#endif
    acc[7 + 3 * k] += (int64_t)(lo & 0xFFFFFFFFull);
    acc[8 + 3 * k] += (int64_t)(lo >> 32);
    acc[9 + 3 * k] += hi;
  }
}

// ---- 192-bit two's-complement integers (6 x 32-bit limbs) ------------------------------------
struct Big {
  uint32_t w[6];
};

DLG_HD inline Big big_i64(int64_t v) {
  Big b;
  const uint64_t u = (uint64_t)v;
  b.w[0] = (uint32_t)u;
  b.w[1] = (uint32_t)(u >> 32);
  const uint32_t s = v < 0 ? 0xFFFFFFFFu : 0u;
  for (int k = 2; k < 6; ++k) b.w[k] = s;
  return b;
}

DLG_HD inline Big big_add(const Big& a, const Big& b) {
  Big r;
  uint64_t c = 0;
  for (int k = 0; k < 6; ++k) {
    c += (uint64_t)a.w[k] + (uint64_t)b.w[k];
    r.w[k] = (uint32_t)c;
    c >>= 32;
  }
  return r;
}

DLG_HD inline Big big_neg(const Big& a) {
  Big r;
  uint64_t c = 1;
  for (int k = 0; k < 6; ++k) {
    c += (uint64_t)(~a.w[k]);
    r.w[k] = (uint32_t)c;
    c >>= 32;
  }
  return r;
}

DLG_HD inline Big big_shl32(const Big& a, int limbs) {
  Big r;
  for (int k = 5; k >= 0; --k) r.w[k] = k >= limbs ? a.w[k - limbs] : 0u;
  return r;
}

// product mod 2^192 (exact when the signed result fits)
DLG_HD inline Big big_mul(const Big& a, const Big& b) {
  uint64_t acc[7] = {0, 0, 0, 0, 0, 0, 0};
  for (int i = 0; i < 6; ++i) {
    uint64_t carry = 0;
    for (int j = 0; i + j < 6; ++j) {
      const uint64_t t = (uint64_t)a.w[i] * (uint64_t)b.w[j] + (acc[i + j] & 0xFFFFFFFFull) + carry;
      acc[i + j] = t & 0xFFFFFFFFull;
      carry = t >> 32;
    }
  }
  Big r;
  for (int k = 0; k < 6; ++k) r.w[k] = (uint32_t)acc[k];
  return r;
}

// correctly rounded (to nearest, ties to even) conversion to double
DLG_HD inline double big_to_double(const Big& a) {
  const bool neg = (a.w[5] >> 31) != 0;
  const Big m = neg ? big_neg(a) : a;
  int top = -1;
  for (int k = 5; k >= 0; --k)
    if (m.w[k]) {
      top = k;
      break;
    }
  if (top < 0) return 0.0;
  int bl = 32;  // bit length of the top limb
  while (!((m.w[top] >> (bl - 1)) & 1u)) --bl;
  const int L = 32 * top + bl;  // bit length of the magnitude
  double r;
  if (L <= 53) {
    uint64_t v = 0;
    for (int k = top; k >= 0; --k) v = (v << 32) | m.w[k];
    r = (double)v;  // exact
  } else {
    // the 53 leading bits, the round bit and the sticky bits below it
    auto bit = [&](int i) -> uint32_t { return (m.w[i >> 5] >> (i & 31)) & 1u; };
    uint64_t mant = 0;
    for (int i = L - 1; i >= L - 53; --i) mant = (mant << 1) | bit(i);
    const uint32_t rb = bit(L - 54);
    bool sticky = false;
    for (int i = L - 55; i >= 0 && !sticky; --i) sticky = bit(i) != 0;
    if (rb && (sticky || (mant & 1ull))) ++mant;  // (mant may become 2^53: still exact)
    r = (double)mant * pow2d(L - 53);
  }
  return neg ? -r : r;
}

// the digit sums of one moment as a Big
DLG_HD inline Big big_lin(const int64_t* d) {  // hi 2^32 + lo
  return big_add(big_shl32(big_i64(d[1]), 1), big_i64(d[0]));
}
DLG_HD inline Big big_prod(const int64_t* d) {  // d2 2^64 + d1 2^32 + d0
  return big_add(big_add(big_shl32(big_i64(d[2]), 2), big_shl32(big_i64(d[1]), 1)), big_i64(d[0]));
}

// cyclic Jacobi on a symmetric 3x3 (row-major); eigenvector columns in V (row-major)
DLG_HD inline void jacobi3(double A[9], double V[9]) {
  for (int k = 0; k < 9; ++k) V[k] = (k % 4 == 0) ? 1.0 : 0.0;
  const int P[3] = {0, 0, 1}, Q[3] = {1, 2, 2};
  for (int sweep = 0; sweep < 16; ++sweep) {
    const double off = (A[1] * A[1] + A[2] * A[2]) + A[5] * A[5];
    if (off == 0.0) break;
    for (int r = 0; r < 3; ++r) {
      const int p = P[r], q = Q[r];
      const double apq = A[3 * p + q];
      if (apq == 0.0) continue;
      const double app = A[3 * p + p], aqq = A[3 * q + q];
      const double theta = (aqq - app) / (2.0 * apq);
      double t;
      if (theta > 1e150 || theta < -1e150) {
        t = 0.5 / theta;
      } else {
        t = 1.0 / ((theta < 0.0 ? -theta : theta) + sqrt(theta * theta + 1.0));
        if (theta < 0.0) t = -t;
      }
      const double c = 1.0 / sqrt(t * t + 1.0), s = t * c;
      A[3 * p + p] = app - t * apq;
      A[3 * q + q] = aqq + t * apq;
      A[3 * p + q] = 0.0;
      A[3 * q + p] = 0.0;
      const int o = 3 - p - q;  // the third index
      const double aop = A[3 * o + p], aoq = A[3 * o + q];
      const double nop = c * aop - s * aoq, noq = s * aop + c * aoq;
      A[3 * o + p] = nop; A[3 * p + o] = nop;
      A[3 * o + q] = noq; A[3 * q + o] = noq;
      for (int i = 0; i < 3; ++i) {
        const double vip = V[3 * i + p], viq = V[3 * i + q];
        V[3 * i + p] = c * vip - s * viq;
        V[3 * i + q] = s * vip + c * viq;
      }
    }
  }
}

// the fast refit from the summed digits (see the definition at the top)
DLG_HD inline void refit_exact(const int64_t* dig, int qexp, const float cin[4], float cout[4]) {
  const int64_t n = dig[0];
  if (n < 4) {
    for (int k = 0; k < 4; ++k) cout[k] = cin[k];
    return;
  }
  Big L[3], Pm[6];
  for (int a = 0; a < 3; ++a) L[a] = big_lin(dig + 1 + 2 * a);
  for (int k = 0; k < 6; ++k) Pm[k] = big_prod(dig + 7 + 3 * k);
  const Big bn = big_i64(n);
  const int ia[6] = {0, 0, 0, 1, 1, 2}, ib[6] = {0, 1, 2, 1, 2, 2};
  double m6[6];
  for (int k = 0; k < 6; ++k)
    m6[k] = big_to_double(big_add(big_mul(bn, Pm[k]), big_neg(big_mul(L[ia[k]], L[ib[k]]))));
  double A[9] = {m6[0], m6[1], m6[2], m6[1], m6[3], m6[4], m6[2], m6[4], m6[5]};
  double V[9];
  jacobi3(A, V);
  int k = 0;  // smallest eigenvalue (ties: lowest index)
  if (A[4] < A[0]) k = 1;
  if (A[8] < A[4 * k]) k = 2;
  double v0 = V[k], v1 = V[3 + k], v2 = V[6 + k];
  const double nv = sqrt((v0 * v0 + v1 * v1) + v2 * v2);
  v0 = v0 / nv; v1 = v1 / nv; v2 = v2 / nv;
  if ((v0 * (double)cin[0] + v1 * (double)cin[1]) + v2 * (double)cin[2] < 0.0) {
    v0 = -v0; v1 = -v1; v2 = -v2;
  }
  const double nd = (double)n, back = pow2d(qexp - kFastBits);
  const double c0 = big_to_double(L[0]) / nd * back;
  const double c1 = big_to_double(L[1]) / nd * back;
  const double c2 = big_to_double(L[2]) / nd * back;
  const double d = -((v0 * c0 + v1 * c1) + v2 * c2);
  cout[0] = (float)v0; cout[1] = (float)v1; cout[2] = (float)v2; cout[3] = (float)d;
}

}  // namespace dlg
