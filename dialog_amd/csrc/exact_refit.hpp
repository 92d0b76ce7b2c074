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
//   q(v)   = trunc(v * 2^(48 - e)), an integer |q| < 2^48 (the product in double is exact)
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
// Accumulation (all exact): per point, with Q = q as a double (an integer < 2^48) split as
// Q = hi 2^24 + lo (hi = floor(Q 2^-24), 0 <= lo < 2^24), q_a q_b = A 2^48 + B 2^24 + C with
// A = hi_a hi_b, B = hi_a lo_b + lo_a hi_b, C = lo_a lo_b -- each < 2^49 in magnitude, summed with
// double FMAs into a per-lane MomAcc (exact while every sum stays < 2^53: at most kMomFlush points
// between flushes).  A flush splits each sum X = X0 + X1 2^24 (0 <= X0 < 2^24, |X1| < 2^29) and
// adds the pieces of equal weight into the int64 digits (each flush adds < 2^30 per digit: all
// sums < 2^63 for n < 2^31):
//   [0] n; [1 + 2a, 2 + 2a] L_a = D0 + D1 2^24;
//   [7 + 4k .. 10 + 4k] P_k (k = xx, xy, xz, yy, yz, zz) = w0 + w24 2^24 + w48 2^48 + w72 2^72
//   (w0 = C0, w24 = C1 + B0, w48 = B1 + A0, w72 = A1).
// The digits are not canonical (they depend on how points were grouped into flushes); the
// integers they stand for are, and only those enter the refit.
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

constexpr int kMomDigits = 31;
constexpr int kFastBits = 48;
constexpr int kMomFlush = 16;  // points per MomAcc between flushes (B: 2 x 16 x 2^48 = 2^53)

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

// q(v) as a double (exact integer)
DLG_HD inline double fast_q(float v, double scale) { return trunc((double)v * scale); }

// per-lane partial sums between flushes (exact integers < 2^53 held in doubles)
struct MomAcc {
  double n, L[3], A[6], B[6], C[6];
};

DLG_HD inline void mom_zero(MomAcc& m) {
  m.n = 0.0;
#pragma unroll
  for (int a = 0; a < 3; ++a) m.L[a] = 0.0;
#pragma unroll
  for (int k = 0; k < 6; ++k) m.A[k] = m.B[k] = m.C[k] = 0.0;
}

// one inlier (Q = fast_q of its coordinates)
DLG_HD inline void mom_point(MomAcc& m, double qx, double qy, double qz) {
  const double q[3] = {qx, qy, qz};
  double hi[3], lo[3];
#pragma unroll
  for (int a = 0; a < 3; ++a) {
    hi[a] = floor(q[a] * 0x1p-24);
    lo[a] = fma(-hi[a], 0x1p24, q[a]);  // exact: 0 <= lo < 2^24
  }
  m.n += 1.0;
#pragma unroll
  for (int a = 0; a < 3; ++a) m.L[a] += q[a];
#pragma unroll
  for (int k = 0; k < 6; ++k) {
    const int a = k < 3 ? 0 : (k < 5 ? 1 : 2);
    const int b = k < 3 ? k : (k < 5 ? k - 2 : 2);
    m.A[k] = fma(hi[a], hi[b], m.A[k]);
    m.B[k] = fma(lo[a], hi[b], fma(hi[a], lo[b], m.B[k]));
    m.C[k] = fma(lo[a], lo[b], m.C[k]);
  }
}

// X = X0 + X1 2^24 with 0 <= X0 < 2^24 (X an integer, |X| < 2^53)
DLG_HD inline void split24(double X, int64_t& x0, int64_t& x1) {
  const double h = floor(X * 0x1p-24);
  x1 = (int64_t)(int32_t)h;
  x0 = (int64_t)(int32_t)fma(-h, 0x1p24, X);
}

// the partial sums into the digits; m is zeroed
DLG_HD inline void mom_flush(int64_t* dig, MomAcc& m) {
  dig[0] += (int64_t)(int32_t)m.n;
  int64_t x0, x1;
#pragma unroll
  for (int a = 0; a < 3; ++a) {
    split24(m.L[a], x0, x1);
    dig[1 + 2 * a] += x0;
    dig[2 + 2 * a] += x1;
  }
#pragma unroll
  for (int k = 0; k < 6; ++k) {
    int64_t c0, c1, b0, b1, a0, a1;
    split24(m.C[k], c0, c1);
    split24(m.B[k], b0, b1);
    split24(m.A[k], a0, a1);
    dig[7 + 4 * k] += c0;
    dig[8 + 4 * k] += c1 + b0;
    dig[9 + 4 * k] += b1 + a0;
    dig[10 + 4 * k] += a1;
  }
  mom_zero(m);
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

DLG_HD inline int clz32(uint32_t v) {  // v != 0
#if defined(__HIP_DEVICE_COMPILE__)
  return __clz((int)v);
#else
  return __builtin_clz(v);
#endif
}

// correctly rounded (to nearest, ties to even) conversion to double: the 64 bits below the
// leading one (53 mantissa bits, the round bit, 10 sticky bits) come from the top three limbs,
// the remaining sticky bits from an OR of the limbs below them -- a fixed handful of integer ops
// (one thread of the device refit runs this for each moment)
DLG_HD inline double big_to_double(const Big& a) {
  const bool neg = (a.w[5] >> 31) != 0;
  const Big m = neg ? big_neg(a) : a;
  // (constant limb indices throughout: no dynamically indexed array on the device)
  int top = -1;
#pragma unroll
  for (int k = 0; k < 6; ++k)
    if (m.w[k]) top = k;
  if (top < 0) return 0.0;
  uint32_t w0 = 0u, l1 = 0u, l2 = 0u;  // the top limb and the two below it
  bool sticky = false;                 // any bit in the limbs below those three
#pragma unroll
  for (int k = 0; k < 6; ++k) {
    if (k == top) {
      w0 = m.w[k];
      l1 = k >= 1 ? m.w[k >= 1 ? k - 1 : 0] : 0u;
      l2 = k >= 2 ? m.w[k >= 2 ? k - 2 : 0] : 0u;
    }
    if (k < top - 2 && m.w[k]) sticky = true;
  }
  const int bl = 32 - clz32(w0);  // bit length of the top limb
  const int L = 32 * top + bl;    // bit length of the magnitude
  double r;
  if (L <= 53) {
    r = (double)(((uint64_t)(top >= 1 ? m.w[1] : 0u) << 32) | m.w[0]);  // exact (top <= 1)
  } else {
    // t = the 64 bits [L - 64, L) of m, left-aligned (bits below 0 read as zero)
    const int sh = 32 - bl;  // left shift that aligns the leading one at bit 95 of (w0,l1,l2)
    const uint64_t hi64 = ((uint64_t)w0 << 32) | l1;
    const uint64_t t = sh == 0 ? hi64 : (hi64 << sh) | (uint64_t)(l2 >> (32 - sh));
    sticky = sticky || (sh == 0 ? l2 : (uint32_t)(l2 << sh)) != 0u;
    uint64_t mant = t >> 11;                      // the 53 leading bits
    const uint32_t rb = (uint32_t)(t >> 10) & 1u;  // the round bit
    sticky = sticky || (t & 0x3FFull) != 0ull;
    if (rb && (sticky || (mant & 1ull))) ++mant;  // (mant may become 2^53: still exact)
    r = (double)mant * pow2d(L - 53);
  }
  return neg ? -r : r;
}

// a << s (0 <= s < 192), mod 2^192
DLG_HD inline Big big_shl(const Big& a, int s) {
  const int L = s >> 5, b = s & 31;
  Big r;
  for (int k = 5; k >= 0; --k) {
    const uint32_t hi = k - L >= 0 ? a.w[k - L] : 0u;
    const uint32_t lo = k - L - 1 >= 0 ? a.w[k - L - 1] : 0u;
    r.w[k] = b == 0 ? hi : (hi << b) | (lo >> (32 - b));
  }
  return r;
}

// the digit sums of one moment as a Big
DLG_HD inline Big big_lin(const int64_t* d) {  // D0 + D1 2^24
  return big_add(big_i64(d[0]), big_shl(big_i64(d[1]), 24));
}
DLG_HD inline Big big_prod(const int64_t* d) {  // w0 + w24 2^24 + w48 2^48 + w72 2^72
  return big_add(big_add(big_i64(d[0]), big_shl(big_i64(d[1]), 24)),
                 big_add(big_shl(big_i64(d[2]), 48), big_shl(big_i64(d[3]), 72)));
}

// one Jacobi rotation annihilating A[p][q] (compile-time indices: everything stays in registers)
template <int p, int q>
DLG_HD inline void jacobi_rot(double A[9], double V[9]) {
  const double apq = A[3 * p + q];
  if (apq == 0.0) return;
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
  constexpr int o = 3 - p - q;  // the third index
  const double aop = A[3 * o + p], aoq = A[3 * o + q];
  const double nop = c * aop - s * aoq, noq = s * aop + c * aoq;
  A[3 * o + p] = nop; A[3 * p + o] = nop;
  A[3 * o + q] = noq; A[3 * q + o] = noq;
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    const double vip = V[3 * i + p], viq = V[3 * i + q];
    V[3 * i + p] = c * vip - s * viq;
    V[3 * i + q] = s * vip + c * viq;
  }
}

// cyclic Jacobi on a symmetric 3x3 (row-major); eigenvector columns in V (row-major): sweeps of
// the rotations (0,1), (0,2), (1,2) until the off-diagonal is exactly zero (at most 16)
DLG_HD inline void jacobi3(double A[9], double V[9]) {
#pragma unroll
  for (int k = 0; k < 9; ++k) V[k] = (k % 4 == 0) ? 1.0 : 0.0;
  for (int sweep = 0; sweep < 16; ++sweep) {
    const double off = (A[1] * A[1] + A[2] * A[2]) + A[5] * A[5];
    if (off == 0.0) break;
    jacobi_rot<0, 1>(A, V);
    jacobi_rot<0, 2>(A, V);
    jacobi_rot<1, 2>(A, V);
  }
}

// the nine correctly rounded quantities of the refit from the summed digits: k < 6 -> M_k =
// RN(n P_k - L_a L_b) (k = xx, xy, xz, yy, yz, zz), k = 6 + a -> RN(L_a).  Independent of each
// other: the device evaluates them in nine lanes.
DLG_HD inline double refit_entry(const int64_t* dig, int k) {
  if (k >= 6) return big_to_double(big_lin(dig + 1 + 2 * (k - 6)));
  const int ia = k < 3 ? 0 : (k < 5 ? 1 : 2), ib = k < 3 ? k : (k < 5 ? k - 2 : 2);
  const Big La = big_lin(dig + 1 + 2 * ia), Lb = big_lin(dig + 1 + 2 * ib);
  return big_to_double(
      big_add(big_mul(big_i64(dig[0]), big_prod(dig + 7 + 4 * k)), big_neg(big_mul(La, Lb))));
}

// the plane from the nine entries (n = dig[0] >= 4): Jacobi, orientation, centre
DLG_HD inline void refit_finish(const double e[9], int64_t n, int qexp, const float cin[4],
                                float cout[4]) {
  const double* m6 = e;
  double A[9] = {m6[0], m6[1], m6[2], m6[1], m6[3], m6[4], m6[2], m6[4], m6[5]};
  double V[9];
  jacobi3(A, V);
  int k = 0;  // smallest eigenvalue (ties: lowest index)
  if (A[4] < A[0]) k = 1;
  if (A[8] < (k == 0 ? A[0] : A[4])) k = 2;
  // (column k by selects: no dynamically indexed array on the device)
  double v0 = k == 0 ? V[0] : (k == 1 ? V[1] : V[2]);
  double v1 = k == 0 ? V[3] : (k == 1 ? V[4] : V[5]);
  double v2 = k == 0 ? V[6] : (k == 1 ? V[7] : V[8]);
  const double nv = sqrt((v0 * v0 + v1 * v1) + v2 * v2);
  v0 = v0 / nv; v1 = v1 / nv; v2 = v2 / nv;
  if ((v0 * (double)cin[0] + v1 * (double)cin[1]) + v2 * (double)cin[2] < 0.0) {
    v0 = -v0; v1 = -v1; v2 = -v2;
  }
  const double nd = (double)n, back = pow2d(qexp - kFastBits);
  const double c0 = e[6] / nd * back;
  const double c1 = e[7] / nd * back;
  const double c2 = e[8] / nd * back;
  const double d = -((v0 * c0 + v1 * c1) + v2 * c2);
  cout[0] = (float)v0; cout[1] = (float)v1; cout[2] = (float)v2; cout[3] = (float)d;
}

// the fast refit from the summed digits (see the definition at the top)
DLG_HD inline void refit_exact(const int64_t* dig, int qexp, const float cin[4], float cout[4]) {
  const int64_t n = dig[0];
  if (n < 4) {
    for (int k = 0; k < 4; ++k) cout[k] = cin[k];
    return;
  }
  double e[9];
  for (int k = 0; k < 9; ++k) e[k] = refit_entry(dig, k);
  refit_finish(e, n, qexp, cin, cout);
}

}  // namespace dlg
