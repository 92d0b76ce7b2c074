// fsum.hpp -- PCL's sequential float sums, evaluated in parallel and bit-exactly.
//
// optimizeModelCoefficients (PCL 1.8 SampleConsensusModelPlane) refits the plane with
// pcl::computeMeanAndCovarianceMatrix, whose dense branch runs nine float accumulators over the
// inliers in list order (accu[0] += x*x, accu[1] += x*y, ..., accu[8] += z; the same arithmetic
// as pcl::computePointNormal at Dialog/PlaneDetect.h:1084, 1130, 1152, 1386, 1485).  Each
// accumulator is a chain s_j = fl(s_{j-1} + p_j) from s_0 = +0: sequential by definition, and
// ~0.4 ms per chain on a CPU core at 450k inliers.  This file evaluates such a chain in parallel
// and gets exactly the sequential bits.
//
// Translation lemma.  In a binade [2^E, 2^(E+1)) floats are the multiples of q_E = 2^(E-150) and
// fl(v) = q_E * rne(v / q_E).  Shifting v by D, an even multiple of q_E, shifts rne by D / q_E
// (ties included: the parity is unchanged).  So a run of the chain started at a, s_0 = a,
// s_j = fl(s_{j-1} + p_j), gives the run started at a + D as s_j + D, provided at every step the
// exact sums v_j and v_j + D fall in the same binade, and D is a multiple of 2 q_j there.
// Sufficient per step (s_j in binade E_j, q_j its quantum):  |D| <= min(|s_j| - 2^E_j,
// 2^(E_j+1) - |s_j|) - q_j  (then |v_j - s_j| <= q_j / 2 keeps v_j and v_j + D inside), and
// D = 0 mod 2 q_j.  A run therefore records its output o, the margin mu = the minimum of that
// bound over its steps and qm = the largest q_j; a run started at g + i q(g) for i = 0..3 (a fan
// of four consecutive floats around a guess g) covers every start t = g + d q(g): take
// i = d mod 4, D = (d - i) q(g); the result is o_i + D when qm_i <= 2 q(g) and |D| <= mu_i, or
// o_i itself when D = 0 (the run is then the computation).
//
// Records and the walk.  Chunks of kFsChunk elements get a record each: the fan of four runs
// from the guess g_k = fl(double prefix of the terms before chunk k), all chunks and chains in
// parallel.  The chain's value is then carried across the chunks from +0: a chunk whose record
// covers the arriving value is applied (one translation), any other chunk is rerun from that
// value.  Every value produced is a literal run of the chain or a shift the lemma proves exact,
// so the result is the sequential sum bit for bit whatever the guesses; the guesses only decide
// how many chunks have to be rerun.  The device walks 64 records at a time, one per lane
// (fsum.hip, k_fs_walk): lane l speculates that its chunk starts at the exact value plus the
// prefix sum of the increments o_m - start_m of the lanes before it, applies its record to that
// start, and checks the result against the next lane's speculated start.  The lanes before the
// first failed check are proven exact by induction (each verified lane's output is the exact
// start of the next); the first failed lane is applied or rerun alone from its start, which is
// exact, and the speculation restarts after it.
//
// Used by fsum.hip (device) and tests/cpp/fsum_host.cpp (host emulation of the same walk, CPU
// test against the literal loop).  Build with -ffp-contract=off: p_j = x * y and s + p are
// separate roundings, as in PCL.
#pragma once

#include <cmath>
#include <cstdint>

#include "host_math.hpp"

namespace dlg {

constexpr int kFsChains = 9;    // accu[0..8] of computeMeanAndCovarianceMatrix
constexpr int kFsChunk = 64;    // elements per record
constexpr int kFsFan = 4;       // member starts per record

DLG_HD inline uint32_t fs_bits(float f) { return __builtin_bit_cast(uint32_t, f); }
DLG_HD inline float fs_float(uint32_t u) { return __builtin_bit_cast(float, u); }

// term p_j of chain c for the point (x, y, z), in PCL's accumulator order
DLG_HD inline float fs_term(int c, float x, float y, float z) {
  switch (c) {
    case 0: return x * x;
    case 1: return x * y;
    case 2: return x * z;
    case 3: return y * y;
    case 4: return y * z;
    case 5: return z * z;
    case 6: return x;
    case 7: return y;
    default: return z;
  }
}

// quantum (ulp spacing) of the binade holding g; NaN for a non-finite g
DLG_HD inline float fs_quantum(float g) {
  const uint32_t e = (fs_bits(g) >> 23) & 0xFFu;
  if (e == 0xFFu) return fs_float(0x7FC00000u);
  if (e <= 23u) return fs_float(1u << (e == 0u ? 0u : e - 1u));  // 2^(e-150), subnormal
  return fs_float((e - 23u) << 23);
}

// 1 / fs_quantum(g) as an exact double (the quantum is 2^(max(e, 1) - 150)); NaN when g is not
// finite.  Multiplying by it is the exact division by the quantum.
DLG_HD inline double fs_inv_quantum(float g) {
  const uint32_t e = (fs_bits(g) >> 23) & 0xFFu;
  if (e == 0xFFu) return __builtin_nan("");
  const uint64_t be = 1023u + 150u - (e == 0u ? 1u : e);
  return __builtin_bit_cast(double, be << 52);
}

// a node's record: guess g (member i starts at g + i q(g)) and per member the run's output, its
// margin (largest |shift| the run tolerates) and its largest quantum; qm = NaN: member unusable
// (its start g + i q(g) is not a float)
struct alignas(16) FsNode {
  float g, pad0, pad1, pad2;
  float o[kFsFan];
  float mu[kFsFan];
  float qm[kFsFan];
};

struct FsRun {
  float o, mu, qm;
};

// one step of a run: s <- fl(s + p), margin and quantum bookkeeping
struct FsState {
  float s, mu, pe;  // value, running margin, largest 2^E
};

DLG_HD inline void fs_step(FsState& st, float p) {
  st.s = st.s + p;
  const float pe = fs_float(fs_bits(st.s) & 0x7F800000u);  // 2^E (0 for zero / subnormal)
  const float as = std::fabs(st.s);
  // |s| - 2^E - q and 2^(E+1) - q - |s|: exact (multiples of q below 2^E); <= 0 for a zero or
  // subnormal s, so such a step tolerates no shift
  const float lo = std::fma(pe, -1.00000012f, as);
  const float hi = std::fma(pe, 1.99999988f, -as);
  st.mu = std::fmin(st.mu, std::fmin(lo, hi));
  st.pe = std::fmax(st.pe, pe);
}

DLG_HD inline FsRun fs_finish(const FsState& st) {
  FsRun r{st.s, st.mu, st.pe * 1.1920929e-07f};  // pe * 2^-23 (exact)
  // a non-finite run (overflow, NaN term) stays non-finite to its end: never shifted
  if (!(std::fabs(st.s) <= 3.40282347e+38f)) r.mu = -1.0f;
  return r;
}

DLG_HD inline FsState fs_start(float a) { return FsState{a, INFINITY, 0.0f}; }

// the start of member i around g, or NaN-flagged when g + i q is not a float
DLG_HD inline bool fs_member_start(float g, int i, float* a) {
  const float q = fs_quantum(g);
  const double ad = (double)g + (double)i * (double)q;
  *a = (float)ad;
  return (double)*a == ad;
}

struct FsApply {
  float out, mu, qm;
};

// a[i] for a runtime i in 0..3 without indexing (keeps a record in registers on the device)
DLG_HD inline float fs_sel4(const float (&a)[kFsFan], int i) {
  return i == 0 ? a[0] : i == 1 ? a[1] : i == 2 ? a[2] : a[3];
}

// apply node nd to the arrival t: true (and the exact result) when the lemma covers it
DLG_HD inline bool fs_apply(float t, const FsNode& nd, FsApply* r) {
  const float q = fs_quantum(nd.g);
  const double qd = (double)q;
  const double iq = fs_inv_quantum(nd.g);
  const double tq = (double)t * iq;  // exact (a power-of-two scaling within double's range)
  if (!(std::fabs(tq) < 4503599627370496.0) || tq != std::floor(tq)) return false;  // NaN too
  const double dl = tq - (double)nd.g * iq;                                           // exact
  const double d4 = std::floor(dl * 0.25);
  const int i = (int)(dl - 4.0 * d4);
  const double D = (dl - (double)i) * qd;
  const float qm = fs_sel4(nd.qm, i), oi = fs_sel4(nd.o, i), mui = fs_sel4(nd.mu, i);
  if (!(qm >= 0.0f)) return false;  // member unusable
  if (D == 0.0) {                   // t is member i's start: its run is the computation
    r->out = oi;
    r->mu = mui;
    r->qm = qm;
    return true;
  }
  const double aD = std::fabs(D);
  if (!((double)qm <= 2.0 * qd) || !(aD <= (double)mui)) return false;
  r->out = (float)((double)oi + D);  // exact
  // the margin left for a further shift, rounded down
  const double rem = (double)mui - aD;
  float rf = (float)rem;
  if ((double)rf > rem) rf = std::nextafter(rf, -INFINITY);
  r->mu = rf;
  r->qm = qm;
  return true;
}

// the speculative increment of a record for a start `off` above its guess: o_i - start_i of the
// member i = (off / q) mod 4 that start would select (member 0 when off is not a multiple of
// q(g), or when i is unusable; exact in double: two floats of nearby binades); NaN when no member
// is usable.  The walk passes the offset between its exact value and the guess of the first
// record it speculates on: the refined guesses lag the chain by the same amount until the next
// chunk whose increment depends on its start.
DLG_HD inline double fs_increment(const FsNode& nd, double off) {
  const double qd = (double)fs_quantum(nd.g);
  const double d = off * fs_inv_quantum(nd.g);
  int i = 0;
  if (std::fabs(d) < 4503599627370496.0 && d == std::floor(d)) i = (int)(d - 4.0 * std::floor(d * 0.25));
  if (!(fs_sel4(nd.qm, i) >= 0.0f))
    i = nd.qm[0] >= 0.0f ? 0 : nd.qm[1] >= 0.0f ? 1 : nd.qm[2] >= 0.0f ? 2 : 3;
  if (!(fs_sel4(nd.qm, i) >= 0.0f)) return __builtin_nan("");
  return (double)fs_sel4(nd.o, i) - ((double)nd.g + (double)i * qd);
}

// chunk records for n elements
DLG_HD inline int64_t fs_chunks(int64_t n) { return (n + kFsChunk - 1) / kFsChunk; }

// the refit's tail (refit_pcl_float after the sums): a = the nine sums, n = inlier count.
// Float transcendentals of eigen33 are PCL's as restated in host_math.hpp (the double function
// rounded to float); on the device the double result may differ from the host's libm by a few
// ulps, so *uncertain is set when it lies within 2^-46 (relative) of a float rounding boundary
// -- then only the host value is authoritative.
struct CheckedTx {
  bool* unc;
  DLG_HD float round_checked(double r) const {
    const float f = (float)r;
    const double e = std::fabs(r) * 1.4210854715202004e-14;  // 2^-46
    if ((float)(r - e) != f || (float)(r + e) != f) *unc = true;
    return f;
  }
  DLG_HD float atan2(float y, float x) const { return round_checked(::atan2((double)y, (double)x)); }
  DLG_HD float cos(float x) const { return round_checked(::cos((double)x)); }
  DLG_HD float sin(float x) const { return round_checked(::sin((double)x)); }
};

template <typename TX>
DLG_HD inline void fs_refit_tail_tx(const float a_in[9], int64_t n, const float cin[4],
                                    float cout[4], const TX& tx) {
  if (n < 4) {
    for (int k = 0; k < 4; ++k) cout[k] = cin[k];
    return;
  }
  float a[9];
  const float cnt = (float)(uint64_t)n;
  for (int k = 0; k < 9; ++k) a[k] = a_in[k] / cnt;
  float cov[9];
  cov[0] = a[0] - a[6] * a[6];
  cov[1] = a[1] - a[6] * a[7];
  cov[2] = a[2] - a[6] * a[8];
  cov[4] = a[3] - a[7] * a[7];
  cov[5] = a[4] - a[7] * a[8];
  cov[8] = a[5] - a[8] * a[8];
  cov[3] = cov[1]; cov[6] = cov[2]; cov[7] = cov[5];
  float ev, v[3];
  eigen33_tx(cov, &ev, v, tx);
  const float c3 = 0.0f, cw = 1.0f;
  const float dot = (v[0] * a[6] + v[2] * a[8]) + (v[1] * a[7] + c3 * cw);
  cout[0] = v[0]; cout[1] = v[1]; cout[2] = v[2]; cout[3] = -1.0f * dot;
}

// device form: flags transcendentals it cannot round for certain
DLG_HD inline void fs_refit_tail(const float a[9], int64_t n, const float cin[4], float cout[4],
                                 bool* uncertain) {
  fs_refit_tail_tx(a, n, cin, cout, CheckedTx{uncertain});
}

// host form: the authoritative value (refit_pcl_float's arithmetic after the sums)
DLG_HD inline void fs_refit_tail_plain(const float a[9], int64_t n, const float cin[4],
                                       float cout[4]) {
  fs_refit_tail_tx(a, n, cin, cout, PlainTx());
}

}  // namespace dlg
