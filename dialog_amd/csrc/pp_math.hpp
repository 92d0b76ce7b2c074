// pp_math.hpp -- float arithmetic of postProcessPlanes' point-in-polygon test, shared by the
// host driver (ray / edge set-up) and the kernels (postprocess.hip).  Build with
// -ffp-contract=off and IEEE f32 division / sqrt: the results are compared bit for bit.
//
// Follows Dialog/PlaneDetect.h: projPoint2Plane (:1437-1443), distP2P (:203-207),
// isBothLineSegsIntersect (:1966-2015), isPointInPoly (:1891-1964).  Eigen 3.3 Vector3f
// (not vectorised): dot = a0 b0 + (a1 b1 + a2 b2), normalize() divides by sqrt(squaredNorm)
// only when it is > 0.  pow(a, 0.5f) in distP2P is the correctly rounded square root.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

#include "host_math.hpp"

namespace dlg {

struct V3 {
  float x, y, z;
};

DLG_HD inline V3 v3(float x, float y, float z) { return V3{x, y, z}; }
DLG_HD inline V3 v3_sub(V3 a, V3 b) { return V3{a.x - b.x, a.y - b.y, a.z - b.z}; }
DLG_HD inline float v3_dot(V3 a, V3 b) { return a.x * b.x + (a.y * b.y + a.z * b.z); }
DLG_HD inline V3 v3_cross(V3 a, V3 b) {
  return V3{a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x};
}
DLG_HD inline V3 v3_normalized(V3 v) {
  const float z = v.x * v.x + (v.y * v.y + v.z * v.z);
  if (z > 0.0f) {
    const float s = m_sqrt(z);
    v.x /= s; v.y /= s; v.z /= s;
  }
  return v;
}
// distP2P: pow(((dx dx + dy dy) + dz dz), 0.5f)
DLG_HD inline float dist_p2p(V3 a, V3 b) {
  const float dx = a.x - b.x, dy = a.y - b.y, dz = a.z - b.z;
  return m_sqrt((dx * dx + dy * dy) + dz * dz);
}

// projPoint2Plane: lambda = float(2.0 * (float dot)), the update in double, stored as float
DLG_HD inline V3 proj_to_plane(V3 p, float4 c) {
  const float lam = (float)(2.0 * (double)(((c.x * p.x + c.y * p.y) + c.z * p.z) + c.w));
  const double h = (double)lam / 2.0;
  return V3{(float)((double)p.x - h * (double)c.x), (float)((double)p.y - h * (double)c.y),
            (float)((double)p.z - h * (double)c.z)};
}

// one border edge, prepared once per plane: a, b, normalize(b - a), distP2P(a, b)
struct PipEdge {
  float4 a_dab;  // a.xyz, |ab|
  float4 b;      // b.xyz, |a|_1
  float4 nab;    // normalize(b - a), 0
};

// one test ray of a candidate: c = projected point, d = c + 10000 * dir, normalize(d - c), |cd|
struct PipRay {
  V3 d, ncd;
  float dcd;
};

DLG_HD inline PipRay make_ray(V3 c, V3 dir) {
  const float lambda = 10000.0f;
  PipRay r;
  r.d = V3{c.x + lambda * dir.x, c.y + lambda * dir.y, c.z + lambda * dir.z};
  r.ncd = v3_normalized(v3_sub(r.d, c));
  r.dcd = dist_p2p(c, r.d);
  return r;
}

// isBothLineSegsIntersect(a, b, c, d) with the edge and ray terms precomputed;
// pa_l1 = |a|_1, pc_l1 = |c|_1 (only used by the early out)
DLG_HD inline bool segs_intersect(V3 pa, V3 pb, V3 nab, float dab, float pa_l1, V3 pc,
                                  float pc_l1, const PipRay& r) {
  const V3 pa_pc = v3_sub(pc, pa);
  const float d = v3_dot(nab, r.ncd);
  // Division-free exact early out.  For 0.05 <= |d| <= 0.97 (general branch below) the
  // position of pi along ab is, in exact arithmetic, s = l1 = (f - e d) / (1 - d^2) with
  // f = nab.(c - a), e = ncd.(c - a).  Propagating the float errors of l2, l1, p1, p2, pi and
  // (pi - a).nab (|l1|, |l2| <= 34 W for W = |c - a|_1, 1 - d^2 >= 0.059) bounds the computed s
  // within 0.0045 W + 1.2e-7 (|a|_1 + |c|_1) of (f - e d) / (1 - d^2), and the margin m of the
  // second early out by 0.0006 + 2.4e-4 W + 4e-6 |ab|; T below exceeds their sum (W term 2x), so
  // a pair rejected here is rejected by that (exact) test as well.
  const float ad = m_fabs(d);
  if (ad >= 0.05f && ad <= 0.97f && dab > 1e-15f) {
    const float f = v3_dot(nab, pa_pc), e = v3_dot(r.ncd, pa_pc);
    const float W = (m_fabs(pa_pc.x) + m_fabs(pa_pc.y)) + m_fabs(pa_pc.z);
    const float T = 0.0006f + 0.0103f * W + 1e-6f * (pa_l1 + pc_l1) + 4e-6f * dab;
    const float c1 = 1.0f - d * d;
    const float num = f - e * d;
    if (num < -T * c1 || num > (dab + T) * c1) return false;
  }
  float l1, l2;
  if (m_fabs(d) <= 0.001f) {
    l1 = v3_dot(nab, pa_pc);
    l2 = -1.0f * v3_dot(r.ncd, pa_pc);
  } else if (d >= 0.9999f) {
    return false;
  } else {
    const float c1 = 1.0f - d * d;
    const float c2 = v3_dot(nab, pa_pc) * d - v3_dot(r.ncd, pa_pc);
    l2 = c2 / c1;
    l1 = (l2 + v3_dot(r.ncd, pa_pc)) / d;
  }
  const V3 p1{pa.x + l1 * nab.x, pa.y + l1 * nab.y, pa.z + l1 * nab.z};
  const V3 p2{pc.x + l2 * r.ncd.x, pc.y + l2 * r.ncd.y, pc.z + l2 * r.ncd.z};
  const V3 pi{(p1.x + p2.x) / 2.0f, (p1.y + p2.y) / 2.0f, (p1.z + p2.z) / 2.0f};
  // Exact early out (same result, fewer square roots): with s = (pi - a).nab the position of
  // pi along ab, |pi-a| + |pi-b| - |ab| >= 2 max(-s, s - |ab|).  When pi lies beyond an end of
  // ab by more than 0.0005 plus a bound on the float errors of s, of the three distances and of
  // their sum (< 1.5e-6 (|pi-a|_1 + |ab|), taken as 4e-6 (... + 1)), the computed
  // |dpa + dpb - dab| is >= 0.001 and the test fails.  Edges shorter than 1e-15 (nab normalised
  // from a denormal squared norm, not unit to 2^-22), NaN and inf take the full test.
  const V3 ha = v3_sub(pi, pa);
  const float s = v3_dot(ha, nab);
  const float m = 0.0005f + 4e-6f * ((m_fabs(ha.x) + m_fabs(ha.y) + m_fabs(ha.z)) + dab + 1.0f);
  if (dab > 1e-15f && (s < -m || s > dab + m)) return false;
  if (!(m_fabs(dist_p2p(pi, pa) + dist_p2p(pi, pb) - dab) < 0.001f)) return false;
  return m_fabs(dist_p2p(pi, pc) + dist_p2p(pi, r.d) - r.dcd) < 0.001f;
}

// MSVC CRT rand() (srand(seed) then rand(): LCG 214013 / 2531011, bits 16..30)
inline uint32_t msvc_rand(uint32_t& state) {
  state = state * 214013u + 2531011u;
  return (state >> 16) & 0x7fffu;
}

constexpr int kPipRays = 10;

}  // namespace dlg
