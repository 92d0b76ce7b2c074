// np_dev.hpp -- device arithmetic of SACMODEL_NORMAL_PLANE and Eigen's normalize(), shared by the
// exhaustive (kernels.hip) and the pruned (spatial.hip) scoring kernels and the select passes.
#pragma once

#include <hip/hip_runtime.h>

#include <cmath>

namespace dlg {

// Eigen Vector4f(v0, v1, v2, 0).normalized(): z = (v0^2 + v2^2) + (v1^2 + 0); z > 0 ? v / sqrt(z)
__device__ __forceinline__ float4 eigen_normalized3(float v0, float v1, float v2, float w) {
  const float z = (v0 * v0 + v2 * v2) + (v1 * v1 + 0.0f * 0.0f);
  if (z > 0.0f) {
    const float s = sqrtf(z);
    return make_float4(v0 / s, v1 / s, v2 / s, w);
  }
  return make_float4(v0, v1, v2, w);
}

// SampleConsensusModelNormalPlane (PCL 1.8 sac_model_normal_plane.hpp), one point:
//   d_euclid = fabs(coeff.dot(p) + c3), coeff = (c0, c1, c2, 0), p = (x, y, z, 0)  [float]
//   d_normal = min(a, pi - a), a = acos(clamp(n.normalized() . coeff.normalized()))   [double]
//   fabs(w d_normal + (1 - w) d_euclid) < thr,  w = lambda (1 - curvature)          [double]
// cn = coeff.normalized(); nn = (n.normalized(), curvature); omw = 1 - w.  Prefilter: w >= 0 and
// d_normal >= 0 give fl(w d_normal + b) >= b = (1 - w) d_euclid, so b >= thr rejects exactly and
// the acos is only evaluated near the plane.
__device__ __forceinline__ float np_deuclid(float4 c, float x, float y, float z) {
  return fabsf(((c.x * x + c.z * z) + (c.y * y + 0.0f * 0.0f)) + c.w);
}
__device__ __forceinline__ bool np_full(float4 cn, float4 nn, double w, double b, double thr) {
  double rad = (double)((nn.x * cn.x + nn.z * cn.z) + (nn.y * cn.y + 0.0f * 0.0f));
  if (rad < -1.0) rad = -1.0;
  else if (rad > 1.0) rad = 1.0;
  // Fast decision: min(acos(rad), pi - acos(rad)) = acos(|rad|) to within 4e-4 when taken as
  // float acos of the float |rad| (the float rounding of rad moves acos by <= sqrt(2 * 6e-8)
  // near |rad| = 1, float acos adds ~1e-6): a result clear of thr by w * 4e-4 (and a few ulps
  // of the double sum) is PCL's; the band in between takes PCL's double arithmetic below.
  if (w == w && b == b && w >= 0.0 && w < 1e30) {
    const double a = (double)acosf((float)fabs(rad));
    const double v = fabs(w * a + b), e = w * 4e-4 + 1e-12 + 1e-9 * fabs(b);
    if (v < thr - e) return true;
    if (v > thr + e) return false;
  }
  double dn = fabs(acos(rad));
  const double alt = 3.14159265358979323846 - dn;  // M_PI
  if (alt < dn) dn = alt;                          // std::min(dn, M_PI - dn)
  return fabs(w * dn + b) < thr;
}
__device__ __forceinline__ bool np_test(float4 c, float4 cn, float x, float y, float z, float4 nn,
                                        double lambda, double thr) {
  const double w = lambda * (1.0 - (double)nn.w);
  const double b = (1.0 - w) * (double)np_deuclid(c, x, y, z);
  if (w >= 0.0 && !(b < thr)) return false;
  return np_full(cn, nn, w, b, thr);
}

// smallest float lim with fl((1 - w) lim) >= thr as a double product (the exact per-point form
// of PCL's prefilter b = (1 - w) d_euclid < thr); +inf when the prefilter does not apply
__device__ inline float np_de_limit(double w, double thr) {
  if (!(w >= 0.0)) return INFINITY;
  const double omw = 1.0 - w;
  if (!(omw > 0.0)) return INFINITY;
  if (!(thr > 0.0)) return thr == thr ? 0.0f : __builtin_nanf("");
  float x = (float)(thr / omw);
  if (!(x == x)) return INFINITY;
  while (!(omw * (double)x >= thr) && x < INFINITY) x = nextafterf(x, INFINITY);
  while (x > 0.0f) {
    const float y = nextafterf(x, -INFINITY);
    if (omw * (double)y >= thr) x = y;
    else break;
  }
  return x;
}


}  // namespace dlg
