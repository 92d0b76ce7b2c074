"""Independent numpy restatement of the PCL-1.8 RANSAC plane path -- TEST INFRASTRUCTURE ONLY.

Written separately from pcl_oracle.c so the two cross-check each other:
  * RNG: numpy's own MT19937 (legacy init_genrand seeding == boost::mt19937(12345u)),
    rnd() = raw >> 1 (boost uniform_int<>(0, INT_MAX), bucket size 2);
  * float32 arithmetic with explicit rounding at every op (numpy never fuses), Eigen SSE
    predux order for 4-vector dots, Eigen-3.3 normalize guard;
  * refit: single-pass float32 sums in index order (np.cumsum is sequential), eigen33 with
    atan2/cos/sin evaluated in double and rounded to float32 (within 1 ulp of the C libm's
    atan2f/cosf/sinf; so refined coefficients agree with the C oracle to ~1e-7, not bitwise).
"""
from __future__ import annotations

import math

import numpy as np

F = np.float32
EPS_F = np.finfo(np.float32).eps
MIN_F = np.finfo(np.float32).tiny
DBL_EPS = np.finfo(np.float64).eps


class Rnd:
    """boost::variate_generator<mt19937&, uniform_int<>(0, INT_MAX)> over numpy's MT19937."""

    def __init__(self, seed=12345, block=4096):
        self.bg = np.random.RandomState(seed)._bit_generator
        self.buf = np.zeros(0, np.int64)
        self.pos = 0
        self.block = block

    def __call__(self) -> int:
        if self.pos >= self.buf.shape[0]:
            self.buf = (self.bg.random_raw(self.block).astype(np.uint64) >> np.uint64(1)).astype(np.int64)
            self.pos = 0
        v = int(self.buf[self.pos])
        self.pos += 1
        return v


def sample_good(p0, p1, p2):
    with np.errstate(divide="ignore", invalid="ignore"):
        d = (p1 - p0) / (p2 - p0)
    return bool((d[0] != d[1]) or (d[2] != d[1]))


def coefficients(p0, p1, p2):
    a = (p1 - p0).astype(F)
    b = (p2 - p0).astype(F)
    with np.errstate(divide="ignore", invalid="ignore"):
        r = a / b
    if r[0] == r[1] and r[2] == r[1]:
        return None
    c0 = F(a[1] * b[2]) - F(a[2] * b[1])
    c1 = F(a[2] * b[0]) - F(a[0] * b[2])
    c2 = F(a[0] * b[1]) - F(a[1] * b[0])
    c3 = F(0.0)
    z = F(F(c0 * c0) + F(c2 * c2)) + F(F(c1 * c1) + F(c3 * c3))
    if z > F(0):
        s = np.sqrt(z)
        c0, c1, c2, c3 = c0 / s, c1 / s, c2 / s, c3 / s
    dot = F(F(c0 * p0[0]) + F(c2 * p0[2])) + F(F(c1 * p0[1]) + F(c3 * F(1.0)))
    return np.array([c0, c1, c2, F(-1.0) * dot], dtype=F)


def abs_dist(c, x, y, z):
    c = c.astype(F)
    return np.abs((c[0] * x + c[2] * z) + (c[1] * y + c[3]))


def within(c, pts, thr):
    d = abs_dist(c, pts[:, 0], pts[:, 1], pts[:, 2])
    return d.astype(np.float64) < thr


def seq_sum(v):
    return F(np.cumsum(v.astype(F), dtype=F)[-1]) if v.shape[0] else F(0)


def mean_cov(pts):
    x, y, z = pts[:, 0], pts[:, 1], pts[:, 2]
    a = [seq_sum(x * x), seq_sum(x * y), seq_sum(x * z), seq_sum(y * y), seq_sum(y * z),
         seq_sum(z * z), seq_sum(x), seq_sum(y), seq_sum(z)]
    n = F(pts.shape[0])
    a = [F(v / n) for v in a]
    cov = np.zeros(9, F)
    cov[0] = a[0] - F(a[6] * a[6]); cov[1] = a[1] - F(a[6] * a[7]); cov[2] = a[2] - F(a[6] * a[8])
    cov[4] = a[3] - F(a[7] * a[7]); cov[5] = a[4] - F(a[7] * a[8]); cov[8] = a[5] - F(a[8] * a[8])
    cov[3], cov[6], cov[7] = cov[1], cov[2], cov[5]
    return cov, np.array([a[6], a[7], a[8], F(1)], F)


def _roots2(b, c):
    d = F(float(F(b * b)) - 4.0 * float(c))
    if d < F(0):
        d = F(0)
    sd = np.sqrt(d)
    return [F(0), F(F(0.5) * F(b - sd)), F(F(0.5) * F(b + sd))]


def compute_roots(m):
    m = m.reshape(3, 3)
    c0 = F(F(F(F(m[0, 0] * m[1, 1]) * m[2, 2]) + F(F(F(F(2) * m[0, 1]) * m[0, 2]) * m[1, 2]))
           - F(F(m[0, 0] * m[1, 2]) * m[1, 2]))
    c0 = F(F(c0 - F(F(m[1, 1] * m[0, 2]) * m[0, 2])) - F(F(m[2, 2] * m[0, 1]) * m[0, 1]))
    c1 = F(F(m[0, 0] * m[1, 1]) - F(m[0, 1] * m[0, 1]))
    c1 = F(c1 + F(m[0, 0] * m[2, 2]))
    c1 = F(c1 - F(m[0, 2] * m[0, 2]))
    c1 = F(c1 + F(m[1, 1] * m[2, 2]))
    c1 = F(c1 - F(m[1, 2] * m[1, 2]))
    c2 = F(F(m[0, 0] + m[1, 1]) + m[2, 2])
    if abs(c0) < EPS_F:
        return _roots2(c2, c1)
    s_inv3 = F(1.0 / 3.0)
    s_sqrt3 = np.sqrt(F(3.0))
    c2_over_3 = F(c2 * s_inv3)
    a_over_3 = F(F(c1 - F(c2 * c2_over_3)) * s_inv3)
    if a_over_3 > F(0):
        a_over_3 = F(0)
    half_b = F(F(0.5) * F(c0 + F(c2_over_3 * F(F(F(F(2) * c2_over_3) * c2_over_3) - c1))))
    q = F(F(half_b * half_b) + F(F(a_over_3 * a_over_3) * a_over_3))
    if q > F(0):
        q = F(0)
    rho = np.sqrt(F(-a_over_3))
    theta = F(F(math.atan2(float(np.sqrt(F(-q))), float(half_b))) * s_inv3)
    ct = F(math.cos(float(theta)))
    st = F(math.sin(float(theta)))
    r = [F(c2_over_3 + F(F(F(2) * rho) * ct)),
         F(c2_over_3 - F(rho * F(ct + F(s_sqrt3 * st)))),
         F(c2_over_3 - F(rho * F(ct - F(s_sqrt3 * st))))]
    if r[0] >= r[1]:
        r[0], r[1] = r[1], r[0]
    if r[1] >= r[2]:
        r[1], r[2] = r[2], r[1]
        if r[0] >= r[1]:
            r[0], r[1] = r[1], r[0]
    if r[0] <= F(0):
        return _roots2(c2, c1)
    return r


def eigen33(mat):
    mat = np.asarray(mat, F).reshape(9)
    scale = F(np.max(np.abs(mat)))
    if scale <= MIN_F:
        scale = F(1)
    m = (mat / scale).astype(F).reshape(3, 3)
    r = compute_roots(m)
    ev = F(r[0] * scale)
    for i in range(3):
        m[i, i] = F(m[i, i] - r[0])

    def cross(a, b):
        return np.array([F(a[1] * b[2]) - F(a[2] * b[1]), F(a[2] * b[0]) - F(a[0] * b[2]),
                         F(a[0] * b[1]) - F(a[1] * b[0])], F)

    v1, v2, v3 = cross(m[0], m[1]), cross(m[0], m[2]), cross(m[1], m[2])

    def sqn(v):
        return F(F(v[0] * v[0]) + F(F(v[1] * v[1]) + F(v[2] * v[2])))

    l1, l2, l3 = sqn(v1), sqn(v2), sqn(v3)
    if l1 >= l2 and l1 >= l3:
        v, l = v1, l1
    elif l2 >= l1 and l2 >= l3:
        v, l = v2, l2
    else:
        v, l = v3, l3
    return ev, (v / np.sqrt(l)).astype(F)


def optimize(pts, inl, c):
    if inl.shape[0] < 4:
        return c.copy()
    cov, cen = mean_cov(pts[inl])
    _, v = eigen33(cov)
    dot = F(F(v[0] * cen[0]) + F(v[2] * cen[2])) + F(F(v[1] * cen[1]) + F(F(0) * cen[3]))
    return np.array([v[0], v[1], v[2], F(-1.0) * dot], F)


def sac_segment(points, threshold, indices=None, max_iterations=50, probability=0.99,
                optimize_coefficients=True, seed=12345):
    pts = np.ascontiguousarray(points, F)[:, :3]
    idx = np.arange(pts.shape[0], dtype=np.int64) if indices is None else np.asarray(indices, np.int64)
    n = idx.shape[0]
    sub = pts[idx]
    shuf = idx.copy()
    rnd = Rnd(seed)
    it, best, k = 0, -(2 ** 31 - 1), 1.0
    log_p = math.log(1.0 - probability) if probability < 1.0 else -math.inf
    one_over = 1.0 / n if n else math.inf
    max_skip = max_iterations * 10
    skipped = 0
    best_c = best_s = None
    draws = 0
    while it < k and skipped < max_skip:
        if n < 3:
            it = 2 ** 31 - 2
            break
        found = False
        for _ in range(1000):
            for i in range(3):
                j = i + rnd() % (n - i)
                shuf[i], shuf[j] = shuf[j], shuf[i]
            draws += 1
            s = shuf[:3].copy()
            if sample_good(pts[s[0]], pts[s[1]], pts[s[2]]):
                found = True
                break
        if not found:
            break
        c = coefficients(pts[s[0]], pts[s[1]], pts[s[2]])
        if c is None:
            skipped += 1
            continue
        cnt = int(np.count_nonzero(within(c, sub, threshold)))
        if cnt > best:
            best, best_c, best_s = cnt, c, s
            w = best * one_over
            pno = 1.0 - w ** 3.0
            pno = min(max(DBL_EPS, pno), 1.0 - DBL_EPS)
            k = log_p / math.log(pno)
        it += 1
        if it > max_iterations:
            break
    if best_c is None:
        return dict(ok=False, coeff=np.zeros(4, F), inliers=np.zeros(0, np.int32), iterations=it,
                    draws=draws, best_sample=None, coeff_unrefined=None, n_unrefined=0)
    inl = idx[within(best_c, sub, threshold)]
    n_unref = inl.shape[0]
    coeff = best_c
    if optimize_coefficients:
        coeff = optimize(pts, inl, best_c)
        inl = idx[within(coeff, sub, threshold)]
    return dict(ok=True, coeff=coeff, inliers=inl.astype(np.int32), iterations=it, draws=draws,
                best_sample=best_s.astype(np.int32), coeff_unrefined=best_c, n_unrefined=n_unref)


def extract_planes(points, threshold, max_planes=20, min_inliers=0, **kw):
    pts = np.ascontiguousarray(points, F)[:, :3]
    rem = np.arange(pts.shape[0], dtype=np.int64)
    coeffs, inls, offs = [], [], [0]
    floor_n = max(3, min_inliers)
    while len(coeffs) < max_planes and rem.shape[0] >= floor_n:
        r = sac_segment(pts, threshold, indices=rem, **kw)
        nin = r["inliers"].shape[0]
        if not r["ok"] or nin == 0 or nin < min_inliers:
            break
        coeffs.append(r["coeff"])
        inls.append(r["inliers"])
        offs.append(offs[-1] + nin)
        rem = np.setdiff1d(rem, r["inliers"].astype(np.int64), assume_unique=True)
    return dict(coeffs=np.array(coeffs, F).reshape(-1, 4), offsets=np.array(offs, np.int64),
                inliers=np.concatenate(inls).astype(np.int32) if inls else np.zeros(0, np.int32),
                n_planes=len(coeffs))
