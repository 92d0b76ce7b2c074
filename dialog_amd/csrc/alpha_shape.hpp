// alpha_shape.hpp -- the 2-D alpha shape pcl::ConcaveHull builds for a plane's border
// (polyPointCloud, Dialog/PlaneDetect.h:1399-1405; alpha = alpha_poly, config.txt:28), host C++.
//
// PCL 1.8's ConcaveHull<PointXYZ>::performReconstruction, dimension 2 (the reference's projected
// plane points), restated step by step:
//   1. centroid (compute3DCentroid, double), covariance (computeCovarianceMatrixNormalized,
//      double) and its eigenvectors (pcl::eigen33, double); transform1's rows are the
//      eigenvectors of the largest, middle and smallest eigenvalue, so the plane maps to z = 0;
//   2. the points demeaned (float) and transformed (double matrix, float result); their x, y are
//      qhull's input, triangulated with "d QJ" (Delaunay, joggled input);
//   3. a Delaunay triangle (qhull facet, not upper-Delaunay) is kept when the distance from its
//      circumcentre (the Voronoi vertex) to a vertex is <= alpha;
//   4. a ridge (edge) of a kept facet whose other facet is not kept, or is upper-Delaunay (the
//      convex hull), is a boundary edge; its vertices become the alpha shape's points in the
//      order the ridges are met; edges[a] lists every boundary neighbour of vertex a;
//   5. the boundary is walked into polygons: from the first vertex of `edges` (a std::map, so
//      the smallest index), repeatedly to its first not yet used neighbour, erasing the vertex;
//      when the next vertex has no edges left a new polygon starts at the smallest remaining
//      vertex; polygons of >= 3 vertices are kept;
//   6. the points go back through transform1's inverse and the centroid.
// The Delaunay triangulation here is a sweep-hull construction with edge flips (points sorted by
// distance from a seed triangle's circumcentre, the convex hull grown around them, every new
// edge legalised by the in-circle test).  Its structure follows mapbox's Delaunator
// (https://github.com/mapbox/delaunator, ISC licence, (c) Vladimir Agafonkin / Mapbox: the
// hullNext / hullPrev / hullTri / hullHash arrays, the pseudo-angle hash key, the legalisation
// edge stack and the hull-triangle fix-up), restated in C++ with double orientation tests and a
// long-double fallback near zero.  For points in general position the triangulation is
// unique, so the kept triangles and the boundary edge SET equal qhull's (checked against
// scipy.spatial.Delaunay, i.e. qhull, with "QJ": tests/test_borders.py).  What stays unpinned:
// qhull's version and joggle seed (cocircular inputs triangulate by the joggle), the order qhull
// visits facets and ridges (it fixes which boundary vertex is first and so where PCL's walk
// starts and which polygon is polygons[0]), and the joggled coordinates qhull hands back.
#pragma once

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <map>
#include <numeric>
#include <vector>

#include "host_math.hpp"

namespace dlg {
namespace alpha {

// 2-D Delaunay triangulation: tri[3t..3t+2] counter-clockwise vertex ids, half[e] the opposite
// half-edge of half-edge e (from tri[e] to tri[next(e)]) or -1 on the convex hull
struct Tri2 {
  std::vector<int32_t> tri, half;
};

inline int nxt(int e) { return e % 3 == 2 ? e - 2 : e + 1; }

// > 0: a, b, c counter-clockwise.  Evaluated in double; when the result is within its rounding
// bound, again in long double (the sign of a near-degenerate triple only decides between
// equally valid triangulations of (nearly) collinear points)
inline double orient2(const double* p, int a, int b, int c) {
  const double l = (p[2 * b] - p[2 * a]) * (p[2 * c + 1] - p[2 * a + 1]);
  const double r = (p[2 * b + 1] - p[2 * a + 1]) * (p[2 * c] - p[2 * a]);
  const double d = l - r;
  if (std::fabs(d) >= 3.3306690738754716e-16 * std::fabs(l + r) && d != 0.0) return d;
  const long double L = ((long double)p[2 * b] - p[2 * a]) * ((long double)p[2 * c + 1] - p[2 * a + 1]);
  const long double R = ((long double)p[2 * b + 1] - p[2 * a + 1]) * ((long double)p[2 * c] - p[2 * a]);
  return (double)(L - R);
}

// d inside the circumcircle of the counter-clockwise triangle a, b, c
inline bool in_circle(const double* p, int a, int b, int c, int d) {
  const long double dx = (long double)p[2 * a] - p[2 * d], dy = (long double)p[2 * a + 1] - p[2 * d + 1];
  const long double ex = (long double)p[2 * b] - p[2 * d], ey = (long double)p[2 * b + 1] - p[2 * d + 1];
  const long double fx = (long double)p[2 * c] - p[2 * d], fy = (long double)p[2 * c + 1] - p[2 * d + 1];
  const long double ap = dx * dx + dy * dy, bp = ex * ex + ey * ey, cp = fx * fx + fy * fy;
  return dx * (ey * cp - bp * fy) - dy * (ex * cp - bp * fx) + ap * (ex * fy - ey * fx) > 0;
}

inline double circum_r2(const double* p, int a, int b, int c, double* cx, double* cy) {
  const double dx = p[2 * b] - p[2 * a], dy = p[2 * b + 1] - p[2 * a + 1];
  const double ex = p[2 * c] - p[2 * a], ey = p[2 * c + 1] - p[2 * a + 1];
  const double bl = dx * dx + dy * dy, cl = ex * ex + ey * ey;
  const double dd = 0.5 / (dx * ey - dy * ex);
  const double x = (ey * bl - dy * cl) * dd, y = (dx * cl - ex * bl) * dd;
  if (cx) {
    *cx = p[2 * a] + x;
    *cy = p[2 * a + 1] + y;
  }
  return x * x + y * y;  // (inf / NaN for collinear points)
}

class Delaunay {
 public:
  Delaunay(const double* xy, int n) : p_(xy), n_(n) {}

  Tri2 run() {
    Tri2 out;
    if (n_ < 3) return out;
    double minx = INFINITY, miny = INFINITY, maxx = -INFINITY, maxy = -INFINITY;
    for (int i = 0; i < n_; ++i) {
      minx = std::min(minx, X(i)); maxx = std::max(maxx, X(i));
      miny = std::min(miny, Y(i)); maxy = std::max(maxy, Y(i));
    }
    const double mx = 0.5 * (minx + maxx), my = 0.5 * (miny + maxy);
    int i0 = -1, i1 = -1, i2 = -1;
    double best = INFINITY;
    for (int i = 0; i < n_; ++i) {
      const double d = dist2(mx, my, X(i), Y(i));
      if (d < best) { best = d; i0 = i; }
    }
    best = INFINITY;
    for (int i = 0; i < n_; ++i) {
      if (i == i0) continue;
      const double d = dist2(X(i0), Y(i0), X(i), Y(i));
      if (d < best && d > 0.0) { best = d; i1 = i; }
    }
    if (i1 < 0) return out;  // (every point identical)
    best = INFINITY;
    for (int i = 0; i < n_; ++i) {
      if (i == i0 || i == i1) continue;
      const double r = circum_r2(p_, i0, i1, i, nullptr, nullptr);
      if (r < best) { best = r; i2 = i; }
    }
    if (!(best < INFINITY)) return out;  // (all collinear: no triangle)
    if (orient2(p_, i0, i1, i2) < 0) std::swap(i1, i2);
    circum_r2(p_, i0, i1, i2, &cx_, &cy_);
    std::vector<double> dist(n_);
    for (int i = 0; i < n_; ++i) dist[i] = dist2(X(i), Y(i), cx_, cy_);
    std::vector<int32_t> ids(n_);
    std::iota(ids.begin(), ids.end(), 0);
    std::sort(ids.begin(), ids.end(), [&](int a, int b) {
      return dist[a] < dist[b] || (dist[a] == dist[b] && a < b);
    });
    hsize_ = (int)std::ceil(std::sqrt((double)n_));
    hash_.assign(hsize_, -1);
    next_.assign(n_, 0); prev_.assign(n_, 0); htri_.assign(n_, -1);
    tri_.reserve(6 * (size_t)n_); half_.reserve(6 * (size_t)n_);
    start_ = i0;
    next_[i0] = prev_[i2] = i1;
    next_[i1] = prev_[i0] = i2;
    next_[i2] = prev_[i1] = i0;
    htri_[i0] = 0; htri_[i1] = 1; htri_[i2] = 2;
    hash_[key(X(i0), Y(i0))] = i0;
    hash_[key(X(i1), Y(i1))] = i1;
    hash_[key(X(i2), Y(i2))] = i2;
    add(i0, i1, i2, -1, -1, -1);
    double xp = 0, yp = 0;
    for (int k = 0; k < n_; ++k) {
      const int i = ids[k];
      const double x = X(i), y = Y(i);
      if (k > 0 && x == xp && y == yp) continue;  // (exact duplicates: one vertex)
      xp = x; yp = y;
      if (i == i0 || i == i1 || i == i2) continue;
      // a hull edge visible from the point, found through the angle hash
      int s = 0;
      for (int j = 0, kk = key(x, y); j < hsize_; ++j) {
        s = hash_[(kk + j) % hsize_];
        if (s != -1 && s != next_[s]) break;
      }
      s = prev_[s];
      int e = s, q;
      while (q = next_[e], !(orient2(p_, e, q, i) < 0)) {
        e = q;
        if (e == s) { e = -1; break; }
      }
      if (e < 0) continue;  // (a duplicate of a hull point, or inside up to rounding)
      int t = add(e, i, next_[e], -1, -1, htri_[e]);
      htri_[i] = legalize(t + 2);
      htri_[e] = t;
      int nn = next_[e];
      while (q = next_[nn], orient2(p_, nn, q, i) < 0) {
        t = add(nn, i, q, htri_[i], -1, htri_[nn]);
        htri_[i] = legalize(t + 2);
        next_[nn] = nn;  // (removed from the hull)
        nn = q;
      }
      if (e == s) {
        while (q = prev_[e], orient2(p_, q, e, i) < 0) {
          t = add(q, i, e, -1, htri_[e], htri_[q]);
          legalize(t + 2);
          htri_[q] = t;
          next_[e] = e;
          e = q;
        }
      }
      start_ = prev_[i] = e;
      next_[e] = prev_[nn] = i;
      next_[i] = nn;
      hash_[key(x, y)] = i;
      hash_[key(X(e), Y(e))] = e;
    }
    out.tri.swap(tri_);
    out.half.swap(half_);
    return out;
  }

 private:
  double X(int i) const { return p_[2 * i]; }
  double Y(int i) const { return p_[2 * i + 1]; }
  static double dist2(double ax, double ay, double bx, double by) {
    const double dx = ax - bx, dy = ay - by;
    return dx * dx + dy * dy;
  }
  int key(double x, double y) const {  // pseudo-angle of (x, y) about the seed centre
    const double dx = x - cx_, dy = y - cy_;
    const double s = std::fabs(dx) + std::fabs(dy);
    const double pa = s > 0 ? dx / s : 0.0;
    const double a = (dy > 0 ? 3.0 - pa : 1.0 + pa) / 4.0;  // [0, 1]
    int k = (int)std::floor(a * hsize_);
    return ((k % hsize_) + hsize_) % hsize_;
  }
  void link(int a, int b) {
    half_[a] = b;
    if (b != -1) half_[b] = a;
  }
  int add(int a, int b, int c, int ha, int hb, int hc) {
    const int t = (int)tri_.size();
    tri_.push_back(a); tri_.push_back(b); tri_.push_back(c);
    half_.push_back(-1); half_.push_back(-1); half_.push_back(-1);
    link(t, ha); link(t + 1, hb); link(t + 2, hc);
    return t;
  }
  // flip half-edge a (and the edges a flip exposes) until the in-circle test holds; returns
  // the half-edge from the new point along the hull (as the recursive form would)
  int legalize(int a) {
    int ar = 0;
    stack_.clear();
    for (;;) {
      const int b = half_[a];
      const int a0 = a - a % 3;
      ar = a0 + (a + 2) % 3;
      if (b == -1) {
        if (stack_.empty()) break;
        a = stack_.back();
        stack_.pop_back();
        continue;
      }
      const int b0 = b - b % 3;
      const int al = a0 + (a + 1) % 3, bl = b0 + (b + 2) % 3;
      const int p0 = tri_[ar], pr = tri_[a], pl = tri_[al], p1 = tri_[bl];
      if (in_circle(p_, p0, pr, pl, p1)) {
        tri_[a] = p1;
        tri_[b] = p0;
        const int hbl = half_[bl];
        if (hbl == -1) {  // (the flipped edge's far side is on the hull: fix its reference)
          int e = start_;
          do {
            if (htri_[e] == bl) {
              htri_[e] = a;
              break;
            }
            e = prev_[e];
          } while (e != start_);
        }
        link(a, hbl);
        link(b, half_[ar]);
        link(ar, bl);
        const int br = b0 + (b + 1) % 3;
        if (stack_.size() < (size_t)(1 << 20)) stack_.push_back(br);
      } else {
        if (stack_.empty()) break;
        a = stack_.back();
        stack_.pop_back();
      }
    }
    return ar;
  }

  const double* p_;
  int n_;
  double cx_ = 0, cy_ = 0;
  int hsize_ = 1, start_ = 0;
  std::vector<int32_t> hash_, next_, prev_, htri_, tri_, half_, stack_;
};

// steps 3-5: the kept triangles (circumradius <= alpha, measured from the circumcentre to the
// triangle's first vertex as PCL measures it), the boundary edges in triangle order, the alpha
// shape's vertices in the order the edges meet them (av: point ids), and PCL's polygon walk
// (polygons of positions into av)
struct AlphaShape {
  std::vector<uint8_t> kept;          // per triangle
  std::vector<int32_t> av;            // alpha-shape vertex -> point id
  std::vector<std::vector<int32_t>> polygons;
};

inline AlphaShape alpha_shape(const double* xy, const Tri2& T, double alpha) {
  AlphaShape S;
  const int nt = (int)T.tri.size() / 3;
  S.kept.assign(nt, 0);
  for (int t = 0; t < nt; ++t) {
    double cx, cy;
    circum_r2(xy, T.tri[3 * t], T.tri[3 * t + 1], T.tri[3 * t + 2], &cx, &cy);
    const int v = T.tri[3 * t];
    const double r = std::sqrt((xy[2 * v] - cx) * (xy[2 * v] - cx) + (xy[2 * v + 1] - cy) * (xy[2 * v + 1] - cy));
    S.kept[t] = r <= alpha ? 1 : 0;  // (NaN: a degenerate triangle, not kept)
  }
  std::map<int32_t, int32_t> pos;  // point id -> alpha-shape index
  std::map<int, std::vector<int>> edges;
  auto idx = [&](int32_t v) {
    auto it = pos.find(v);
    if (it != pos.end()) return it->second;
    const int32_t k = (int32_t)S.av.size();
    pos.emplace(v, k);
    S.av.push_back(v);
    return k;
  };
  for (int t = 0; t < nt; ++t) {
    if (!S.kept[t]) continue;
    for (int j = 0; j < 3; ++j) {
      const int e = 3 * t + j, o = T.half[e];
      if (o != -1 && S.kept[o / 3]) continue;  // (interior edge of the alpha complex)
      const int a = idx(T.tri[e]), b = idx(T.tri[nxt(e)]);
      edges[a].push_back(b);
      edges[b].push_back(a);
    }
  }
  // PCL's walk (ConcaveHull::performReconstruction, dimension 2: the "Sort" loop)
  const int nv = (int)S.av.size();
  std::vector<uint8_t> used(nv, 0);
  std::vector<int32_t> order;
  std::vector<size_t> starts{0};
  auto cur = edges.begin();
  int next = -1;
  while (!edges.empty()) {
    order.push_back(cur->first);
    for (int v : cur->second)
      if (!used[v]) {
        next = v;
        break;
      }
    used[cur->first] = 1;
    edges.erase(cur);
    if (edges.empty()) break;
    cur = edges.find(next);
    if (cur == edges.end()) {
      cur = edges.begin();
      starts.push_back(order.size());
    }
  }
  starts.push_back(order.size());
  for (size_t k = 0; k + 1 < starts.size(); ++k)
    if (starts[k + 1] - starts[k] >= 3)
      S.polygons.emplace_back(order.begin() + (long)starts[k], order.begin() + (long)starts[k + 1]);
  return S;
}

// pcl::eigen33 (common/impl/eigen.hpp, the (matrix, evecs, evals) form): eigenvalues ascending
// (computeRoots of the scaled matrix) and all three eigenvectors (columns, evecs[3 * row + col])
// by cross products of the shifted rows, the weakest one re-derived from the other two
inline void eigen33_full(const double mat[9], double evecs[9], double evals[3]) {
  double scale = 0;
  for (int k = 0; k < 9; ++k) scale = std::max(scale, std::fabs(mat[k]));
  if (scale <= 2.2250738585072014e-308) scale = 1.0;
  double m[9];
  for (int k = 0; k < 9; ++k) m[k] = mat[k] / scale;
  compute_roots(m, evals);
  const double eps = 2.220446049250313e-16;
  auto cross = [](const double* a, const double* b, double* o) {
    o[0] = a[1] * b[2] - a[2] * b[1];
    o[1] = a[2] * b[0] - a[0] * b[2];
    o[2] = a[0] * b[1] - a[1] * b[0];
  };
  auto sqn = [](const double* v) { return v[0] * v[0] + (v[1] * v[1] + v[2] * v[2]); };
  auto setcol = [&](int c, const double* v) {
    for (int r = 0; r < 3; ++r) evecs[3 * r + c] = v[r];
  };
  auto col = [&](int c, double* v) {
    for (int r = 0; r < 3; ++r) v[r] = evecs[3 * r + c];
  };
  // the strongest cross product of the rows of (m - ev I), normalised; its squared length
  auto vec_for = [&](double ev, double* out) {
    double t[9];
    for (int k = 0; k < 9; ++k) t[k] = m[k];
    t[0] -= ev; t[4] -= ev; t[8] -= ev;
    double v1[3], v2[3], v3[3];
    cross(t + 0, t + 3, v1);
    cross(t + 0, t + 6, v2);
    cross(t + 3, t + 6, v3);
    const double l1 = sqn(v1), l2 = sqn(v2), l3 = sqn(v3);
    const double* v = v3;
    double l = l3;
    if (l1 >= l2 && l1 >= l3) { v = v1; l = l1; }
    else if (l2 >= l1 && l2 >= l3) { v = v2; l = l2; }
    const double sl = std::sqrt(l);
    for (int k = 0; k < 3; ++k) out[k] = v[k] / sl;
    return l;
  };
  // Eigen's unitOrthogonal for a 3-vector
  auto unit_orth = [](const double* v, double* o) {
    // (Eigen: x or y not much smaller than z, precision 1e-12 for double)
    if (!(std::fabs(v[0]) <= std::fabs(v[2]) * 1e-12) || !(std::fabs(v[1]) <= std::fabs(v[2]) * 1e-12)) {
      const double inv = 1.0 / std::sqrt(v[0] * v[0] + v[1] * v[1]);
      o[0] = -v[1] * inv; o[1] = v[0] * inv; o[2] = 0.0;
    } else {
      const double inv = 1.0 / std::sqrt(v[1] * v[1] + v[2] * v[2]);
      o[0] = 0.0; o[1] = -v[2] * inv; o[2] = v[1] * inv;
    }
  };
  auto normalized = [&](double* v) {
    const double l = std::sqrt(sqn(v));
    for (int k = 0; k < 3; ++k) v[k] /= l;
  };
  double a[3], b[3], c3[3];
  if (evals[2] - evals[0] <= eps) {
    for (int k = 0; k < 9; ++k) evecs[k] = (k % 4 == 0) ? 1.0 : 0.0;
  } else if (evals[1] - evals[0] <= eps) {
    vec_for(evals[2], a);
    setcol(2, a);
    unit_orth(a, b);
    setcol(1, b);
    cross(b, a, c3);
    setcol(0, c3);
  } else if (evals[2] - evals[1] <= eps) {
    vec_for(evals[0], a);
    setcol(0, a);
    unit_orth(a, b);
    setcol(1, b);
    cross(a, b, c3);
    setcol(2, c3);
  } else {
    double mmax[3];
    int min_el = 2, max_el = 2;
    mmax[2] = vec_for(evals[2], a);
    setcol(2, a);
    mmax[1] = vec_for(evals[1], a);
    setcol(1, a);
    if (mmax[1] > mmax[max_el]) max_el = 1;
    if (mmax[1] < mmax[min_el]) min_el = 1;
    mmax[0] = vec_for(evals[0], a);
    setcol(0, a);
    if (mmax[0] > mmax[max_el]) max_el = 0;
    if (mmax[0] < mmax[min_el]) min_el = 0;
    const int mid_el = 3 - min_el - max_el;
    double u[3], w[3];
    col((min_el + 1) % 3, u); col((min_el + 2) % 3, w);
    cross(u, w, a); normalized(a); setcol(min_el, a);
    col((mid_el + 1) % 3, u); col((mid_el + 2) % 3, w);
    cross(u, w, a); normalized(a); setcol(mid_el, a);
  }
  for (int k = 0; k < 3; ++k) evals[k] *= scale;
}

// ConcaveHull<PointXYZ>::reconstruct(output, polygons) on n points (xyz: 3 floats each, finite),
// dimension 2 (steps 1-6 above).  out_xyz: the alpha shape's points (3 floats each, in the order
// of S.av after the walk: out point k = polygon-walk position k); returns the shape
struct Hull2 {
  AlphaShape S;
  std::vector<float> pts;              // the output cloud (alpha shape, walk order), 3 per point
  std::vector<std::vector<int32_t>> polygons;  // indices into pts
  std::vector<int32_t> ids;            // output point -> input point
};

inline Hull2 concave_hull_2d(const float* xyz, int64_t n, double alpha) {
  Hull2 H;
  if (n < 3) return H;
  double c[3] = {0, 0, 0};
  for (int64_t i = 0; i < n; ++i)
    for (int k = 0; k < 3; ++k) c[k] += xyz[3 * i + k];
  for (int k = 0; k < 3; ++k) c[k] /= (double)n;
  double cov[9] = {0};
  for (int64_t i = 0; i < n; ++i) {
    const double d[3] = {xyz[3 * i] - c[0], xyz[3 * i + 1] - c[1], xyz[3 * i + 2] - c[2]};
    cov[4] += d[1] * d[1]; cov[5] += d[1] * d[2]; cov[8] += d[2] * d[2];
    cov[0] += d[0] * d[0]; cov[1] += d[0] * d[1]; cov[2] += d[0] * d[2];
  }
  cov[3] = cov[1]; cov[6] = cov[2]; cov[7] = cov[5];
  for (int k = 0; k < 9; ++k) cov[k] /= (double)n;
  double ev[9], el[3];
  eigen33_full(cov, ev, el);
  // transform1: row 0 = eigenvector of the largest eigenvalue, row 1 the middle, row 2 the
  // smallest (the plane's normal -> z)
  double T[9];
  for (int k = 0; k < 3; ++k) {
    T[0 * 3 + k] = ev[3 * k + 2];
    T[1 * 3 + k] = ev[3 * k + 1];
    T[2 * 3 + k] = ev[3 * k + 0];
  }
  const float cf[3] = {(float)c[0], (float)c[1], (float)c[2]};
  std::vector<double> xy(2 * (size_t)n);
  for (int64_t i = 0; i < n; ++i) {
    const float d[3] = {xyz[3 * i] - cf[0], xyz[3 * i + 1] - cf[1], xyz[3 * i + 2] - cf[2]};
    xy[2 * i] = (double)(float)(T[0] * d[0] + T[1] * d[1] + T[2] * d[2]);
    xy[2 * i + 1] = (double)(float)(T[3] * d[0] + T[4] * d[1] + T[5] * d[2]);
  }
  const Tri2 tri = Delaunay(xy.data(), (int)n).run();
  H.S = alpha_shape(xy.data(), tri, alpha);
  // the inverse transform (Eigen's 3 x 3 inverse by cofactors) and the centroid back
  const double det = T[0] * (T[4] * T[8] - T[5] * T[7]) - T[1] * (T[3] * T[8] - T[5] * T[6]) +
                     T[2] * (T[3] * T[7] - T[4] * T[6]);
  double I[9];
  I[0] = (T[4] * T[8] - T[5] * T[7]) / det; I[1] = (T[2] * T[7] - T[1] * T[8]) / det;
  I[2] = (T[1] * T[5] - T[2] * T[4]) / det; I[3] = (T[5] * T[6] - T[3] * T[8]) / det;
  I[4] = (T[0] * T[8] - T[2] * T[6]) / det; I[5] = (T[2] * T[3] - T[0] * T[5]) / det;
  I[6] = (T[3] * T[7] - T[4] * T[6]) / det; I[7] = (T[1] * T[6] - T[0] * T[7]) / det;
  I[8] = (T[0] * T[4] - T[1] * T[3]) / det;
  // output cloud in walk order (PCL's alpha_shape_sorted): the polygons are runs of it
  std::vector<int32_t> pos_of(H.S.av.size(), -1);
  for (const auto& poly : H.S.polygons) {
    std::vector<int32_t> pp;
    for (int32_t a : poly) {
      const int32_t pid = H.S.av[a];
      const float u = (float)xy[2 * pid], v = (float)xy[2 * pid + 1];
      for (int r = 0; r < 3; ++r) {
        const float tr = (float)(I[3 * r + 0] * u + I[3 * r + 1] * v + I[3 * r + 2] * 0.0);
        H.pts.push_back(tr - (float)(-c[r]));
      }
      pp.push_back((int32_t)H.ids.size());
      H.ids.push_back(pid);
    }
    H.polygons.push_back(std::move(pp));
  }
  return H;
}

}  // namespace alpha
}  // namespace dlg
