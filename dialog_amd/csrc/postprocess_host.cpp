// postprocess_host.cpp -- host driver of postProcessPlanes (Dialog/PlaneDetect.h:1454-1579):
// dlg_refit_planes, dlg_post_process_planes, dlg_cluster_filter (include/dialog_ransac.h).
//
// The refit (pcl::computePointNormal per plane, :1477-1498) is a sequential float sum per plane
// in list order, i.e. sequential by definition: it runs on host threads, one plane each.  The
// per-point work -- nearest-neighbour marking (:1518-1526), the point-in-polygon absorption
// (:1530-1556) and clusterFilt (:1569) -- runs on the device (postprocess.hip, normals.hip).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <exception>
#include <limits>
#include <thread>
#include <vector>

#include "driver.hpp"
#include "grid_host.hpp"
#include "normals.hpp"
#include "alpha_shape.hpp"
#include "postprocess.hpp"

namespace dlg {
namespace {

void check_records(const float* p, int64_t n, int64_t stride, const char* what) {
  if (n > 0 && !p) throw DlgError(DLG_ERR_INVALID, std::string(what) + " is null");
  if ((stride != 12 && stride < 16) || stride % 4)
    throw DlgError(DLG_ERR_INVALID, std::string(what) + " stride must be 12 or >= 16, multiple of 4");
}

void check_offsets(const int64_t* off, int np, const char* what) {
  if (!off) throw DlgError(DLG_ERR_INVALID, std::string(what) + " offsets are null");
  if (off[0] != 0) throw DlgError(DLG_ERR_INVALID, std::string(what) + " offsets must start at 0");
  for (int k = 0; k < np; ++k)
    if (off[k + 1] < off[k]) throw DlgError(DLG_ERR_INVALID, std::string(what) + " offsets decrease");
  if (off[np] > INT32_MAX / 2) throw DlgError(DLG_ERR_INVALID, std::string(what) + ": too many records");
}

void check_planes(const dlg_planes* P) {
  if (!P || P->n_planes < 0) throw DlgError(DLG_ERR_INVALID, "planes: null or negative count");
  if (P->n_planes == 0) return;
  if (!P->coeffs) throw DlgError(DLG_ERR_INVALID, "planes: coeffs are null");
  check_offsets(P->point_offsets, P->n_planes, "plane points");
  check_offsets(P->border_offsets, P->n_planes, "borders");
  check_records(P->points, P->point_offsets[P->n_planes], P->points_stride_bytes, "plane points");
  check_records(P->borders, P->border_offsets[P->n_planes], P->borders_stride_bytes, "borders");
}

// pcl::computePointNormal (features/normal_3d.h) over all points of one plane [PCL-1.8 ext]:
// computeMeanAndCovarianceMatrix (dense, float, list order) + solvePlaneParameters
void compute_point_normal(const float* pts, int64_t stride_f, int64_t n, float out[4]) {
  if (n < 3) {
    out[0] = out[1] = out[2] = out[3] = std::numeric_limits<float>::quiet_NaN();
    return;
  }
  float a[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
  for (int64_t i = 0; i < n; ++i) {
    const float* p = pts + i * stride_f;
    const float x = p[0], y = p[1], z = p[2];
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
  out[0] = v[0]; out[1] = v[1]; out[2] = v[2];
  // plane_parameters[3] = -1 * plane_parameters.dot(centroid): Vector4f SSE predux order
  out[3] = -1.0f * ((v[0] * a[6] + v[2] * a[8]) + (v[1] * a[7] + 0.0f * 1.0f));
}

void refit_planes(const dlg_planes* P, float* out) {
  const int np = P->n_planes;
  if (np == 0) return;
  if (!out) throw DlgError(DLG_ERR_INVALID, "coeffs_out is null");
  const int64_t sf = P->points_stride_bytes / 4;
  auto one = [&](int k) {
    float prm[4];
    const int64_t b = P->point_offsets[k], e = P->point_offsets[k + 1];
    compute_point_normal(P->points + b * sf, sf, e - b, prm);
    const float* v = P->coeffs + 4 * k;
    // Vector4f(v0, v1, v2, 0).dot(param) < 0 -> param = -1.0f * param
    const float d = (v[0] * prm[0] + v[2] * prm[2]) + (v[1] * prm[1] + 0.0f * prm[3]);
    if (d < 0.0f)
      for (float& x : prm) x = -1.0f * x;
    std::memcpy(out + 4 * k, prm, sizeof(prm));
  };
  const int64_t total = P->point_offsets[np];
  const int nt = (int)std::min<int64_t>(
      {(int64_t)np, (int64_t)std::max(1u, std::thread::hardware_concurrency()), 16,
       1 + total / 200000});
  if (nt <= 1) {
    for (int k = 0; k < np; ++k) one(k);
    return;
  }
  std::vector<std::thread> th;
  for (int t = 0; t < nt; ++t)
    th.emplace_back([&, t] {
      for (int k = t; k < np; k += nt) one(k);
    });
  for (auto& x : th) x.join();
}

// device copy of strided host records -> (X, Y, Z)
void upload_records(dlg_ctx* c, const float* rec, int64_t n, int64_t stride_bytes, float* X,
                    float* Y, float* Z) {
  if (n <= 0) return;
  NormalsWork& w = c->nw;
  const size_t bytes = (size_t)n * (size_t)stride_bytes;
  w.raw.ensure(bytes);
  HIPCHK(hipMemcpyAsync(w.raw.p, rec, bytes, hipMemcpyHostToDevice, c->stream));
  launch_deinterleave(reinterpret_cast<const float*>(w.raw.p), (int)n, stride_bytes / 4, X, Y, Z,
                      c->stream);
}

// clusterFilt over (X, Y, Z)[0..n) on the device: keep flags in input order -> pw.keep
void cluster_keep(dlg_ctx* c, const float* X, const float* Y, const float* Z, int n,
                  float radius, int32_t t_cluster_num) {
  PostWork& pw = c->pw;
  pw.keep.ensure(n);
  if (n == 0) return;
  const BBox b = bbox_of(c, X, Y, Z, n);
  const double r = (double)radius;
  const GridDesc G = make_grid(b, r > 0.0 ? r : 1.0);
  GridBufs B;
  build_grid(c, n, G, 0, &B, X, Y, Z);
  const float r2 = (float)(r * r);  // KdTreeFLANN::radiusSearch: (float)(radius * radius)
  pw.parent.ensure(n);
  pw.csize.ensure(n);
  launch_cc(G, B, n, r2, (int64_t)t_cluster_num, pw.parent.p, pw.csize.p, pw.keep.p, c->stream);
  HIPCHK(hipGetLastError());
}

uint32_t select_count(dlg_ctx* c, const uint8_t* flags, int n, int32_t* out) {
  NormalsWork& w = c->nw;
  w.sort_tmp.ensure(select_tmp_bytes(n));
  w.counters.ensure(8);
  w.h_cnt.ensure(8);
  HIPCHK(select_flagged(w.sort_tmp.p, w.sort_tmp.cap, flags, n, out, w.counters.p, c->stream));
  HIPCHK(hipMemcpyAsync(w.h_cnt.p, w.counters.p, 4, hipMemcpyDeviceToHost, c->stream));
  sync(c);
  return w.h_cnt.p[0];
}

void check_radius(float radius) {
  if (!(radius >= 0.0f)) throw DlgError(DLG_ERR_INVALID, "radius must be >= 0");
}

void cluster_filter(dlg_ctx* c, const dlg_points* pts, float radius, int32_t t_cluster_num,
                    int32_t* kept_ids, int64_t cap, int64_t* n_kept) {
  check_points(pts);
  check_radius(radius);
  const int n = (int)pts->n;
  if (n == 0) return;
  NormalsWork& w = c->nw;
  PostWork& pw = c->pw;
  w.qx.ensure(n); w.qy.ensure(n); w.qz.ensure(n);
  upload_records(c, pts->xyz, n, pts->stride_bytes, w.qx.p, w.qy.p, w.qz.p);
  cluster_keep(c, w.qx.p, w.qy.p, w.qz.p, n, radius, t_cluster_num);
  pw.sel.ensure(n);
  const int64_t k = select_count(c, pw.keep.p, n, pw.sel.p);
  *n_kept = k;
  if (k > cap) throw DlgError(DLG_ERR_CAPACITY, "kept_ids too small: need " + std::to_string(k));
  if (k > 0) {
    if (!kept_ids) throw DlgError(DLG_ERR_INVALID, "kept_ids is null");
    HIPCHK(hipMemcpyAsync(kept_ids, pw.sel.p, 4 * (size_t)k, hipMemcpyDeviceToHost, c->stream));
    sync(c);
  }
}

// isPointInPoly set-up of one plane: the ten ray directions (srand(seed), rand() % border size)
void plane_rays(const float* border, int64_t nb, int64_t sf, const float coeff[4], uint32_t seed,
                float4* rays) {
  uint32_t st = seed;
  const V3 pn{coeff[0], coeff[1], coeff[2]};
  for (int k = 0; k < kPipRays; ++k) {
    const int64_t idx = (int64_t)((uint64_t)msvc_rand(st) % (uint64_t)nb);
    const float* s = border + idx * sf;
    const float* e = border + (idx == nb - 1 ? 0 : idx + 1) * sf;
    const V3 dir = v3_normalized(v3_sub(V3{e[0], e[1], e[2]}, V3{s[0], s[1], s[2]}));
    const V3 dp = v3_normalized(v3_cross(dir, pn));
    rays[k] = make_float4(dp.x, dp.y, dp.z, 0.0f);
  }
}

void plane_edges(const float* border, int64_t nb, int64_t sf, PipEdge* out) {
  for (int64_t j = 0; j < nb; ++j) {
    const float* a = border + j * sf;
    const float* b = border + (j == nb - 1 ? 0 : j + 1) * sf;
    const V3 pa{a[0], a[1], a[2]}, pb{b[0], b[1], b[2]};
    const V3 nab = v3_normalized(v3_sub(pb, pa));
    out[j].a_dab = make_float4(pa.x, pa.y, pa.z, dist_p2p(pa, pb));
    out[j].b = make_float4(pb.x, pb.y, pb.z,
                           (std::fabs(pa.x) + std::fabs(pa.y)) + std::fabs(pa.z));
    out[j].nab = make_float4(nab.x, nab.y, nab.z, 0.0f);
  }
}

bool finite4(const float* c) {
  return std::isfinite(c[0]) && std::isfinite(c[1]) && std::isfinite(c[2]) && std::isfinite(c[3]);
}

// the nearest cloud point of every plane point (KdTreeFLANN nearestKSearch k = 1, ties -> lowest
// index; PlaneDetect.h:1518-1526) -> processed.  Plane points that are cloud points (the usual
// case: points_set holds copies) are found in an exact-coordinate table; the others take the
// grid hierarchy search.  Cloud in nw.x/y/z, plane points in nw.qx/qy/qz.
void mark_nearest(dlg_ctx* c, int n, const BBox& b, int m) {
  NormalsWork& w = c->nw;
  PostWork& pw = c->pw;
  uint32_t tcap = 1024;
  while (tcap < 2u * (uint32_t)n && tcap < (1u << 31)) tcap <<= 1;
  pw.table.ensure(tcap);
  pw.rest.ensure(m);
  w.nn.ensure(m);
  w.counters.ensure(8);
  w.h_cnt.ensure(8);
  HIPCHK(hipMemsetAsync(pw.table.p, 0xff, (size_t)tcap * 4, c->stream));
  HIPCHK(hipMemsetAsync(w.counters.p, 0, 4, c->stream));
  launch_xyz_insert(w.x.p, w.y.p, w.z.p, n, pw.table.p, tcap - 1, c->stream);
  launch_xyz_lookup(w.qx.p, w.qy.p, w.qz.p, m, pw.table.p, tcap - 1, w.x.p, w.y.p, w.z.p, w.nn.p,
                    pw.rest.p, w.counters.p, c->stream);
  HIPCHK(hipMemcpyAsync(w.h_cnt.p, w.counters.p, 4, hipMemcpyDeviceToHost, c->stream));
  sync(c);
  int nq = (int)w.h_cnt.p[0];
  if (nq > 0) {
    const KnnLevels L = build_hierarchy(c, n, b, 1);
    w.queue.ensure(m);
    w.cand.ensure(m);
    int32_t* qin = pw.rest.p;
    int32_t* qout = w.queue.p;
    for (int l = 0; l < L.levels && nq > 0; ++l) {
      HIPCHK(hipMemsetAsync(w.counters.p, 0, 4, c->stream));
      launch_nn1(L, l, qin, nq, w.qx.p, w.qy.p, w.qz.p, w.nn.p, qout, w.counters.p, c->stream);
      if (l == L.levels - 1) break;
      HIPCHK(hipMemcpyAsync(w.h_cnt.p, w.counters.p, 4, hipMemcpyDeviceToHost, c->stream));
      sync(c);
      nq = (int)w.h_cnt.p[0];
      qin = qout;
      qout = qout == w.queue.p ? w.cand.p : w.queue.p;
    }
  }
  launch_mark_nn(w.nn.p, m, pw.processed.p, c->stream);
  HIPCHK(hipGetLastError());
}

// the refit runs on host threads while the device does the nearest-neighbour marking
struct RefitJob {
  std::thread th;
  std::exception_ptr err;
  ~RefitJob() {
    if (th.joinable()) th.join();
  }
  void wait() {
    if (th.joinable()) th.join();
    if (err) std::rethrow_exception(err);
  }
};

void post_process(dlg_ctx* c, const dlg_points* cloud, const dlg_planes* P,
                  const dlg_postprocess_params* prm, float* coeffs_out, int64_t* abs_off,
                  int32_t* abs_ids, int64_t abs_cap, int32_t* rem_ids, int64_t rem_cap,
                  int64_t* n_rem) {
  check_points(cloud);
  check_planes(P);
  if (!prm) throw DlgError(DLG_ERR_INVALID, "params are null");
  check_radius(prm->radius_local);
  if (!abs_off || !n_rem) throw DlgError(DLG_ERR_INVALID, "absorbed_offsets / n_remaining are null");
  const int np = P->n_planes;
  if (np > 0 && !coeffs_out) throw DlgError(DLG_ERR_INVALID, "coeffs_out is null");
  const int start = std::max(0, prm->plane_start_index);
  for (int k = start; k < np; ++k)
    if (P->border_offsets[k + 1] == P->border_offsets[k])
      throw DlgError(DLG_ERR_INVALID, "plane " + std::to_string(k) + " has an empty border");
  const int n = (int)cloud->n;
  if ((int64_t)n * std::max(np - start, 0) > (int64_t)INT32_MAX)
    throw DlgError(DLG_ERR_INVALID, "points x absorbing planes exceeds 2^31");
  for (int k = 0; k <= np; ++k) abs_off[k] = 0;
  *n_rem = 0;
  RefitJob refit;
  refit.th = std::thread([&] {
    try {
      refit_planes(P, coeffs_out);
    } catch (...) {
      refit.err = std::current_exception();
    }
  });
  if (n == 0) {
    refit.wait();
    return;
  }
  NormalsWork& w = c->nw;
  PostWork& pw = c->pw;

  // (1) isProcessed from the plane points' nearest cloud points (:1518-1526)
  const BBox b = upload_points(c, cloud);  // nw.x/y/z
  pw.processed.ensure(n);
  HIPCHK(hipMemsetAsync(pw.processed.p, 0, n, c->stream));
  const int m = np > 0 ? (int)P->point_offsets[np] : 0;
  if (m > 0) {
    w.qx.ensure(m); w.qy.ensure(m); w.qz.ensure(m);
    upload_records(c, P->points, m, P->points_stride_bytes, w.qx.p, w.qy.p, w.qz.p);
    mark_nearest(c, n, b, m);
  }
  refit.wait();

  // (2) absorption into planes [start, np) (:1530-1556)
  std::vector<int> act;  // participating planes; a NaN plane accepts nothing (every test is NaN)
  for (int k = start; k < np; ++k)
    if (finite4(coeffs_out + 4 * k)) act.push_back(k);
  const int na = (int)act.size();
  std::vector<int64_t> abs_cnt_h(np, 0);
  int64_t abs_total = 0;
  if (na > 0) {
    const int64_t bsf = P->borders_stride_bytes / 4;
    std::vector<float4> h_planes(na), h_rays((size_t)na * kPipRays);
    std::vector<int64_t> h_eoff(na + 1, 0);
    for (int a = 0; a < na; ++a) {
      const int k = act[a];
      h_eoff[a + 1] = h_eoff[a] + (P->border_offsets[k + 1] - P->border_offsets[k]);
    }
    std::vector<PipEdge> h_edges(h_eoff[na]);
    for (int a = 0; a < na; ++a) {
      const int k = act[a];
      const float* cf = coeffs_out + 4 * k;
      h_planes[a] = make_float4(cf[0], cf[1], cf[2], cf[3]);
      const float* bor = P->borders + P->border_offsets[k] * bsf;
      const int64_t nb = P->border_offsets[k + 1] - P->border_offsets[k];
      plane_rays(bor, nb, bsf, cf, prm->rand_seed, h_rays.data() + (size_t)a * kPipRays);
      plane_edges(bor, nb, bsf, h_edges.data() + h_eoff[a]);
    }
    pw.planes.ensure(na);
    pw.rays.ensure((size_t)na * kPipRays);
    pw.edges.ensure(h_edges.size());
    pw.edge_off.ensure(na + 1);
    pw.offs.ensure(na + 1);
    pw.abs_cnt.ensure(na);
    const size_t nbk = (size_t)na * pip_blocks(n);
    pw.bcnt.ensure(nbk);
    pw.boff.ensure(nbk);
    w.sort_tmp.ensure(pip_scan_tmp_bytes(nbk));
    HIPCHK(hipMemcpyAsync(pw.planes.p, h_planes.data(), na * sizeof(float4), hipMemcpyHostToDevice, c->stream));
    HIPCHK(hipMemcpyAsync(pw.rays.p, h_rays.data(), h_rays.size() * sizeof(float4), hipMemcpyHostToDevice, c->stream));
    HIPCHK(hipMemcpyAsync(pw.edges.p, h_edges.data(), h_edges.size() * sizeof(PipEdge), hipMemcpyHostToDevice, c->stream));
    HIPCHK(hipMemcpyAsync(pw.edge_off.p, h_eoff.data(), (na + 1) * sizeof(int64_t), hipMemcpyHostToDevice, c->stream));
    HIPCHK(launch_pip_candidates(w.x.p, w.y.p, w.z.p, n, pw.processed.p, pw.planes.p, na,
                                 prm->t_dist_point_plane, pw.bcnt.p, pw.boff.p, w.sort_tmp.p,
                                 w.sort_tmp.cap, nullptr, pw.offs.p, c->stream));
    std::vector<uint32_t> offs(na + 1);
    HIPCHK(hipMemcpyAsync(offs.data(), pw.offs.p, (na + 1) * 4, hipMemcpyDeviceToHost, c->stream));
    sync(c);
    const uint32_t total = offs[na];
    int max_cnt = 0;
    for (int a = 0; a < na; ++a) max_cnt = std::max(max_cnt, (int)(offs[a + 1] - offs[a]));
    if (total > 0) {
      pw.cand.ensure(total);
      pw.cand2.ensure(total);
      pw.mask.ensure(total);
      HIPCHK(hipMemsetAsync(pw.mask.p, 0, (size_t)total * 4, c->stream));
      HIPCHK(launch_pip_candidates(w.x.p, w.y.p, w.z.p, n, pw.processed.p, pw.planes.p, na,
                                   prm->t_dist_point_plane, pw.bcnt.p, pw.boff.p, nullptr, 0,
                                   pw.cand2.p, pw.offs.p, c->stream));
      {  // spatial order within each plane (Morton code over the cloud's bounding box)
        float ext = 0.0f;
        for (int k = 0; k < 3; ++k) ext = std::max(ext, b.hi[k] - b.lo[k]);
        const float4 ls = make_float4(b.lo[0], b.lo[1], b.lo[2], ext > 0.0f ? 16383.0f / ext : 0.0f);
        w.keys64.ensure(total);
        w.keys_alt.ensure(total);
        w.sort_tmp.ensure(pip_sort_tmp_bytes((int)total));
        HIPCHK(launch_pip_sort(pw.cand2.p, (int)total, pw.offs.p, na, max_cnt, w.x.p, w.y.p, w.z.p,
                               ls, reinterpret_cast<uint64_t*>(w.keys64.p),
                               reinterpret_cast<uint64_t*>(w.keys_alt.p), pw.cand.p, w.sort_tmp.p,
                               w.sort_tmp.cap, c->stream));
      }
      // tasks: 256 candidates x a run of edges; edges split so the launch fills the chip
      int64_t cblocks = 0;
      for (int a = 0; a < na; ++a) cblocks += (offs[a + 1] - offs[a] + 255) / 256;
      const int64_t want = 8LL * 256;
      const int64_t split = std::max<int64_t>(1, (want + cblocks - 1) / std::max<int64_t>(cblocks, 1));
      std::vector<PipTask> tasks;
      for (int a = 0; a < na; ++a) {
        const int64_t nb = h_eoff[a + 1] - h_eoff[a];
        const int64_t chunk = std::max<int64_t>(16, (nb + split - 1) / split);
        const uint32_t cnt = offs[a + 1] - offs[a];
        for (uint32_t cb = 0; cb < cnt; cb += 256)
          for (int64_t e = 0; e < nb; e += chunk)
            tasks.push_back(PipTask{a, (int32_t)(offs[a] + cb), (int32_t)std::min<uint32_t>(256, cnt - cb),
                                    (int32_t)e, (int32_t)std::min(nb, e + chunk)});
      }
      pw.tasks.ensure(tasks.size());
      HIPCHK(hipMemcpyAsync(pw.tasks.p, tasks.data(), tasks.size() * sizeof(PipTask), hipMemcpyHostToDevice, c->stream));
      launch_pip_test(pw.tasks.p, (int)tasks.size(), pw.cand.p, w.x.p, w.y.p, w.z.p, pw.planes.p,
                      pw.rays.p, pw.edges.p, pw.edge_off.p, pw.mask.p, c->stream);
      HIPCHK(hipGetLastError());
      pw.absorbed.ensure((size_t)na * n);
      HIPCHK(hipMemsetAsync(pw.absorbed.p, 0, (size_t)na * n, c->stream));
      HIPCHK(hipMemsetAsync(pw.abs_cnt.p, 0, na * 4, c->stream));
      launch_pip_mark(pw.cand.p, pw.mask.p, pw.offs.p, na, max_cnt, n, pw.absorbed.p,
                      pw.processed.p, pw.abs_cnt.p, c->stream);
      HIPCHK(hipGetLastError());
      std::vector<uint32_t> ac(na);
      HIPCHK(hipMemcpyAsync(ac.data(), pw.abs_cnt.p, na * 4, hipMemcpyDeviceToHost, c->stream));
      sync(c);
      for (int a = 0; a < na; ++a) {
        abs_cnt_h[act[a]] = ac[a];
        abs_total += ac[a];
      }
    }
  }
  for (int k = 0; k < np; ++k) abs_off[k + 1] = abs_off[k] + abs_cnt_h[k];
  // absorbed ids per plane: ascending (select over the plane's flags)
  if (abs_total > 0) {
    pw.ids.ensure(abs_total);
    for (int a = 0; a < na; ++a) {
      const int k = act[a];
      if (abs_cnt_h[k] == 0) continue;
      (void)select_count(c, pw.absorbed.p + (size_t)a * n, n, pw.ids.p + abs_off[k]);
    }
  }

  // (3) the rest -> clusterFilt (:1559-1569)
  pw.flags.ensure(n);
  pw.rids.ensure(n);
  launch_invert_flags(pw.processed.p, n, pw.flags.p, c->stream);
  const int nr = (int)select_count(c, pw.flags.p, n, pw.rids.p);
  int64_t kept = 0;
  if (nr > 0) {
    w.qx.ensure(nr); w.qy.ensure(nr); w.qz.ensure(nr);
    launch_gather3(pw.rids.p, nr, w.x.p, w.y.p, w.z.p, w.qx.p, w.qy.p, w.qz.p, c->stream);
    cluster_keep(c, w.qx.p, w.qy.p, w.qz.p, nr, prm->radius_local, prm->t_cluster_num);
    pw.sel.ensure(nr);
    pw.out.ensure(nr);
    kept = select_count(c, pw.keep.p, nr, pw.sel.p);
    launch_gather_ids(pw.sel.p, (int)kept, pw.rids.p, pw.out.p, c->stream);
  }
  *n_rem = kept;
  if (abs_total > abs_cap)
    throw DlgError(DLG_ERR_CAPACITY, "absorbed_ids too small: need " + std::to_string(abs_total));
  if (kept > rem_cap)
    throw DlgError(DLG_ERR_CAPACITY, "remaining_ids too small: need " + std::to_string(kept));
  if (abs_total > 0) {
    if (!abs_ids) throw DlgError(DLG_ERR_INVALID, "absorbed_ids is null");
    HIPCHK(hipMemcpyAsync(abs_ids, pw.ids.p, 4 * (size_t)abs_total, hipMemcpyDeviceToHost, c->stream));
  }
  if (kept > 0) {
    if (!rem_ids) throw DlgError(DLG_ERR_INVALID, "remaining_ids is null");
    HIPCHK(hipMemcpyAsync(rem_ids, pw.out.p, 4 * (size_t)kept, hipMemcpyDeviceToHost, c->stream));
  }
  sync(c);
}

// polyPointCloud (PlaneDetect.h:1376-1440) for one plane; see dlg_plane_border
int64_t plane_border(const float* pts, int64_t stride_f, int64_t n, const float pn[3], float alpha,
                     float* out, int64_t out_stride_f, int64_t cap, int64_t* n_needed) {
  if (!(alpha > 0.0f) || !std::isfinite(alpha)) throw DlgError(DLG_ERR_INVALID, "alpha must be > 0");
  float prm[4];
  compute_point_normal(pts, stride_f, n, prm);  // (NaN with < 3 points)
  if (!(prm[0] == prm[0])) return 0;
  // projPoint2Plane (PlaneDetect.h:1437-1444): lambda = 2.0 * (float dot + d), in double, stored
  // as float; dest = src - lambda / 2.0 * param (double), stored as float.  (Non-finite points
  // are left out: the reference's clouds have none after preProcess.)
  std::vector<float> q;
  q.reserve(3 * (size_t)n);
  for (int64_t i = 0; i < n; ++i) {
    const float* p = pts + i * stride_f;
    const float lambda =
        (float)(2.0 * (double)(prm[0] * p[0] + prm[1] * p[1] + prm[2] * p[2] + prm[3]));
    float d[3];
    for (int k = 0; k < 3; ++k) d[k] = (float)((double)p[k] - lambda / 2.0 * prm[k]);
    if (std::isfinite(d[0]) && std::isfinite(d[1]) && std::isfinite(d[2])) q.insert(q.end(), d, d + 3);
  }
  const int64_t m = (int64_t)q.size() / 3;
  if (m > INT32_MAX / 4) throw DlgError(DLG_ERR_INVALID, "too many plane points");
  // pcl::ConcaveHull (setAlpha(alpha_poly), reconstruct(output, polygons)): alpha_shape.hpp
  const alpha::Hull2 H = alpha::concave_hull_2d(q.data(), m, (double)alpha);
  if (H.polygons.empty()) return 0;
  // the reference takes polygons[0]; which polygon qhull's facet order puts first is not
  // reproducible (alpha_shape.hpp), so the border is the polygon enclosing the largest area --
  // polygons[0] whenever the plane's alpha shape is one simple polygon
  size_t best = 0;
  double best_a = -1.0;
  for (size_t k = 0; k < H.polygons.size(); ++k) {
    const auto& pg = H.polygons[k];
    double ax = 0, ay = 0, az = 0;
    for (size_t j = 0; j < pg.size(); ++j) {
      const float* a0 = &H.pts[3 * (size_t)pg[j]];
      const float* a1 = &H.pts[3 * (size_t)pg[(j + 1) % pg.size()]];
      ax += (double)a0[1] * a1[2] - (double)a0[2] * a1[1];
      ay += (double)a0[2] * a1[0] - (double)a0[0] * a1[2];
      az += (double)a0[0] * a1[1] - (double)a0[1] * a1[0];
    }
    const double ar = std::sqrt(ax * ax + ay * ay + az * az);
    if (ar > best_a) {
      best_a = ar;
      best = k;
    }
  }
  std::vector<int32_t> bi = H.polygons[best];
  const int64_t nb = (int64_t)bi.size();
  *n_needed = nb;
  if (nb > cap) throw DlgError(DLG_ERR_CAPACITY, "border buffer too small: need " + std::to_string(nb));
  // the walk's start is qhull's (unpinned); start one vertex before an extreme vertex in the
  // plane, a convex one: the reference orients by the turn at the second vertex, whose sign is
  // then the polygon's orientation (from a reflex second vertex its rule would reverse a
  // correctly oriented border)
  {
    double u[3] = {0, 0, 0};
    const int ax = std::fabs(pn[0]) <= std::fabs(pn[1]) && std::fabs(pn[0]) <= std::fabs(pn[2]) ? 0
                   : std::fabs(pn[1]) <= std::fabs(pn[2]) ? 1 : 2;
    u[ax] = 1.0;
    const double nn = (double)pn[0] * pn[0] + (double)pn[1] * pn[1] + (double)pn[2] * pn[2];
    const double dt = ((double)pn[0] * u[0] + (double)pn[1] * u[1] + (double)pn[2] * u[2]) / nn;
    for (int k = 0; k < 3; ++k) u[k] -= dt * pn[k];
    // ties along u (a straight edge perpendicular to u) broken by the smallest coordinate along
    // w = n x u: the lexicographic minimum is always a strictly convex vertex (never a collinear
    // middle one, whose turn the reference's rule cannot read)
    const double w[3] = {(double)pn[1] * u[2] - (double)pn[2] * u[1],
                         (double)pn[2] * u[0] - (double)pn[0] * u[2],
                         (double)pn[0] * u[1] - (double)pn[1] * u[0]};
    int64_t mk = 0;
    double mv = INFINITY, mw = INFINITY;
    for (int64_t k = 0; k < nb; ++k) {
      const float* a = &H.pts[3 * (size_t)bi[k]];
      const double v = a[0] * u[0] + a[1] * u[1] + a[2] * u[2];
      const double vw = a[0] * w[0] + a[1] * w[1] + a[2] * w[2];
      if (v < mv || (v == mv && vw < mw)) { mv = v; mw = vw; mk = k; }
    }
    std::rotate(bi.begin(), bi.begin() + (mk + nb - 1) % nb, bi.end());
  }
  // the reference's orientation rule (PlaneDetect.h:1415-1434): v01, v12 normalized (float),
  // v_dir = v01 x v12 normalized; the order reversed when v_dir . pn < 0
  auto P = [&](int64_t k) { return &H.pts[3 * (size_t)bi[k]]; };
  float v01[3], v12[3];
  for (int k = 0; k < 3; ++k) {
    v01[k] = P(1)[k] - P(0)[k];
    v12[k] = P(2)[k] - P(1)[k];
  }
  auto nrm = [](float* w) {
    const float l = std::sqrt((w[0] * w[0] + w[1] * w[1]) + w[2] * w[2]);
    for (int k = 0; k < 3; ++k) w[k] = w[k] / l;
  };
  nrm(v01);
  nrm(v12);
  float vd[3] = {v01[1] * v12[2] - v01[2] * v12[1], v01[2] * v12[0] - v01[0] * v12[2],
                 v01[0] * v12[1] - v01[1] * v12[0]};
  nrm(vd);
  if ((vd[0] * pn[0] + vd[1] * pn[1]) + vd[2] * pn[2] < 0.0f) {
    std::reverse(bi.begin(), bi.end());
    // (the convex vertex second again: the border passes the reference's own test)
    std::rotate(bi.begin(), bi.begin() + (nb - 3) % nb, bi.end());
  }
  for (int64_t k = 0; k < nb; ++k)
    for (int j = 0; j < 3; ++j) out[k * out_stride_f + j] = H.pts[3 * (size_t)bi[k] + j];
  return nb;
}

}  // namespace
}  // namespace dlg

extern "C" {

dlg_status dlg_plane_border(const dlg_points* plane_pts, const float pn[3], float alpha,
                            float* border_out, int64_t out_stride_bytes, int64_t cap,
                            int64_t* n_out) {
  if (!plane_pts || !pn || !n_out) return DLG_ERR_INVALID;
  *n_out = 0;
  return guarded(nullptr, [&] {
    check_records(plane_pts->xyz, plane_pts->n, plane_pts->stride_bytes, "plane points");
    if (out_stride_bytes < 12 || out_stride_bytes % 4)
      throw DlgError(DLG_ERR_INVALID, "out_stride_bytes must be >= 12 and a multiple of 4");
    if (cap > 0 && !border_out) throw DlgError(DLG_ERR_INVALID, "border_out is null");
    *n_out = plane_border(plane_pts->xyz, plane_pts->stride_bytes / 4, plane_pts->n, pn, alpha,
                          border_out, out_stride_bytes / 4, cap, n_out);
  });
}

dlg_status dlg_refit_planes(const dlg_planes* planes, float* coeffs_out) {
  return guarded(nullptr, [&] {
    check_planes(planes);
    refit_planes(planes, coeffs_out);
  });
}

dlg_status dlg_post_process_planes(dlg_ctx* ctx, const dlg_points* cloud, const dlg_planes* planes,
                                   const dlg_postprocess_params* params, float* coeffs_out,
                                   int64_t* absorbed_offsets, int32_t* absorbed_ids,
                                   int64_t absorbed_cap, int32_t* remaining_ids,
                                   int64_t remaining_cap, int64_t* n_remaining) {
  if (!ctx) return DLG_ERR_INVALID;
  return guarded(ctx, [&] {
    post_process(ctx, cloud, planes, params, coeffs_out, absorbed_offsets, absorbed_ids,
                 absorbed_cap, remaining_ids, remaining_cap, n_remaining);
  });
}

dlg_status dlg_cluster_filter(dlg_ctx* ctx, const dlg_points* pts, float radius,
                              int32_t t_cluster_num, int32_t* kept_ids, int64_t cap,
                              int64_t* n_kept) {
  if (!ctx) return DLG_ERR_INVALID;
  return guarded(ctx, [&] {
    if (!n_kept) throw DlgError(DLG_ERR_INVALID, "n_kept is null");
    *n_kept = 0;
    cluster_filter(ctx, pts, radius, t_cluster_num, kept_ids, cap, n_kept);
  });
}

}  // extern "C"
