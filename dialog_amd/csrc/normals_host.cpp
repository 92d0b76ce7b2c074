// normals_host.cpp -- host driver of the normals path: dlg_estimate_normals and
// dlg_regulate_normals (include/dialog_ransac.h; Dialog/PlaneDetect.h:515-665).
//
// Both calls take host buffers (the reference keeps source_cloud / source_normal on the host,
// PlaneDetect.h:104-107): the strided records are uploaded raw and de-interleaved on the device,
// a uniform grid is built (normals.hip), the kernels run, and the results are packed into the
// caller's record layout on the device before one D2H copy.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>
#include <cstring>
#include <limits>
#include <vector>

#include "driver.hpp"
#include "grid_host.hpp"
#include "normals.hpp"

namespace dlg {

BBox bbox_of(dlg_ctx* c, const float* X, const float* Y, const float* Z, int n) {
  NormalsWork& w = c->nw;
  const int nb = bbox_blocks(n);
  w.partial.ensure(6 * nb);
  launch_bbox(X, Y, Z, n, w.partial.p, c->stream);
  std::vector<float> part(6 * nb);
  HIPCHK(hipMemcpyAsync(part.data(), w.partial.p, part.size() * 4, hipMemcpyDeviceToHost, c->stream));
  sync(c);
  BBox b;
  for (int k = 0; k < 3; ++k) {
    b.lo[k] = INFINITY;
    b.hi[k] = -INFINITY;
  }
  for (int i = 0; i < nb; ++i)
    for (int k = 0; k < 3; ++k) {
      b.lo[k] = std::fmin(b.lo[k], part[6 * i + k]);
      b.hi[k] = std::fmax(b.hi[k], part[6 * i + 3 + k]);
    }
  b.any = b.lo[0] <= b.hi[0];
  return b;
}

// points -> device SoA (nw.x/y/z) + bounding box of the finite points
BBox upload_points(dlg_ctx* c, const dlg_points* pts) {
  NormalsWork& w = c->nw;
  const int n = (int)pts->n;
  const size_t bytes = (size_t)pts->n * (size_t)pts->stride_bytes;
  w.raw.ensure(bytes);
  w.x.ensure(n); w.y.ensure(n); w.z.ensure(n);
  HIPCHK(hipMemcpyAsync(w.raw.p, pts->xyz, bytes, hipMemcpyHostToDevice, c->stream));
  launch_deinterleave(reinterpret_cast<const float*>(w.raw.p), n, pts->stride_bytes / 4, w.x.p,
                      w.y.p, w.z.p, c->stream);
  return bbox_of(c, w.x.p, w.y.p, w.z.p, n);
}

// grid with cell edge `cell` (grown until the key space fits 2^30 cells)
GridDesc make_grid(const BBox& b, double cell) {
  GridDesc G;
  for (;;) {
    double tot = 1.0;
    for (int k = 0; k < 3; ++k) {
      const double ext = b.any ? (double)b.hi[k] - (double)b.lo[k] : 0.0;
      const double gk = std::floor(ext / cell) + 1.0;
      G.g[k] = (int)std::min(gk, 1e9);
      tot *= gk;
    }
    if (tot <= (double)(1u << 30)) break;
    cell *= 1.25;
  }
  for (int k = 0; k < 3; ++k) G.lo[k] = b.any ? b.lo[k] : 0.0f;
  // cell_of() computes floor((v - lo) * inv_cell) in float; shrinking inv_cell by 1e-3 keeps the
  // effective cell edge >= `cell` despite the rounding of (v - lo) and of the product (<= 1024
  // cells per axis at float precision: ~1e-4 cell), so points within r stay in adjacent cells
  G.inv_cell = (float)((1.0 / cell) * (1.0 - 1e-3));
  G.cell = (float)(cell * (1.0 - 1e-6));  // guaranteed coverage radius of the 27 cells
  G.ncells = (uint32_t)((uint64_t)G.g[0] * G.g[1] * G.g[2]);
  int bits = 1;
  while (bits < 32 && ((uint64_t)1 << bits) <= (uint64_t)G.ncells) ++bits;
  G.key_bits = bits;
  return G;
}

// builds grid level `lv` over (X, Y, Z) (default nw.x/y/z); returns the number of occupied cells
// (and the point-weighted mean occupancy sum(occ^2) / n in *pw_occ)
// (clouds from this size gather their sorted coordinates from packed records)
constexpr int kGridRecMin = 1 << 16;
uint32_t build_grid(dlg_ctx* c, int n, const GridDesc& G, int lv, GridBufs* B, const float* X,
                    const float* Y, const float* Z, double* pw_occ) {
  NormalsWork& w = c->nw;
  GridLevelBufs& L = w.lv[lv];
  w.keys_in.ensure(n); w.keys_out.ensure(n); w.idx_in.ensure(n);
  L.idx.ensure(n); L.sx.ensure(n); L.sy.ensure(n); L.sz.ensure(n);
  const uint64_t occ_max = std::min<uint64_t>((uint64_t)n, G.ncells);
  uint32_t tcap = 1024;
  while (tcap < 2 * occ_max && tcap < (1u << 31)) tcap <<= 1;
  L.tkeys.ensure(tcap);
  L.trange.ensure(tcap);
  const size_t tmp = sort_tmp_bytes(n, G.key_bits);
  w.sort_tmp.ensure(tmp);
  w.counters.ensure(8);
  w.h_cnt.ensure(8);
  B->keys_in = w.keys_in.p; B->keys_out = w.keys_out.p;
  B->idx_in = w.idx_in.p; B->idx_out = L.idx.p;
  B->sx = L.sx.p; B->sy = L.sy.p; B->sz = L.sz.p;
  B->tkeys = L.tkeys.p; B->trange = L.trange.p; B->tmask = tcap - 1;
  B->sort_tmp = w.sort_tmp.p; B->sort_tmp_bytes = w.sort_tmp.cap;
  float4* rec = nullptr;
  if (n >= kGridRecMin) {
    w.rec.ensure(n);
    rec = w.rec.p;
  }
  HIPCHK(grid_build(X ? X : w.x.p, Y ? Y : w.y.p, Z ? Z : w.z.p, n, G, *B, w.counters.p,
                    c->stream, rec));
  HIPCHK(hipMemcpyAsync(w.h_cnt.p, w.counters.p, 16, hipMemcpyDeviceToHost, c->stream));
  sync(c);
  if (pw_occ) {
    unsigned long long sq;
    std::memcpy(&sq, w.h_cnt.p + 2, 8);
    *pw_occ = n > 0 ? (double)sq / (double)n : 0.0;
  }
  return w.h_cnt.p[0];
}

// grid hierarchy over nw.x/y/z for k-nearest-neighbour queries (normals.hip, k_normals_knn):
// level-0 cell guessed from the bounding volume, then resized once from the measured occupancy
// so an occupied cell holds ~k/2 points (surface-like clouds: occupancy ~ cell^2); levels above
// grow 2x until one has <= 2 cells per axis
// the hierarchy's plan: level 0 built (cell tuned on the occupancy), the coarser cells recorded;
// build_level() builds a planned level on demand (the k-NN normals build a level only when some
// query needs it: most clouds resolve every query within a few levels of the planned ~10)
struct KnnPlan {
  BBox b;
  int n = 0;
  double cell[kMaxLevels] = {};
  int planned = 0;
};

void build_level(dlg_ctx* c, const KnnPlan& P, KnnLevels& L, int l, const GridBufs* B0) {
  GridBufs BL;
  GridDesc G;
  if (l == 0) {
    BL = *B0;
    G = L.G[0];
  } else {
    G = make_grid(P.b, P.cell[l]);
    build_grid(c, P.n, G, l, &BL);
  }
  L.G[l] = G;
  L.sx[l] = BL.sx; L.sy[l] = BL.sy; L.sz[l] = BL.sz; L.idx[l] = BL.idx_out;
  c->nw.lv[l].pos.ensure(P.n);
  launch_inverse_perm(BL.idx_out, P.n, c->nw.lv[l].pos.p, c->stream);
  L.pos_of[l] = c->nw.lv[l].pos.p;
  L.tkeys[l] = BL.tkeys; L.trange[l] = BL.trange; L.tmask[l] = BL.tmask;
}

// grid hierarchy over nw.x/y/z for k-nearest-neighbour queries (normals.hip, k_normals_knn):
// level-0 cell guessed from the bounding volume, then resized once from the measured occupancy
// so an occupied cell holds ~k/2 points (surface-like clouds: occupancy ~ cell^2); levels above
// grow 2x until one has <= 2 cells per axis.  Builds `eager_levels` levels (all: -1); L.levels
// is the planned count either way.
KnnLevels build_hierarchy_plan(dlg_ctx* c, int n, const BBox& b, int k_nn, KnnPlan* plan,
                               int eager_levels) {
  GridBufs B;
  double ext[3], maxe = 0.0;
  for (int k = 0; k < 3; ++k) {
    ext[k] = b.any ? (double)b.hi[k] - (double)b.lo[k] : 0.0;
    maxe = std::max(maxe, ext[k]);
  }
  if (maxe <= 0.0) maxe = 1.0;
  double vol = 1.0;
  for (int k = 0; k < 3; ++k) vol *= std::max(ext[k], maxe * 1e-3);
  double cell = std::cbrt(vol * k_nn / n);
  GridDesc G = make_grid(b, cell);
  // tune on the point-weighted occupancy (what a typical query sees; sparse outlier cells do
  // not drag it down), assuming surface-like scaling occ ~ cell^2; two corrections at most
  const double target = std::max(2.0, k_nn / 2.0);
  // large clouds tune on a prefix of 1/8 of the points (a sampled cell's occupancy is ~1/8 of the
  // full one: pw_full ~ (pw_sample - (1 - f)) / f), then build level 0 once; the cell size only
  // affects the speed, never the neighbour sets
  const int ns = n >= (1 << 20) ? n / 8 : n;
  const double f = (double)ns / (double)n;
  for (int it = 0; it < 3; ++it) {
    double pw = 0.0;
    build_grid(c, ns, G, 0, &B, nullptr, nullptr, nullptr, &pw);
    if (ns < n) pw = (pw - (1.0 - f)) / f;
    if (it == 2 || pw <= 0.0 || (pw <= 2.0 * target && pw >= 0.5 * target)) break;
    cell *= std::sqrt(target / pw);
    G = make_grid(b, cell);
  }
  if (ns < n) build_grid(c, n, G, 0, &B);
  KnnPlan P;
  P.b = b;
  P.n = n;
  const double top_cell = maxe * 0.75;  // floor(ext / cell) + 1 <= 2 on every axis
  // 2x per level, more when the hierarchy would not fit kMaxLevels
  const double fac = std::max(2.0, std::pow(top_cell / cell, 1.0 / (kMaxLevels - 1)));
  for (int l = 0; l < kMaxLevels; ++l) {
    const bool last = cell >= top_cell || l == kMaxLevels - 1;
    if (last) cell = std::max(cell, top_cell);
    P.cell[l] = cell;
    P.planned = l + 1;
    if (last) break;
    cell *= fac;
  }
  KnnLevels L;
  L.levels = P.planned;
  L.G[0] = G;
  const int eager = eager_levels < 0 ? P.planned : std::min(eager_levels, P.planned);
  for (int l = 0; l < eager; ++l) build_level(c, P, L, l, &B);
  if (plan) *plan = P;
  return L;
}

KnnLevels build_hierarchy(dlg_ctx* c, int n, const BBox& b, int k_nn) {
  return build_hierarchy_plan(c, n, b, k_nn, nullptr, -1);
}

void check_points(const dlg_points* pts) {
  if (!pts || pts->n < 0 || (pts->n > 0 && !pts->xyz))
    throw DlgError(DLG_ERR_INVALID, "points: null or negative size");
  if (pts->stride_bytes < 12 || pts->stride_bytes % 4)
    throw DlgError(DLG_ERR_INVALID, "stride_bytes must be >= 12 and a multiple of 4");
  if (pts->n > INT32_MAX / 2) throw DlgError(DLG_ERR_INVALID, "more than 2^30 points");
}

namespace {

void check_normals_args(float radius, int k_nn, int mode) {
  if (mode != DLG_NORMALS_PCL_FLOAT && mode != DLG_NORMALS_CENTRED_DOUBLE)
    throw DlgError(DLG_ERR_INVALID, "mode must be DLG_NORMALS_PCL_FLOAT or DLG_NORMALS_CENTRED_DOUBLE");
  if (k_nn < 0 || k_nn > kMaxKnn) throw DlgError(DLG_ERR_INVALID, "k_nn must be in 0..64");
  if (k_nn == 0 && !(radius > 0.0f && std::isfinite(radius)))
    throw DlgError(DLG_ERR_INVALID, "neither radius nor k set");  // PCL initCompute error
}

// the normals of the n points in nw.x/y/z (bounding box b) -> nw.nrm (nx, ny, nz, curvature)
void normals_core(dlg_ctx* c, int n, const BBox& b, float radius, int k_nn, const float* vp_in,
                  int mode);

void estimate_normals(dlg_ctx* c, const dlg_points* pts, float radius, int k_nn, const float* vp_in,
                      float* out, int64_t out_stride, int mode) {
  check_normals_args(radius, k_nn, mode);
  check_points(pts);
  if (!out) throw DlgError(DLG_ERR_INVALID, "normals_out is null");
  if (out_stride != 16 && out_stride < 32) throw DlgError(DLG_ERR_INVALID, "out_stride_bytes must be 16 or >= 32");
  if (out_stride % 4) throw DlgError(DLG_ERR_INVALID, "out_stride_bytes must be a multiple of 4");
  const int n = (int)pts->n;
  if (n == 0) return;
  const BBox b = upload_points(c, pts);
  normals_core(c, n, b, radius, k_nn, vp_in, mode);
  NormalsWork& w = c->nw;
  const size_t obytes = (size_t)n * (size_t)out_stride;
  w.out.ensure(obytes);
  launch_pack_normals(w.nrm.p, n, reinterpret_cast<float*>(w.out.p), out_stride / 4,
                      out_stride == 16 ? 3 : 4, c->stream);
  HIPCHK(hipMemcpyAsync(out, w.out.p, obytes, hipMemcpyDeviceToHost, c->stream));
  sync(c);
}

void normals_core(dlg_ctx* c, int n, const BBox& b, float radius, int k_nn, const float* vp_in,
                  int mode) {
  const bool pclf = mode == DLG_NORMALS_PCL_FLOAT;
  const float vp[3] = {vp_in ? vp_in[0] : 0.0f, vp_in ? vp_in[1] : 0.0f, vp_in ? vp_in[2] : 0.0f};
  NormalsWork& w = c->nw;
  w.nrm.ensure(n);
  GridBufs B;
  if (k_nn == 0) {
    const GridDesc G = make_grid(b, (double)radius);
    build_grid(c, n, G, 0, &B);
    const float r2 = (float)((double)radius * (double)radius);  // KdTreeFLANN: radius * radius
    bool chunked = pclf && !c->opt.nbr_fused;
    if (!pclf) {
      launch_normals_radius(G, B, n, r2, vp, w.nrm.p, c->stream);
    } else if (!chunked) {
      // one fused pass (<= 512 neighbours per query), the overflow in a wider one (<= 1024); a
      // query beyond that (none at the configs' radii) sends the whole call down the chunked path
      w.ovfa.ensure(n);
      w.ovfb.ensure(n);
      w.ovfc.ensure(2);
      w.h_cnt.ensure(2);
      HIPCHK(hipMemsetAsync(w.ovfc.p, 0, 2 * sizeof(uint32_t), c->stream));
      launch_nbr_fused(G, B, n, nullptr, nullptr, 0, r2, vp,
                       w.nrm.p, w.ovfa.p, w.ovfc.p, c->num_cus, c->stream);
      launch_nbr_fused(G, B, n, w.ovfa.p, w.ovfc.p, 1, r2, vp, w.nrm.p, w.ovfb.p, w.ovfc.p + 1,
                       c->num_cus, c->stream);
      HIPCHK(hipMemcpyAsync(w.h_cnt.p, w.ovfc.p + 1, sizeof(uint32_t), hipMemcpyDeviceToHost,
                            c->stream));
      sync(c);
      chunked = w.h_cnt.p[0] > 0;
    }
    if (chunked) {
      // queries in chunks of the sorted order: neighbour counts, offsets, then the (d2, index)
      // keys of the chunk (bounded by kMaxKeys; a chunk is halved until it fits)
      constexpr int64_t kMaxKeys = int64_t(1) << 28;  // 2 GiB of keys
      const int qc_max = std::min(n, 1 << 22);
      w.ncnt.ensure(qc_max);
      w.noff.ensure(qc_max);
      w.sort_tmp.ensure(std::max(w.sort_tmp.cap, nbr_scan_tmp_bytes(qc_max)));
      w.h_bst.ensure(2);
      for (int q0 = 0; q0 < n;) {
        int nq = std::min(qc_max, n - q0);
        int64_t total = 0;
        for (;;) {
          launch_nbr_count(G, B, q0, nq, r2, w.ncnt.p, c->stream);
          HIPCHK(nbr_scan(w.sort_tmp.p, w.sort_tmp.cap, w.ncnt.p, w.noff.p, nq, c->stream));
          HIPCHK(hipMemcpyAsync(w.h_bst.p, w.noff.p + (nq - 1), 8, hipMemcpyDeviceToHost, c->stream));
          HIPCHK(hipMemcpyAsync(reinterpret_cast<int32_t*>(w.h_bst.p + 1), w.ncnt.p + (nq - 1), 4,
                                hipMemcpyDeviceToHost, c->stream));
          sync(c);
          total = (int64_t)w.h_bst.p[0] + *reinterpret_cast<int32_t*>(w.h_bst.p + 1);
          if (total <= kMaxKeys || nq == 1) break;
          nq = (nq + 1) / 2;
        }
        w.nkeys.ensure((size_t)std::max<int64_t>(total, 1));
        launch_nbr_fill_sort_normals(G, B, q0, nq, r2, w.ncnt.p, w.noff.p, w.nkeys.p, w.x.p,
                                     w.y.p, w.z.p, vp, w.nrm.p, c->num_cus, c->stream);
        HIPCHK(hipGetLastError());
        q0 += nq;
      }
    }
  } else {
    KnnPlan plan;
    KnnLevels L = build_hierarchy_plan(c, n, b, k_nn, &plan, 1);
    w.queue.ensure(n);
    w.processed.ensure(n);
    // deferred-query flags per level, indexed by point: a level is built only once some query
    // is flagged for it (most clouds resolve every query within a few of the planned levels)
    w.dflags.ensure((size_t)n * L.levels);
    if (L.levels > 1)
      HIPCHK(hipMemsetAsync(w.dflags.p + n, 0, (size_t)n * (L.levels - 1), c->stream));
    w.sort_tmp.ensure(select_tmp_bytes(n));
    bool built[kMaxLevels] = {true};
    auto count_flags = [&](const uint8_t* f) {
      HIPCHK(select_flagged(w.sort_tmp.p, w.sort_tmp.cap, f, n, w.queue.p, w.counters.p,
                            c->stream));
      HIPCHK(hipMemcpyAsync(w.h_cnt.p, w.counters.p, 4, hipMemcpyDeviceToHost, c->stream));
      sync(c);
      return (int)w.h_cnt.p[0];
    };
    for (int l = 0; l < L.levels; ++l) {
      const int32_t* qpos = nullptr;  // level 0: every point
      int nq = n;
      int tnext = -1;
      if (l > 0 && l + 2 < L.levels && !built[l + 1]) {
        // a level nothing has been sent to yet is skipped by this level's deferrals when the
        // level above it has queries already (it will be built anyway; C5: level 0 sends its
        // sparse queries to level 3, so level 1's few deferrals need no level 2)
        if (count_flags(w.dflags.p + (size_t)(l + 1) * n) == 0 &&
            count_flags(w.dflags.p + (size_t)(l + 2) * n) > 0)
          tnext = l + 2;
      }
      if (l > 0) {
        const uint8_t* f = w.dflags.p + (size_t)l * n;
        nq = count_flags(f);
        if (nq == 0) {
          if (l >= 4) break;  // (queries skip levels only from level 0, at most to level 3)
          continue;
        }
        if (!built[l]) build_level(c, plan, L, l, nullptr), built[l] = true;
        // the flagged queries in this level's cell order
        launch_gather_flags(f, L.idx[l], n, w.processed.p, c->stream);
        nq = count_flags(w.processed.p);
        qpos = w.queue.p;
      }
      launch_normals_knn(L, l, qpos, nq, w.x.p, w.y.p, w.z.p, k_nn, vp, w.nrm.p, w.dflags.p,
                         (int64_t)n, L.levels - 1, pclf, c->stream, tnext);
    }
  }
  HIPCHK(hipGetLastError());
}

int64_t regulate_core(dlg_ctx* c, int n, const float* X, const float* Y, const float* Z,
                      const BBox& b, int64_t seed, int seed_is_outward, float radius);

int64_t regulate_normals(dlg_ctx* c, const dlg_points* pts, float* nrm_io, int64_t stride,
                         int64_t seed, int seed_is_outward, float radius, uint8_t* processed_out) {
  check_points(pts);
  if (!nrm_io) throw DlgError(DLG_ERR_INVALID, "normals_inout is null");
  if (stride < 12 || stride % 4) throw DlgError(DLG_ERR_INVALID, "stride_bytes must be >= 12 and a multiple of 4");
  if (!(radius > 0.0f && std::isfinite(radius))) throw DlgError(DLG_ERR_INVALID, "radius must be > 0");
  const int n = (int)pts->n;
  if (seed < 0) {  // PlaneDetect.h:592-596: "invalid point index", return
    if (processed_out) std::memset(processed_out, 0, (size_t)n);
    return 0;
  }
  if (seed >= n) throw DlgError(DLG_ERR_INVALID, "seed index out of range");
  NormalsWork& w = c->nw;
  const BBox b = upload_points(c, pts);
  const size_t nbytes = (size_t)n * (size_t)stride;
  w.out.ensure(nbytes);
  w.nrm.ensure(n);
  HIPCHK(hipMemcpyAsync(w.out.p, nrm_io, nbytes, hipMemcpyHostToDevice, c->stream));
  launch_unpack_normals(reinterpret_cast<const float*>(w.out.p), n, stride / 4, w.nrm.p, c->stream);
  const int64_t qt = regulate_core(c, n, w.x.p, w.y.p, w.z.p, b, seed, seed_is_outward, radius);
  launch_pack_normals(w.nrm.p, n, reinterpret_cast<float*>(w.out.p), stride / 4, -1, c->stream);
  HIPCHK(hipMemcpyAsync(nrm_io, w.out.p, nbytes, hipMemcpyDeviceToHost, c->stream));
  if (processed_out)
    HIPCHK(hipMemcpyAsync(processed_out, w.processed.p, n, hipMemcpyDeviceToHost, c->stream));
  sync(c);
  return qt;
}

// the BFS of regulateNormal over the n points X/Y/Z (bounding box b) and the normals in nw.nrm
// (x, y, z; .w carried through): nw.nrm flipped in place (PCL's queue order, float dots),
// nw.processed = isProcessed; returns the queue length (points reached)
int64_t regulate_core(dlg_ctx* c, int n, const float* X, const float* Y, const float* Z,
                      const BBox& b, int64_t seed, int seed_is_outward, float radius) {
  NormalsWork& w = c->nw;
  const GridDesc G = make_grid(b, (double)radius);
  GridBufs B;
  build_grid(c, n, G, 0, &B, X, Y, Z);
  const float r2 = (float)((double)radius * (double)radius);
  w.nrm_s.ensure(n);
  w.pos_of.ensure(n);
  w.processed.ensure(n);
  w.processed_s.ensure(n);
  w.claim.ensure(n);
  w.queue.ensure(n);
  w.cand.ensure(n);
  w.ids.ensure(n);
  w.counters.ensure(8);
  w.h_cnt.ensure(8);
  HIPCHK(hipMemsetAsync(w.processed_s.p, 0, n, c->stream));
  HIPCHK(hipMemsetAsync(w.claim.p, 0xff, (size_t)n * 4, c->stream));
  launch_bfs_prepare(B, n, w.nrm.p, w.nrm_s.p, w.pos_of.p, c->stream);
  // PlaneDetect.h:600-607: seed flipped unless its direction was confirmed outward
  launch_bfs_seed((int32_t)seed, seed_is_outward ? 0 : 1, w.pos_of.p, w.nrm_s.p, w.processed_s.p,
                  w.queue.p, c->stream);
  // levels run back to back on the device (state in w.bst); the host checks the level size every
  // 16 levels -- levels enqueued after the frontier empties are no-ops
  w.bst.ensure(4);
  w.ccnt.ensure(n); w.coffs.ensure(n); w.ccur.ensure(n); w.sd2.ensure(n);
  w.ctile.ensure(n / 1024 + 2); w.cslot.ensure(n);
  w.cdone.ensure((size_t)B.tmask + 1);
  HIPCHK(hipMemsetAsync(w.cdone.p, 0, ((size_t)B.tmask + 1) * 4, c->stream));
  const Bfs2Bufs W{w.ccnt.p, w.ccur.p, w.coffs.p, w.ctile.p, w.cslot.p, w.sd2.p, w.ids.p, w.cdone.p};
  w.h_bst.ensure(4);
  w.h_bst.p[0] = 0; w.h_bst.p[1] = 1; w.h_bst.p[2] = 0; w.h_bst.p[3] = 1;
  HIPCHK(hipMemcpyAsync(w.bst.p, w.h_bst.p, 32, hipMemcpyHostToDevice, c->stream));
  const int grid = c->num_cus * 4;
  for (;;) {
    for (int k = 0; k < 16; ++k)
      launch_bfs2_level(w.queue.p, w.bst.p, w.pos_of.p, G, B, r2, w.processed_s.p, w.claim.p,
                        w.nrm_s.p, w.cand.p, W, grid, c->stream, c->opt.bfs_wave);
    HIPCHK(hipGetLastError());
    HIPCHK(hipMemcpyAsync(w.h_bst.p, w.bst.p, 32, hipMemcpyDeviceToHost, c->stream));
    sync(c);
    if (w.h_bst.p[3] > n) throw DlgError(DLG_ERR_INTERNAL, "BFS queue overflow");
    if (w.h_bst.p[1] == 0) break;
  }
  const int64_t qt = w.h_bst.p[3];
  launch_bfs_finish(B, n, w.nrm_s.p, w.processed_s.p, w.nrm.p, w.processed.p, c->stream);
  HIPCHK(hipGetLastError());
  return qt;
}

// regulateNormal on the cloud's device copy and its attached normals (no host round trip): the
// flipped normals replace the attached ones (raw and normalised, the Morton copy's too)
int64_t cloud_regulate_normals(dlg_ctx* c, dlg_cloud* cl, int64_t seed, int seed_is_outward,
                               float radius, uint8_t* processed_out, float* normals_out,
                               int64_t out_stride) {
  if (c->comm->world() > 1)
    throw DlgError(DLG_ERR_INVALID, "dlg_cloud_regulate_normals: the cloud is one rank's shard "
                                    "(world > 1); the BFS needs the whole cloud");
  if (!cl->has_normals) throw DlgError(DLG_ERR_INVALID, "the cloud has no normals attached");
  if (!(radius > 0.0f && std::isfinite(radius))) throw DlgError(DLG_ERR_INVALID, "radius must be > 0");
  if (normals_out && (out_stride % 4 || (out_stride != 16 && out_stride < 32)))
    throw DlgError(DLG_ERR_INVALID, "out_stride_bytes must be 16 or >= 32 (multiple of 4)");
  if (cl->n_total > INT32_MAX / 2) throw DlgError(DLG_ERR_INVALID, "more than 2^30 points");
  const int n = (int)cl->n_total;
  if (seed < 0 || n == 0) {  // PlaneDetect.h:592-596: "invalid point index", return
    if (processed_out && n) std::memset(processed_out, 0, (size_t)n);
    if (seed >= 0 && n == 0) throw DlgError(DLG_ERR_INVALID, "seed index out of range");
    return 0;
  }
  if (seed >= n) throw DlgError(DLG_ERR_INVALID, "seed index out of range");
  NormalsWork& w = c->nw;
  w.nrm.ensure(n);
  HIPCHK(hipMemcpyAsync(w.nrm.p, cl->raw_nrm.p, 16 * (size_t)n, hipMemcpyDeviceToDevice, c->stream));
  const float* X = cl->pristine.x.p;
  const float* Y = cl->pristine.y.p;
  const float* Z = cl->pristine.z.p;
  const BBox b = bbox_of(c, X, Y, Z, n);
  const int64_t qt = regulate_core(c, n, X, Y, Z, b, seed, seed_is_outward, radius);
  HIPCHK(hipMemcpyAsync(cl->raw_nrm.p, w.nrm.p, 16 * (size_t)n, hipMemcpyDeviceToDevice, c->stream));
  attach_normals(c, cl, reinterpret_cast<const float*>(cl->raw_nrm.p), 4, 3, true);
  if (normals_out) {
    const size_t obytes = (size_t)n * (size_t)out_stride;
    w.out.ensure(obytes);
    launch_pack_normals(w.nrm.p, n, reinterpret_cast<float*>(w.out.p), out_stride / 4,
                        out_stride == 16 ? 3 : 4, c->stream);
    HIPCHK(hipMemcpyAsync(normals_out, w.out.p, obytes, hipMemcpyDeviceToHost, c->stream));
  }
  if (processed_out)
    HIPCHK(hipMemcpyAsync(processed_out, w.processed.p, n, hipMemcpyDeviceToHost, c->stream));
  sync(c);
  return qt;
}

// regulateNormal() later-round branch (PlaneDetect.h:553-584): for every point of the current
// cloud, its nearest neighbour in the backup cloud (KdTreeFLANN::nearestKSearch, k = 1); the
// normal flips when Vector3f(n).dot(Vector3f(n_backup)) < 0
void orient_normals_nn(dlg_ctx* c, const dlg_points* pts, float* nrm_io, int64_t stride,
                       const dlg_points* ref, const float* ref_nrm, int64_t ref_stride) {
  check_points(pts);
  check_points(ref);
  if (!nrm_io || (ref->n > 0 && !ref_nrm)) throw DlgError(DLG_ERR_INVALID, "normals are null");
  if (stride < 12 || stride % 4 || ref_stride < 12 || ref_stride % 4)
    throw DlgError(DLG_ERR_INVALID, "normal strides must be >= 12 and a multiple of 4");
  const int n = (int)pts->n, m = (int)ref->n;
  if (n == 0) return;
  if (m == 0) throw DlgError(DLG_ERR_INVALID, "empty backup cloud");
  NormalsWork& w = c->nw;
  // queries: the current cloud (own buffers), grid: the backup cloud (nw.x/y/z)
  w.qx.ensure(n); w.qy.ensure(n); w.qz.ensure(n);
  {
    const size_t bytes = (size_t)n * (size_t)pts->stride_bytes;
    w.raw.ensure(bytes);
    HIPCHK(hipMemcpyAsync(w.raw.p, pts->xyz, bytes, hipMemcpyHostToDevice, c->stream));
    launch_deinterleave(reinterpret_cast<const float*>(w.raw.p), n, pts->stride_bytes / 4, w.qx.p,
                        w.qy.p, w.qz.p, c->stream);
  }
  const BBox b = upload_points(c, ref);
  const KnnLevels L = build_hierarchy(c, m, b, 1);
  w.nn.ensure(n);
  w.queue.ensure(n);
  w.cand.ensure(n);
  int32_t* qin = nullptr;
  int32_t* qout = w.queue.p;
  int nq = n;
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
  // normals: current (in/out) and backup, raw strided records on the device
  const size_t nbytes = (size_t)n * (size_t)stride, rbytes = (size_t)m * (size_t)ref_stride;
  w.out.ensure(nbytes);
  w.raw.ensure(rbytes);
  HIPCHK(hipMemcpyAsync(w.out.p, nrm_io, nbytes, hipMemcpyHostToDevice, c->stream));
  HIPCHK(hipMemcpyAsync(w.raw.p, ref_nrm, rbytes, hipMemcpyHostToDevice, c->stream));
  launch_flip_to_reference(reinterpret_cast<float*>(w.out.p), stride / 4,
                           reinterpret_cast<const float*>(w.raw.p), ref_stride / 4, w.nn.p, n,
                           c->stream);
  HIPCHK(hipGetLastError());
  HIPCHK(hipMemcpyAsync(nrm_io, w.out.p, nbytes, hipMemcpyDeviceToHost, c->stream));
  sync(c);
}

// preProcess() (PlaneDetect.h:448-512): removeNaNFromPointCloud, optional translation of the
// cloud to its centroid (sequential float sums, as the reference), then the redundancy removal
// with radius min_dist.  Output: kept points (translated) in input order and their input index.
int64_t preprocess(dlg_ctx* c, const dlg_points* pts, int translate, float min_dist, float* out,
                   int64_t out_stride, int32_t* out_idx, int64_t cap, float* translation,
                   int64_t* n_needed) {
  check_points(pts);
  if (out_stride != 12 && out_stride < 16) throw DlgError(DLG_ERR_INVALID, "out_stride_bytes must be 12 or >= 16");
  if (out_stride % 4) throw DlgError(DLG_ERR_INVALID, "out_stride_bytes must be a multiple of 4");
  if (!(min_dist == min_dist)) throw DlgError(DLG_ERR_INVALID, "min_dist is NaN");
  if (translation) translation[0] = translation[1] = translation[2] = 0.0f;
  const int n0 = (int)pts->n;
  if (n0 == 0) return 0;
  NormalsWork& w = c->nw;
  (void)upload_points(c, pts);  // nw.x/y/z
  // 1. removeNaNFromPointCloud: ascending indices of the finite points
  w.processed.ensure(n0);
  w.ids.ensure(n0);
  w.counters.ensure(8);
  w.h_cnt.ensure(8);
  w.sort_tmp.ensure(select_tmp_bytes(n0));
  launch_finite_flags(w.x.p, w.y.p, w.z.p, n0, w.processed.p, c->stream);
  HIPCHK(select_flagged(w.sort_tmp.p, w.sort_tmp.cap, w.processed.p, n0, w.ids.p, w.counters.p,
                        c->stream));
  HIPCHK(hipMemcpyAsync(w.h_cnt.p, w.counters.p, 4, hipMemcpyDeviceToHost, c->stream));
  sync(c);
  const int n = (int)w.h_cnt.p[0];
  if (n == 0) return 0;
  w.qx.ensure(n); w.qy.ensure(n); w.qz.ensure(n);
  launch_gather3(w.ids.p, n, w.x.p, w.y.p, w.z.p, w.qx.p, w.qy.p, w.qz.p, c->stream);
  // 2. translation to the centroid (PlaneDetect.h:458-479)
  if (translate) {
    w.partial.ensure(6);
    // the loop's three float chains p.x += x_i ... in index order, evaluated exactly in parallel
    // by the PCL-refit machinery (fsum.hip; the six product chains ride along); a
    // single-wave sequential pass took ~86 ms at 10M points
    w.fs_scr.ensure(fs_scratch_bytes(n, 1));
    const FsBuffers fb = fs_carve(w.fs_scr.p, n, 1);
    HIPCHK(fs_reset(fb, c->stream, c->opt.fs_poison));
    launch_fs_refit(w.qx.p, w.qy.p, w.qz.p, 1, reinterpret_cast<const int32_t*>(w.counters.p), n,
                    fb, nullptr, nullptr, nullptr, c->num_cus, c->stream, nullptr, nullptr, nullptr,
                    nullptr, nullptr, 0, nullptr, c->opt.fs_segments);
    launch_centroid_div(fb.sums + 6, n, w.partial.p, c->stream);
    launch_translate(w.qx.p, w.qy.p, w.qz.p, n, w.partial.p, c->stream);
    float p[3];
    HIPCHK(hipMemcpyAsync(p, w.partial.p, 12, hipMemcpyDeviceToHost, c->stream));
    sync(c);
    if (translation) std::memcpy(translation, p, 12);
  }
  // 3. redundancy removal (PlaneDetect.h:482-508)
  const BBox b = bbox_of(c, w.qx.p, w.qy.p, w.qz.p, n);
  const double r = min_dist > 0.0f ? (double)min_dist : 0.0;
  const GridDesc G = make_grid(b, r > 0.0 ? r : 1.0);
  GridBufs B;
  build_grid(c, n, G, 0, &B, w.qx.p, w.qy.p, w.qz.p);
  const float r2 = (float)(r * r);  // radiusSearch(point, float radius): (float)(r * r)
  w.processed_s.ensure(n);
  w.queue.ensure(n);
  w.cand.ensure(n);
  HIPCHK(hipMemsetAsync(w.processed_s.p, 0, n, c->stream));
  int32_t* qin = nullptr;
  int32_t* qout = w.queue.p;
  int nq = n;
  while (nq > 0) {
    HIPCHK(hipMemsetAsync(w.counters.p, 0, 4, c->stream));
    launch_mis_round(qin, nq, G, B, r2, w.processed_s.p, qout, w.counters.p, c->stream);
    HIPCHK(hipMemcpyAsync(w.h_cnt.p, w.counters.p, 4, hipMemcpyDeviceToHost, c->stream));
    sync(c);
    const int left = (int)w.h_cnt.p[0];
    if (left >= nq) throw DlgError(DLG_ERR_INTERNAL, "redundancy removal made no progress");
    nq = left;
    qin = qout;
    qout = qout == w.queue.p ? w.cand.p : w.queue.p;
  }
  launch_mis_flags(B, n, w.processed_s.p, w.processed.p, c->stream);
  HIPCHK(select_flagged(w.sort_tmp.p, w.sort_tmp.cap, w.processed.p, n, w.cand.p, w.counters.p,
                        c->stream));
  HIPCHK(hipMemcpyAsync(w.h_cnt.p, w.counters.p, 4, hipMemcpyDeviceToHost, c->stream));
  sync(c);
  const int64_t kept = w.h_cnt.p[0];
  *n_needed = kept;
  if (kept > cap) throw DlgError(DLG_ERR_CAPACITY, "output too small: need " + std::to_string(kept));
  if (!out || !out_idx) throw DlgError(DLG_ERR_INVALID, "output buffers are null");
  const size_t obytes = (size_t)kept * (size_t)out_stride;
  w.out.ensure(obytes + 4 * (size_t)kept);
  float* dout = reinterpret_cast<float*>(w.out.p);
  int32_t* didx = reinterpret_cast<int32_t*>(w.out.p + obytes);
  launch_emit_points(w.cand.p, (int)kept, w.qx.p, w.qy.p, w.qz.p, w.ids.p, dout, out_stride / 4,
                     didx, c->stream);
  HIPCHK(hipGetLastError());
  HIPCHK(hipMemcpyAsync(out, dout, obytes, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(hipMemcpyAsync(out_idx, didx, 4 * (size_t)kept, hipMemcpyDeviceToHost, c->stream));
  sync(c);
  return kept;
}

}  // namespace
}  // namespace dlg

extern "C" {

dlg_status dlg_estimate_normals(dlg_ctx* c, const dlg_points* pts, float radius, int k_nn,
                                const float viewpoint[3], float* normals_out,
                                int64_t out_stride_bytes) {
  return dlg_estimate_normals_ex(c, pts, radius, k_nn, viewpoint, normals_out, out_stride_bytes,
                                 DLG_NORMALS_PCL_FLOAT);
}

dlg_status dlg_estimate_normals_ex(dlg_ctx* c, const dlg_points* pts, float radius, int k_nn,
                                   const float viewpoint[3], float* normals_out,
                                   int64_t out_stride_bytes, int mode) {
  if (!c) return DLG_ERR_INVALID;
  return guarded(c, [&] {
    estimate_normals(c, pts, radius, k_nn, viewpoint, normals_out, out_stride_bytes, mode);
  });
}

dlg_status dlg_cloud_estimate_normals(dlg_ctx* c, dlg_cloud* cl, float radius, int k_nn,
                                      const float viewpoint[3], int mode, float* normals_out,
                                      int64_t out_stride_bytes) {
  if (!c || !cl || cl->ctx != c) return DLG_ERR_INVALID;
  return guarded(c, [&] {
    if (c->comm->world() > 1)
      throw DlgError(DLG_ERR_INVALID, "dlg_cloud_estimate_normals: the cloud is one rank's shard "
                                      "(world > 1); its normals need the whole cloud");
    check_normals_args(radius, k_nn, mode);
    if (normals_out && (out_stride_bytes % 4 || (out_stride_bytes != 16 && out_stride_bytes < 32)))
      throw DlgError(DLG_ERR_INVALID, "out_stride_bytes must be 16 or >= 32 (multiple of 4)");
    if (cl->n_total > INT32_MAX / 2) throw DlgError(DLG_ERR_INVALID, "more than 2^30 points");
    const int n = (int)cl->n_total;
    NormalsWork& w = c->nw;
    if (n > 0) {
      // the cloud's own device copy (upload order) is the point set
      w.x.ensure(n); w.y.ensure(n); w.z.ensure(n);
      HIPCHK(hipMemcpyAsync(w.x.p, cl->pristine.x.p, 4 * (size_t)n, hipMemcpyDeviceToDevice, c->stream));
      HIPCHK(hipMemcpyAsync(w.y.p, cl->pristine.y.p, 4 * (size_t)n, hipMemcpyDeviceToDevice, c->stream));
      HIPCHK(hipMemcpyAsync(w.z.p, cl->pristine.z.p, 4 * (size_t)n, hipMemcpyDeviceToDevice, c->stream));
      const BBox b = bbox_of(c, w.x.p, w.y.p, w.z.p, n);
      normals_core(c, n, b, radius, k_nn, viewpoint, mode);
    }
    attach_normals(c, cl, n > 0 ? reinterpret_cast<const float*>(w.nrm.p) : nullptr, 4, 3, true);
    if (normals_out && n > 0) {
      const size_t obytes = (size_t)n * (size_t)out_stride_bytes;
      w.out.ensure(obytes);
      launch_pack_normals(w.nrm.p, n, reinterpret_cast<float*>(w.out.p), out_stride_bytes / 4,
                          out_stride_bytes == 16 ? 3 : 4, c->stream);
      HIPCHK(hipMemcpyAsync(normals_out, w.out.p, obytes, hipMemcpyDeviceToHost, c->stream));
    }
    sync(c);
  });
}

dlg_status dlg_regulate_normals(dlg_ctx* c, const dlg_points* pts, float* normals_inout,
                                int64_t stride_bytes, int64_t seed_idx, int seed_is_outward,
                                float radius, uint8_t* processed_out, int64_t* n_processed) {
  if (!c) return DLG_ERR_INVALID;
  return guarded(c, [&] {
    const int64_t k = regulate_normals(c, pts, normals_inout, stride_bytes, seed_idx,
                                       seed_is_outward, radius, processed_out);
    if (n_processed) *n_processed = k;
  });
}

dlg_status dlg_cloud_regulate_normals(dlg_ctx* c, dlg_cloud* cl, int64_t seed_idx,
                                      int seed_is_outward, float radius, uint8_t* processed_out,
                                      int64_t* n_processed, float* normals_out,
                                      int64_t out_stride_bytes) {
  if (!c || !cl || cl->ctx != c) return DLG_ERR_INVALID;
  return guarded(c, [&] {
    const int64_t k = cloud_regulate_normals(c, cl, seed_idx, seed_is_outward, radius,
                                             processed_out, normals_out, out_stride_bytes);
    if (n_processed) *n_processed = k;
  });
}

dlg_status dlg_orient_normals_nn(dlg_ctx* c, const dlg_points* pts, float* normals_inout,
                                 int64_t stride_bytes, const dlg_points* ref_pts,
                                 const float* ref_normals, int64_t ref_stride_bytes) {
  if (!c) return DLG_ERR_INVALID;
  return guarded(c, [&] {
    orient_normals_nn(c, pts, normals_inout, stride_bytes, ref_pts, ref_normals, ref_stride_bytes);
  });
}

dlg_status dlg_preprocess(dlg_ctx* c, const dlg_points* pts, int translate, float min_dist,
                          float* out_xyz, int64_t out_stride_bytes, int32_t* out_index,
                          int64_t cap, int64_t* n_out, float translation[3]) {
  if (!c || !n_out) return DLG_ERR_INVALID;
  *n_out = 0;
  return guarded(c, [&] {
    preprocess(c, pts, translate, min_dist, out_xyz, out_stride_bytes, out_index, cap, translation,
               n_out);  // *n_out = points kept, also when the output capacity is too small
  });
}

}  // extern "C"

