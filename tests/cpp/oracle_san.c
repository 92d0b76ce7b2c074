/* Host sanitizer run (ASan + UBSan, built by tests/test_sanitizers.py with gcc) of the oracle
 * restatement oracle/pcl_oracle.c -- TEST INFRASTRUCTURE: every entry point on small seeded
 * clouds with NaN points, duplicates, collinear samples, empty / tiny inputs.  Exit 0 = clean
 * (a sanitizer report aborts with a non-zero status).  Prints a checksum line. */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../../oracle/pcl_oracle.h"

static uint32_t lcg(uint32_t* s) { *s = *s * 1664525u + 1013904223u; return *s >> 8; }
static float unif(uint32_t* s) { return (float)(lcg(s) & 0xFFFF) / 65535.0f; }

static void make_cloud(float* p, int n, uint32_t seed) {
  uint32_t s = seed;
  for (int i = 0; i < n; ++i) {
    float u = unif(&s) * 4 - 2, v = unif(&s) * 4 - 2, w = (unif(&s) - 0.5f) * 0.01f;
    int k = i % 4;
    if (k == 0) { p[3 * i] = u; p[3 * i + 1] = v; p[3 * i + 2] = 0.5f + w; }
    else if (k == 1) { p[3 * i] = u; p[3 * i + 1] = -0.3f + w; p[3 * i + 2] = v; }
    else if (k == 2) { p[3 * i] = 0.7f + w; p[3 * i + 1] = u; p[3 * i + 2] = v; }
    else { p[3 * i] = u; p[3 * i + 1] = v; p[3 * i + 2] = unif(&s) * 2 - 1; }
  }
  for (int i = 13; i < n; i += 97) p[3 * i + 1] = NAN;
  if (n > 20) memcpy(p + 3 * 20, p + 3 * 19, 12); /* a duplicate */
}

int main(void) {
  double sum = 0;
  const int N = 3000;
  float* p = malloc(sizeof(float) * 3 * N);
  make_cloud(p, N, 7);
  int32_t* inl = malloc(sizeof(int32_t) * N);
  for (int mode = 0; mode < 3; ++mode)
    for (int n = 0; n <= N; n = n ? n * 4 : 1) {
      orc_sac_params prm;
      memset(&prm, 0, sizeof(prm));
      prm.threshold = 0.02; prm.max_iterations = 200; prm.probability = 0.99; prm.optimize = 1;
      prm.seed = 12345u; prm.refit_double = mode; prm.fast_qexp = ORC_QEXP_AUTO;
      float c[4]; int64_t nin = 0; orc_sac_stats st;
      orc_sac_segment(p, n, 3, NULL, n, &prm, c, inl, &nin, &st);
      sum += (double)nin + st.iterations;
    }
  {
    orc_sac_params prm;
    memset(&prm, 0, sizeof(prm));
    prm.threshold = 0.02; prm.max_iterations = 100; prm.probability = 1.0; prm.optimize = 1;
    prm.seed = 12345u; prm.refit_double = 2; prm.fast_qexp = ORC_QEXP_AUTO;
    float co[4 * 6]; int64_t off[7]; int np = 0;
    orc_extract_planes(p, N, 3, &prm, 6, 50, co, off, inl, &np);
    sum += np + (double)off[np];
  }
  float* nrm = malloc(sizeof(float) * 4 * N);
  const float vp[3] = {0, 0, 0};
  orc_estimate_normals(p, N, 3, 0.2f, vp, nrm);
  orc_estimate_normals_knn(p, 800, 3, 20, vp, nrm);
  orc_estimate_normals(p, N, 3, 0.2f, vp, nrm);
  for (int i = 0; i < N; ++i) sum += isnan(nrm[4 * i]) ? 0 : nrm[4 * i + 3];
  {
    orc_sac_params prm;
    memset(&prm, 0, sizeof(prm));
    prm.threshold = 0.05; prm.max_iterations = 100; prm.probability = 0.99; prm.optimize = 1;
    prm.seed = 12345u; prm.model = ORC_SACMODEL_NORMAL_PLANE; prm.normal_distance_weight = 0.1;
    prm.normals = nrm; prm.fast_qexp = ORC_QEXP_AUTO;
    float c[4]; int64_t nin = 0; orc_sac_stats st;
    orc_sac_segment(p, N, 3, NULL, N, &prm, c, inl, &nin, &st);
    sum += (double)nin;
  }
  uint8_t* proc = malloc(N);
  sum += (double)orc_regulate_normals(p, N, 3, nrm, 0, 0, 0.15f, proc);
  sum += (double)orc_regulate_normals(p, N, 3, nrm, -1, 1, 0.15f, proc);
  float* out = malloc(sizeof(float) * 3 * N);
  float tr[3];
  sum += (double)orc_preprocess(p, N, 3, 1, 0.01f, out, inl, tr);
  sum += (double)orc_preprocess(p, 0, 3, 1, 0.01f, out, inl, tr);
  orc_orient_normals_nn(p, 500, 3, nrm, p + 3 * 500, 400, 3, nrm + 4 * 500);
  /* post-process: two square borders, points_set = a few cloud points */
  float border[2 * 4 * 3] = {-1, -1, 0.5f, 1, -1, 0.5f, 1, 1, 0.5f, -1, 1, 0.5f,
                             -1, -0.3f, -1, 1, -0.3f, -1, 1, -0.3f, 1, -1, -0.3f, 1};
  int64_t boff[3] = {0, 4, 8}, poff[3] = {0, 40, 80};
  float pts[80 * 3];
  for (int k = 0; k < 80; ++k) memcpy(pts + 3 * k, p + 3 * (k < 40 ? 4 * k : 4 * (k - 40) + 1), 12);
  float cin[8] = {0, 0, 1, 0, 0, 1, 0, 0}, cout[8];
  uint8_t* ab = malloc(2 * N);
  uint8_t* rem = malloc(N);
  orc_post_process_planes(p, N, 3, 2, cin, pts, 3, poff, border, 3, boff, 0.1f, 0, 4242u, 0.1f, 5,
                          cout, ab, rem);
  for (int i = 0; i < N; ++i) sum += ab[i] + ab[N + i] + rem[i];
  uint8_t* valid = malloc(N);
  orc_cluster_filter(p, N, 3, 0.05f, 3, valid);
  for (int i = 0; i < N; ++i) sum += valid[i];
  printf("checksum %.6f\n", sum);
  free(p); free(inl); free(nrm); free(proc); free(out); free(ab); free(rem); free(valid);
  return 0;
}
