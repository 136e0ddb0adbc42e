/*
 * dpvo_oracle.c -- TEST INFRASTRUCTURE ONLY.
 *
 * A plain-C CPU restatement of the reference DPVO hot path (cuteboyqq/DPVO,
 * mounted read-only at /root/reference).  It exists so that tests/,
 * __graft_entry__.smoke() and bench.py's `cpu_baseline` leg can CHECK the
 * MI355X HIP path; it is never linked into, loaded by, or called from the
 * product path (dpvo_amd/ fails loudly when its HIP extension is missing).
 *
 * Pinning (see DESIGN.md "Oracle"):
 *   - A-CORR / A-PATCH are pinned against golden vectors produced by the
 *     reference's own Python restatements (dpvo/altcorr/correlation_kernel.py:
 *     corr_forward_torch_wrapper 388-458, patchify_forward_kernel_CPU 141-178),
 *     committed under tests/golden/ by oracle/make_golden.py.
 *   - F-BA is pinned against dpvo/ba.py (BA 88-297) run on inputs where the ten
 *     ba.py <-> ba_cuda.cu divergences (SURVEY.md 8a, A-BA-PY) are inert.
 *   - L-SE3 is pinned by the reference's property tests
 *     (dpvo/lietorch/run_tests.py) and by scipy.linalg.expm of the 4x4 hat.
 *
 * Accumulation: the reference accumulates with unordered fp32 atomics
 * (non-deterministic).  The oracle accumulates every reduction in double in
 * a fixed order and keeps the per-element fp32 arithmetic of the reference.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define ORC_API __attribute__((visibility("default")))

/* ------------------------------------------------------------------------ */
/* A-CORR: corr_forward_kernel  correlation_kernel.cu:82-175                 */
/*         host bilinear+permute correlation_kernel.cu:232-272              */
/* ------------------------------------------------------------------------ */

static inline int within_bounds(int h, int w, int H, int W) {
  /* correlation_kernel.cu:11-14 */
  return h >= 0 && h < H && w >= 0 && w < W;
}

static inline int ifloor(float v) {
  /* static_cast<int>(floor(v)) (correlation_kernel.cu:156-157); values outside
     int range are clamped far out of bounds (the reference is UB there). */
  float f = floorf(v);
  if (!(f > -1.0e8f)) return -100000000;
  if (f > 1.0e8f) return 100000000;
  return (int)f;
}

/* raw[b][m][yy][xx][i0][j0], D = 2R+2 (correlation_kernel.cu:118-173) */
static void corr_raw(const float* f1, const float* f2, const float* coords, const int64_t* us,
                     const int64_t* vs, int B, int M, int C, int H, int W, int N1, int N2, int H2,
                     int W2, int R, float* raw) {
  const int D = 2 * R + 2;
  for (int b = 0; b < B; b++)
    for (int m = 0; m < M; m++) {
      const int64_t ix = us[m], jx = vs[m];
      for (int i0 = 0; i0 < H; i0++)
        for (int j0 = 0; j0 < W; j0++) {
          const float x = coords[((((size_t)b * M + m) * 2 + 0) * H + i0) * W + j0];
          const float y = coords[((((size_t)b * M + m) * 2 + 1) * H + i0) * W + j0];
          for (int yy = 0; yy < D; yy++)
            for (int xx = 0; xx < D; xx++) {
              const int i1 = ifloor(y) + (yy - R);
              const int j1 = ifloor(x) + (xx - R);
              double s = 0.0;
              if (within_bounds(i1, j1, H2, W2) && ix >= 0 && ix < N1 && jx >= 0 && jx < N2) {
                for (int c = 0; c < C; c++) {
                  const float a = f1[((((size_t)b * N1 + ix) * C + c) * H + i0) * W + j0];
                  const float v = f2[((((size_t)b * N2 + jx) * C + c) * H2 + i1) * W2 + j1];
                  s += (double)a * (double)v;
                }
              }
              raw[(((((size_t)b * M + m) * D + yy) * D + xx) * H + i0) * W + j0] = (float)s;
            }
        }
    }
}

/* out[b][m][xx][yy][i0][j0] (after permute(0,1,3,2,4,5)), xx,yy in [0, 2R+1) */
ORC_API int orc_corr_fwd(const float* fmap1, const float* fmap2, const float* coords,
                         const int64_t* ii, const int64_t* jj, int B, int M, int C, int H, int W,
                         int N1, int N2, int H2, int W2, int R, float* out) {
  const int D = 2 * R + 2, Dp = D - 1;
  float* raw = (float*)malloc(sizeof(float) * (size_t)B * M * D * D * H * W);
  if (!raw) return -1;
  corr_raw(fmap1, fmap2, coords, ii, jj, B, M, C, H, W, N1, N2, H2, W2, R, raw);
  for (int b = 0; b < B; b++)
    for (int m = 0; m < M; m++)
      for (int i0 = 0; i0 < H; i0++)
        for (int j0 = 0; j0 < W; j0++) {
          const float x = coords[((((size_t)b * M + m) * 2 + 0) * H + i0) * W + j0];
          const float y = coords[((((size_t)b * M + m) * 2 + 1) * H + i0) * W + j0];
          const float dx = x - floorf(x), dy = y - floorf(y); /* cu:260-263 */
          for (int a = 0; a < Dp; a++)     /* y offset (first raw window axis) */
            for (int c = 0; c < Dp; c++) { /* x offset */
#define RAW(YY, XX) raw[(((((size_t)b * M + m) * D + (YY)) * D + (XX)) * H + i0) * W + j0]
              /* cu:266-269, evaluated left to right as ATen does */
              float o = ((1.0f - dx) * (1.0f - dy)) * RAW(a, c);
              o = o + (dx * (1.0f - dy)) * RAW(a, c + 1);
              o = o + ((1.0f - dx) * dy) * RAW(a + 1, c);
              o = o + (dx * dy) * RAW(a + 1, c + 1);
#undef RAW
              out[(((((size_t)b * M + m) * Dp + c) * Dp + a) * H + i0) * W + j0] = o;
            }
        }
  free(raw);
  return 0;
}

/* A-CORR-BWD: corr_backward_kernel correlation_kernel.cu:178-229, host 275-325.
   grad is in the forward output layout [B,M,Dp(x),Dp(y),H,W]. */
ORC_API int orc_corr_bwd(const float* fmap1, const float* fmap2, const float* coords,
                         const int64_t* ii, const int64_t* jj, const float* grad, int B, int M,
                         int C, int H, int W, int N1, int N2, int H2, int W2, int R,
                         float* fmap1_grad, float* fmap2_grad) {
  const int D = 2 * R + 2, Dp = D - 1;
  const size_t n1 = (size_t)B * N1 * C * H * W, n2 = (size_t)B * N2 * C * H2 * W2;
  double* g1 = (double*)calloc(n1, sizeof(double));
  double* g2 = (double*)calloc(n2, sizeof(double));
  if (!g1 || !g2) { free(g1); free(g2); return -1; }
  for (int b = 0; b < B; b++)
    for (int m = 0; m < M; m++) {
      const int64_t ix = ii[m], jx = jj[m];
      if (ix < 0 || ix >= N1 || jx < 0 || jx >= N2) continue;
      for (int i0 = 0; i0 < H; i0++)
        for (int j0 = 0; j0 < W; j0++) {
          const float x = coords[((((size_t)b * M + m) * 2 + 0) * H + i0) * W + j0];
          const float y = coords[((((size_t)b * M + m) * 2 + 1) * H + i0) * W + j0];
          const float dx = x - floorf(x), dy = y - floorf(y); /* cu:292-295 */
          for (int yy = 0; yy < D; yy++)
            for (int xx = 0; xx < D; xx++) {
              /* corr_grad = g1 + g2 + g3 + g4 (cu:303-308) */
#define GP(A, Cc) grad[(((((size_t)b * M + m) * Dp + (Cc)) * Dp + (A)) * H + i0) * W + j0]
              float t1 = 0.f, t2 = 0.f, t3 = 0.f, t4 = 0.f;
              if (yy < Dp && xx < Dp) t1 = ((1.0f - dx) * (1.0f - dy)) * GP(yy, xx);
              if (yy < Dp && xx >= 1) t2 = (dx * (1.0f - dy)) * GP(yy, xx - 1);
              if (yy >= 1 && xx < Dp) t3 = ((1.0f - dx) * dy) * GP(yy - 1, xx);
              if (yy >= 1 && xx >= 1) t4 = (dx * dy) * GP(yy - 1, xx - 1);
#undef GP
              const float g = ((t1 + t2) + t3) + t4;
              const int i1 = ifloor(y) + (yy - R);
              const int j1 = ifloor(x) + (xx - R);
              if (!within_bounds(i1, j1, H2, W2)) continue;
              for (int c = 0; c < C; c++) {
                const size_t o1 = ((((size_t)b * N1 + ix) * C + c) * H + i0) * W + j0;
                const size_t o2 = ((((size_t)b * N2 + jx) * C + c) * H2 + i1) * W2 + j1;
                g1[o1] += (double)g * (double)fmap2[o2];
                g2[o2] += (double)g * (double)fmap1[o1];
              }
            }
        }
    }
  for (size_t i = 0; i < n1; i++) fmap1_grad[i] = (float)g1[i];
  for (size_t i = 0; i < n2; i++) fmap2_grad[i] = (float)g2[i];
  free(g1);
  free(g2);
  return 0;
}

/* A-PATCH: patchify_forward_kernel correlation_kernel.cu:16-47 (clamp=0, zero
   fill) or the fork's runtime patchify_forward_kernel_python
   correlation_kernel.py:181-224 (clamp=1). net [B,C,H,W], coords [B,M,2],
   out [B,M,C,D,D] with D=2R+2. */
ORC_API int orc_patchify_fwd(const float* net, const float* coords, int B, int C, int H, int W,
                             int M, int R, int clamp, float* out) {
  const int D = 2 * R + 2;
  for (int b = 0; b < B; b++)
    for (int m = 0; m < M; m++) {
      const float x = coords[((size_t)b * M + m) * 2 + 0];
      const float y = coords[((size_t)b * M + m) * 2 + 1];
      for (int c = 0; c < C; c++)
        for (int yy = 0; yy < D; yy++)
          for (int xx = 0; xx < D; xx++) {
            int i = ifloor(y) + (yy - R), j = ifloor(x) + (xx - R);
            float v = 0.f;
            if (clamp) {
              i = i < 0 ? 0 : (i > H - 1 ? H - 1 : i);
              j = j < 0 ? 0 : (j > W - 1 ? W - 1 : j);
              v = net[(((size_t)b * C + c) * H + i) * W + j];
            } else if (within_bounds(i, j, H, W)) {
              v = net[(((size_t)b * C + c) * H + i) * W + j];
            }
            out[((((size_t)b * M + m) * C + c) * D + yy) * D + xx] = v;
          }
    }
  return 0;
}

/* A-PATCH-BWD: patchify_backward_kernel correlation_kernel.cu:49-80 (clamp=0)
   or correlation_kernel.py:242-287 (clamp=1). */
ORC_API int orc_patchify_bwd(const float* grad, const float* coords, int B, int C, int H, int W,
                             int M, int R, int clamp, float* net_grad) {
  const int D = 2 * R + 2;
  const size_t n = (size_t)B * C * H * W;
  double* acc = (double*)calloc(n, sizeof(double));
  if (!acc) return -1;
  for (int b = 0; b < B; b++)
    for (int m = 0; m < M; m++) {
      const float x = coords[((size_t)b * M + m) * 2 + 0];
      const float y = coords[((size_t)b * M + m) * 2 + 1];
      for (int yy = 0; yy < D; yy++)
        for (int xx = 0; xx < D; xx++) {
          int i = ifloor(y) + (yy - R), j = ifloor(x) + (xx - R);
          if (clamp) {
            i = i < 0 ? 0 : (i > H - 1 ? H - 1 : i);
            j = j < 0 ? 0 : (j > W - 1 ? W - 1 : j);
          } else if (!within_bounds(i, j, H, W)) {
            continue;
          }
          for (int c = 0; c < C; c++)
            acc[(((size_t)b * C + c) * H + i) * W + j] +=
                grad[((((size_t)b * M + m) * C + c) * D + yy) * D + xx];
        }
    }
  for (size_t i = 0; i < n; i++) net_grad[i] = (float)acc[i];
  free(acc);
  return 0;
}

/* ------------------------------------------------------------------------ */
/* fastba device helpers restated: ba_cuda.cu:36-174                        */
/* ------------------------------------------------------------------------ */

static void actSO3(const float* q, const float* X, float* Y) { /* ba_cuda.cu:36-46 */
  float uv[3];
  uv[0] = 2.0f * (q[1] * X[2] - q[2] * X[1]);
  uv[1] = 2.0f * (q[2] * X[0] - q[0] * X[2]);
  uv[2] = 2.0f * (q[0] * X[1] - q[1] * X[0]);
  Y[0] = X[0] + q[3] * uv[0] + (q[1] * uv[2] - q[2] * uv[1]);
  Y[1] = X[1] + q[3] * uv[1] + (q[2] * uv[0] - q[0] * uv[2]);
  Y[2] = X[2] + q[3] * uv[2] + (q[0] * uv[1] - q[1] * uv[0]);
}

static void actSE3(const float* t, const float* q, const float* X, float* Y) { /* :48-55 */
  actSO3(q, X, Y);
  Y[3] = X[3];
  Y[0] += X[3] * t[0];
  Y[1] += X[3] * t[1];
  Y[2] += X[3] * t[2];
}

static void adjSE3(const float* t, const float* q, const float* X, float* Y) { /* :57-72 */
  float qinv[4] = {-q[0], -q[1], -q[2], q[3]};
  actSO3(qinv, &X[0], &Y[0]);
  actSO3(qinv, &X[3], &Y[3]);
  float u[3], v[3];
  u[0] = t[2] * X[1] - t[1] * X[2];
  u[1] = t[0] * X[2] - t[2] * X[0];
  u[2] = t[1] * X[0] - t[0] * X[1];
  actSO3(qinv, u, v);
  Y[3] += v[0];
  Y[4] += v[1];
  Y[5] += v[2];
}

static void relSE3(const float* ti, const float* qi, const float* tj, const float* qj, float* tij,
                   float* qij) { /* :74-85 */
  qij[0] = -qj[3] * qi[0] + qj[0] * qi[3] - qj[1] * qi[2] + qj[2] * qi[1];
  qij[1] = -qj[3] * qi[1] + qj[1] * qi[3] - qj[2] * qi[0] + qj[0] * qi[2];
  qij[2] = -qj[3] * qi[2] + qj[2] * qi[3] - qj[0] * qi[1] + qj[1] * qi[0];
  qij[3] = qj[3] * qi[3] + qj[0] * qi[0] + qj[1] * qi[1] + qj[2] * qi[2];
  actSO3(qij, ti, tij);
  tij[0] = tj[0] - tij[0];
  tij[1] = tj[1] - tij[1];
  tij[2] = tj[2] - tij[2];
}

static void expSO3f(const float* phi, float* q) { /* :88-110 */
  float theta_sq = phi[0] * phi[0] + phi[1] * phi[1] + phi[2] * phi[2];
  float theta_p4 = theta_sq * theta_sq;
  float theta = sqrtf(theta_sq);
  float imag, real;
  if (theta_sq < 1e-8) {
    imag = (float)(0.5 - (1.0 / 48.0) * theta_sq + (1.0 / 3840.0) * theta_p4);
    real = (float)(1.0 - (1.0 / 8.0) * theta_sq + (1.0 / 384.0) * theta_p4);
  } else {
    imag = sinf(0.5f * theta) / theta;
    real = cosf(0.5f * theta);
  }
  q[0] = imag * phi[0];
  q[1] = imag * phi[1];
  q[2] = imag * phi[2];
  q[3] = real;
}

static void crossInplace(const float* a, float* b) { /* :112-123 */
  float x[3] = {a[1] * b[2] - a[2] * b[1], a[2] * b[0] - a[0] * b[2], a[0] * b[1] - a[1] * b[0]};
  b[0] = x[0];
  b[1] = x[1];
  b[2] = x[2];
}

static void expSE3f(const float* xi, float* t, float* q) { /* :125-153 */
  expSO3f(xi + 3, q);
  float tau[3] = {xi[0], xi[1], xi[2]};
  float phi[3] = {xi[3], xi[4], xi[5]};
  float theta_sq = phi[0] * phi[0] + phi[1] * phi[1] + phi[2] * phi[2];
  float theta = sqrtf(theta_sq);
  t[0] = tau[0];
  t[1] = tau[1];
  t[2] = tau[2];
  if (theta > 1e-4) {
    float a = (1 - cosf(theta)) / theta_sq;
    crossInplace(phi, tau);
    t[0] += a * tau[0];
    t[1] += a * tau[1];
    t[2] += a * tau[2];
    float b = (theta - sinf(theta)) / (theta * theta_sq);
    crossInplace(phi, tau);
    t[0] += b * tau[0];
    t[1] += b * tau[1];
    t[2] += b * tau[2];
  }
}

static void retrSE3(const float* xi, const float* t, const float* q, float* t1,
                    float* q1) { /* :156-174 */
  float dt[3] = {0, 0, 0};
  float dq[4] = {0, 0, 0, 1};
  expSE3f(xi, dt, dq);
  q1[0] = dq[3] * q[0] + dq[0] * q[3] + dq[1] * q[2] - dq[2] * q[1];
  q1[1] = dq[3] * q[1] + dq[1] * q[3] + dq[2] * q[0] - dq[0] * q[2];
  q1[2] = dq[3] * q[2] + dq[2] * q[3] + dq[0] * q[1] - dq[1] * q[0];
  q1[3] = dq[3] * q[3] - dq[0] * q[0] - dq[1] * q[1] - dq[2] * q[2];
  actSO3(dq, t, t1);
  t1[0] += dt[0];
  t1[1] += dt[1];
  t1[2] += dt[2];
}

/* F-REPROJ: reproject kernel ba_cuda.cu:379-429, host 585-616.
   poses [*,7], patches [*,3,P,P], coords out [E,2,P,P]. intrinsics row 0 only. */
ORC_API int orc_reproject(const float* poses, const float* patches, const float* intrinsics,
                          const int64_t* ii, const int64_t* jj, const int64_t* kk, int E, int P,
                          float* coords) {
  const float fx = intrinsics[0], fy = intrinsics[1], cx = intrinsics[2], cy = intrinsics[3];
  for (int n = 0; n < E; n++) {
    const float* pi = poses + 7 * ii[n];
    const float* pj = poses + 7 * jj[n];
    float tij[3], qij[4];
    relSE3(pi, pi + 3, pj, pj + 3, tij, qij);
    const float* pk = patches + (size_t)kk[n] * 3 * P * P;
    for (int i = 0; i < P; i++)
      for (int j = 0; j < P; j++) {
        float Xi[4], Xj[4];
        Xi[0] = (pk[0 * P * P + i * P + j] - cx) / fx;
        Xi[1] = (pk[1 * P * P + i * P + j] - cy) / fy;
        Xi[2] = 1.0f;
        Xi[3] = pk[2 * P * P + i * P + j];
        actSE3(tij, qij, Xi, Xj);
        coords[(((size_t)n * 2 + 0) * P + i) * P + j] = fx * (Xj[0] / Xj[2]) + cx;
        coords[(((size_t)n * 2 + 1) * P + i) * P + j] = fy * (Xj[1] / Xj[2]) + cy;
      }
  }
  return 0;
}

/* F-NBR: neighbors ba.cpp:59-97 (called as neighbors(kk, jj) by DPVO).  Edges
   grouped by ii value; inside a group stable-sorted by jj; ix = previous edge,
   jx = next edge, -1 at the ends. */
static const int64_t* g_sort_key;
static int cmp_stable_jj(const void* a, const void* b) {
  const int64_t ia = *(const int64_t*)a, ib = *(const int64_t*)b;
  const int64_t ka = g_sort_key[ia], kb = g_sort_key[ib];
  if (ka != kb) return ka < kb ? -1 : 1;
  return ia < ib ? -1 : (ia > ib); /* stable: original order */
}
static const int64_t* g_grp_key;
static int cmp_group(const void* a, const void* b) {
  const int64_t ia = *(const int64_t*)a, ib = *(const int64_t*)b;
  const int64_t ka = g_grp_key[ia], kb = g_grp_key[ib];
  if (ka != kb) return ka < kb ? -1 : 1;
  const int64_t ja = g_sort_key[ia], jb = g_sort_key[ib];
  if (ja != jb) return ja < jb ? -1 : 1;
  return ia < ib ? -1 : (ia > ib);
}
ORC_API int orc_neighbors(const int64_t* ii, const int64_t* jj, int E, int64_t* ix, int64_t* jx) {
  int64_t* order = (int64_t*)malloc(sizeof(int64_t) * (E > 0 ? E : 1));
  if (!order) return -1;
  for (int i = 0; i < E; i++) order[i] = i;
  g_grp_key = ii;
  g_sort_key = jj;
  qsort(order, E, sizeof(int64_t), cmp_group);
  int s = 0;
  while (s < E) {
    int e = s;
    while (e < E && ii[order[e]] == ii[order[s]]) e++;
    for (int k = s; k < e; k++) {
      ix[order[k]] = (k > s) ? order[k - 1] : -1;
      jx[order[k]] = (k < e - 1) ? order[k + 1] : -1;
    }
    s = e;
  }
  free(order);
  return 0;
}

/* ------------------------------------------------------------------------ */
/* F-BA: cuda_ba ba_cuda.cu:433-582 (dense Schur path; the eff_impl path of   */
/* block_e.cu computes the same S = B - E Q E^T and differs only in fp32     */
/* summation order).  Per-edge arithmetic is fp32 exactly as                 */
/* reprojection_residuals_and_hessian (ba_cuda.cu:232-376); every reduction  */
/* and the Cholesky solve run in double.                                     */
/* ------------------------------------------------------------------------ */

static int cmp_i64(const void* a, const void* b) {
  const int64_t x = *(const int64_t*)a, y = *(const int64_t*)b;
  return x < y ? -1 : (x > y);
}

/* returns number of unique values; kx sorted unique, ku inverse index */
static int unique_inverse(const int64_t* kk, int E, int64_t* kx, int64_t* ku) {
  int64_t* tmp = (int64_t*)malloc(sizeof(int64_t) * (E > 0 ? E : 1));
  memcpy(tmp, kk, sizeof(int64_t) * E);
  qsort(tmp, E, sizeof(int64_t), cmp_i64);
  int M = 0;
  for (int i = 0; i < E; i++)
    if (i == 0 || tmp[i] != tmp[i - 1]) kx[M++] = tmp[i];
  for (int i = 0; i < E; i++) {
    int lo = 0, hi = M - 1;
    while (lo < hi) {
      int mid = (lo + hi) / 2;
      if (kx[mid] < kk[i]) lo = mid + 1; else hi = mid;
    }
    ku[i] = lo;
  }
  free(tmp);
  return M;
}

/* dense Cholesky S = L L^T (lower, in place); returns 0 on success */
static int cholesky_d(double* S, int n) {
  for (int j = 0; j < n; j++) {
    double d = S[j * n + j];
    for (int k = 0; k < j; k++) d -= S[j * n + k] * S[j * n + k];
    if (!(d > 0.0)) return j + 1;
    d = sqrt(d);
    S[j * n + j] = d;
    for (int i = j + 1; i < n; i++) {
      double s = S[i * n + j];
      for (int k = 0; k < j; k++) s -= S[i * n + k] * S[j * n + k];
      S[i * n + j] = s / d;
    }
  }
  return 0;
}

static void chol_solve_d(const double* L, int n, double* y) {
  for (int i = 0; i < n; i++) {
    double s = y[i];
    for (int k = 0; k < i; k++) s -= L[i * n + k] * y[k];
    y[i] = s / L[i * n + i];
  }
  for (int i = n - 1; i >= 0; i--) {
    double s = y[i];
    for (int k = i + 1; k < n; k++) s -= L[k * n + i] * y[k];
    y[i] = s / L[i * n + i];
  }
}

/* Per-edge linearisation, ba_cuda.cu:265-333.  Writes the fp32 quantities
   used by the accumulation: w[2], r[2], Jz[2], Ji[2][6], Jj[2][6]. */
static void edge_linearize(const float* poses, const float* patches, int P, float fx, float fy,
                           float cx, float cy, const float* target, const float* weight, int64_t ix,
                           int64_t jx, int64_t kx, float w[2], float r[2], float Jz[2],
                           float Ji[2][6], float Jj[2][6]) {
  const float* pi = poses + 7 * ix;
  const float* pj = poses + 7 * jx;
  const float* pk = patches + (size_t)kx * 3 * P * P;
  const int c11 = 1 * P + 1; /* patches[kx][*][1][1] (ba_cuda.cu:282-285) */
  float Xi[4], Xj[4];
  Xi[0] = (pk[0 * P * P + c11] - cx) / fx;
  Xi[1] = (pk[1 * P * P + c11] - cy) / fy;
  Xi[2] = 1.0f;
  Xi[3] = pk[2 * P * P + c11];
  float tij[3], qij[4];
  relSE3(pi, pi + 3, pj, pj + 3, tij, qij);
  actSE3(tij, qij, Xi, Xj);
  const float X = Xj[0], Y = Xj[1], Z = Xj[2], W = Xj[3];
  const float d = ((double)Z >= 0.2) ? (float)(1.0 / (double)Z) : 0.0f;
  const float d2 = d * d;
  const float x1 = fx * (X / Z) + cx;
  const float y1 = fy * (Y / Z) + cy;
  const float rx = target[0] - x1;
  const float ry = target[1] - y1;
  const int in_bounds = (sqrtf(rx * rx + ry * ry) < 128) && ((double)Z > 0.2) && (x1 > -64) &&
                        (y1 > -64) && (x1 < 2 * cx + 64) && (y1 < 2 * cy + 64);
  const float mask = in_bounds ? 1.0f : 0.0f;
  /* row 0 (ba_cuda.cu:317-324) */
  r[0] = target[0] - x1;
  w[0] = mask * weight[0];
  Jz[0] = fx * (tij[0] * d - tij[2] * (X * d2));
  Jj[0][0] = fx * W * d; Jj[0][1] = 0; Jj[0][2] = fx * -X * W * d2;
  Jj[0][3] = fx * -X * Y * d2; Jj[0][4] = fx * (1 + X * X * d2); Jj[0][5] = fx * -Y * d;
  /* row 1 (ba_cuda.cu:325-332) */
  r[1] = target[1] - y1;
  w[1] = mask * weight[1];
  Jz[1] = fy * (tij[1] * d - tij[2] * (Y * d2));
  Jj[1][0] = 0; Jj[1][1] = fy * W * d; Jj[1][2] = fy * -Y * W * d2;
  Jj[1][3] = fy * (-1 - Y * Y * d2); Jj[1][4] = fy * (X * Y * d2); Jj[1][5] = fy * X * d;
  adjSE3(tij, qij, Jj[0], Ji[0]); /* ba_cuda.cu:337 */
  adjSE3(tij, qij, Jj[1], Ji[1]);
}

/* Runs `iterations` LM/Schur steps in place on poses and patches.
   poses [*,7], patches [*,3,P,P], intrinsics row 0, target/weight [E,2].
   Optional diagnostics of the LAST iteration: dX_out [6N], dZ_out [M_u],
   S_out [(6N)^2] (damped Schur matrix before factorisation), y_out [6N].
   Returns 0, or 1 + column on a failed Cholesky (then dX = 0, as
   dpvo/ba.py:17-21 does; ba_cuda.cu does not check info). */
/* Edge-sharded form, same arithmetic: only edges whose patch
   belongs to a source frame kk / PPF in [own_lo, own_hi) are linearised, and
   only those patches are retracted.  phase 0: full iterations (orc_ba);
   phase 1: one linearisation -> this rank's UNDAMPED S_io [(6N)^2], y_io [6N];
   phase 2: one step from the GLOBAL (summed, undamped) S_io / y_io: damp,
   factorise, dX, dZ of owned patches, retractions. */
static int ba_core(float* poses, float* patches, const float* intrinsics, const float* target,
                   const float* weight, float lmbda, const int64_t* ii, const int64_t* jj,
                   const int64_t* kk, int E, int P, int t0, int t1, int iterations, int PPF,
                   int own_lo, int own_hi, int phase, double* S_io, double* y_io, double* dX_out,
                   double* dZ_out, double* S_out, double* y_out);

ORC_API int orc_ba(float* poses, float* patches, const float* intrinsics, const float* target,
                   const float* weight, float lmbda, const int64_t* ii, const int64_t* jj,
                   const int64_t* kk, int E, int P, int t0, int t1, int iterations, double* dX_out,
                   double* dZ_out, double* S_out, double* y_out) {
  return ba_core(poses, patches, intrinsics, target, weight, lmbda, ii, jj, kk, E, P, t0, t1,
                 iterations, 1, -0x7fffffff, 0x7fffffff, 0, NULL, NULL, dX_out, dZ_out, S_out,
                 y_out);
}

ORC_API int orc_ba_shard(float* poses, float* patches, const float* intrinsics,
                         const float* target, const float* weight, float lmbda, const int64_t* ii,
                         const int64_t* jj, const int64_t* kk, int E, int P, int t0, int t1,
                         int PPF, int own_lo, int own_hi, int phase, double* S_io, double* y_io) {
  if (phase != 1 && phase != 2) return -1;
  return ba_core(poses, patches, intrinsics, target, weight, lmbda, ii, jj, kk, E, P, t0, t1, 1,
                 PPF, own_lo, own_hi, phase, S_io, y_io, NULL, NULL, NULL, NULL);
}

static int ba_core(float* poses, float* patches, const float* intrinsics, const float* target,
                   const float* weight, float lmbda, const int64_t* ii, const int64_t* jj,
                   const int64_t* kk, int E, int P, int t0, int t1, int iterations, int PPF,
                   int own_lo, int own_hi, int phase, double* S_io, double* y_io, double* dX_out,
                   double* dZ_out, double* S_out, double* y_out) {
  const float fx = intrinsics[0], fy = intrinsics[1], cx = intrinsics[2], cy = intrinsics[3];
  const int N = t1 - t0;
  int64_t* kx = (int64_t*)malloc(sizeof(int64_t) * (E > 0 ? E : 1));
  int64_t* ku = (int64_t*)malloc(sizeof(int64_t) * (E > 0 ? E : 1));
  const int M = unique_inverse(kk, E, kx, ku); /* ba_cuda.cu:447-449 */
  const int n6 = 6 * (N > 0 ? N : 0);
  double* Bm = (double*)calloc((size_t)n6 * n6 + 1, sizeof(double));
  /* E stored transposed, [M][6N]: a patch's nonzero rows are contiguous */
  double* Em = (double*)calloc((size_t)n6 * M + 1, sizeof(double));
  int* nzr = (int*)malloc(sizeof(int) * (n6 + 1));
  double* Cv = (double*)calloc(M + 1, sizeof(double));
  double* v = (double*)calloc(n6 + 1, sizeof(double));
  double* u = (double*)calloc(M + 1, sizeof(double));
  double* Q = (double*)calloc(M + 1, sizeof(double));
  double* S = (double*)calloc((size_t)n6 * n6 + 1, sizeof(double));
  double* y = (double*)calloc(n6 + 1, sizeof(double));
  double* dZ = (double*)calloc(M + 1, sizeof(double));
  int status = 0;

  for (int itr = 0; itr < iterations; itr++) {
    memset(Bm, 0, sizeof(double) * n6 * n6);
    memset(Em, 0, sizeof(double) * n6 * M);
    memset(Cv, 0, sizeof(double) * M);
    memset(v, 0, sizeof(double) * n6);
    memset(u, 0, sizeof(double) * M);
    for (int n = 0; n < E; n++) {
      if (kk[n] / PPF < own_lo || kk[n] / PPF >= own_hi) continue; /* another rank's patch */
      float w[2], r[2], Jz[2], Ji[2][6], Jj[2][6];
      edge_linearize(poses, patches, P, fx, fy, cx, cy, target + 2 * n, weight + 2 * n, ii[n],
                     jj[n], kk[n], w, r, Jz, Ji, Jj);
      const int64_t k = ku[n];
      int64_t ix = ii[n] - t0, jx = jj[n] - t0;
      const int fi = ix >= 0 && ix < N, fj = jx >= 0 && jx < N; /* free poses (ba_cuda.cu:341-345) */
      for (int row = 0; row < 2; row++) {
        const double wr = w[row];
        for (int a = 0; a < 6; a++)
          for (int b = 0; b < 6; b++) { /* ba_cuda.cu:339-350 */
            if (fi) Bm[(6 * ix + a) * n6 + 6 * ix + b] += wr * Ji[row][a] * Ji[row][b];
            if (fj) Bm[(6 * jx + a) * n6 + 6 * jx + b] += wr * Jj[row][a] * Jj[row][b];
            if (fi && fj) {
              Bm[(6 * ix + a) * n6 + 6 * jx + b] -= wr * Ji[row][a] * Jj[row][b];
              Bm[(6 * jx + a) * n6 + 6 * ix + b] -= wr * Jj[row][a] * Ji[row][b];
            }
          }
        for (int a = 0; a < 6; a++) { /* :352-370 */
          if (fi) Em[k * n6 + 6 * ix + a] -= wr * Jz[row] * Ji[row][a];
          if (fj) Em[k * n6 + 6 * jx + a] += wr * Jz[row] * Jj[row][a];
          if (fi) v[6 * ix + a] -= wr * r[row] * Ji[row][a];
          if (fj) v[6 * jx + a] += wr * r[row] * Jj[row][a];
        }
        Cv[k] += wr * Jz[row] * Jz[row]; /* :372-373 */
        u[k] += wr * r[row] * Jz[row];
      }
    }
    for (int k = 0; k < M; k++) Q[k] = 1.0 / (Cv[k] + (double)lmbda); /* :519 */

    if (N <= 0) { /* structure only, :521-531 */
      for (int k = 0; k < M; k++) dZ[k] = Q[k] * u[k];
    } else {
      /* S = B - E Q E^T ; y = v - E Q u (:554-558).  Per entry the patches are
         summed in ascending k; zero terms of E are skipped (exact no-ops). */
      if (phase == 2) {
        memcpy(Bm, S_io, sizeof(double) * n6 * n6);
        memcpy(v, y_io, sizeof(double) * n6);
      }
      memcpy(S, Bm, sizeof(double) * n6 * n6);
      memcpy(y, v, sizeof(double) * n6);
      for (int k = 0; k < M && phase != 2; k++) {
        const double* ek = Em + (size_t)k * n6;
        int nz = 0;
        for (int a = 0; a < n6; a++)
          if (ek[a] != 0.0) nzr[nz++] = a;
        for (int x = 0; x < nz; x++) {
          const int a = nzr[x];
          y[a] -= ek[a] * Q[k] * u[k];
          for (int z = 0; z < nz; z++) {
            const int b = nzr[z];
            S[(size_t)a * n6 + b] -= ek[a] * Q[k] * ek[b];
          }
        }
      }
      if (phase == 1) {
        memcpy(S_io, S, sizeof(double) * n6 * n6);
        memcpy(y_io, y, sizeof(double) * n6);
        break;
      }
      for (int a = 0; a < n6; a++) S[a * n6 + a] += 1e-4 * S[a * n6 + a] + 1.0; /* :560 */
      if (S_out) memcpy(S_out, S, sizeof(double) * n6 * n6);
      if (y_out) memcpy(y_out, y, sizeof(double) * n6);
      int info = cholesky_d(S, n6); /* :561-562 */
      if (info) {
        status = 1 + info;
        for (int a = 0; a < n6; a++) y[a] = 0.0;
      } else {
        chol_solve_d(S, n6, y); /* y <- dX */
      }
      for (int k = 0; k < M; k++) { /* dZ = Q (u - E^T dX) (:563) */
        double s = u[k];
        for (int a = 0; a < n6; a++) s -= Em[(size_t)k * n6 + a] * y[a];
        dZ[k] = Q[k] * s;
      }
      for (int i = 0; i < N; i++) { /* pose_retr_kernel :178-206 */
        float* pt = poses + 7 * (t0 + i);
        float xi[6], t1v[3], q1v[4];
        for (int a = 0; a < 6; a++) xi[a] = (float)y[6 * i + a];
        retrSE3(xi, pt, pt + 3, t1v, q1v);
        pt[0] = t1v[0]; pt[1] = t1v[1]; pt[2] = t1v[2];
        pt[3] = q1v[0]; pt[4] = q1v[1]; pt[5] = q1v[2]; pt[6] = q1v[3];
      }
      if (dX_out) memcpy(dX_out, y, sizeof(double) * n6);
    }
    if (phase == 1) break;
    for (int k = 0; k < M; k++) { /* patch_retr_kernel :209-229 */
      if (kx[k] / PPF < own_lo || kx[k] / PPF >= own_hi) continue;
      float* pk = patches + (size_t)kx[k] * 3 * P * P;
      float d = pk[2 * P * P + 0];
      d = d + (float)dZ[k];
      d = (d > 20) ? 1.0f : d;
      d = (float)fmax((double)d, 1e-4); /* max(float, double) -> double overload */
      for (int a = 0; a < P * P; a++) pk[2 * P * P + a] = d;
    }
    if (dZ_out) memcpy(dZ_out, dZ, sizeof(double) * M);
  }
  free(kx); free(ku); free(Bm); free(Em); free(nzr); free(Cv); free(v); free(u); free(Q); free(S); free(y);
  free(dZ);
  return status;
}

/* ------------------------------------------------------------------------ */
/* L-SE3: lietorch SO3 (group 1) and SE3 (group 3), double precision.        */
/* so3.h:12-225, se3.h:13-226, kernels lietorch_gpu.cu:20-294.               */
/* Quaternions are (x,y,z,w) and normalised on load (so3.h:95-97).           */
/* ------------------------------------------------------------------------ */

#define EPS 1e-6 /* common.h:7 */
#define PI_D 3.14159265358979323846

typedef struct { double q[4]; } so3_t;           /* x y z w */
typedef struct { double t[3]; so3_t r; } se3_t;

static so3_t so3_norm(double x, double y, double z, double w) {
  so3_t r;
  double n = sqrt(x * x + y * y + z * z + w * w);
  r.q[0] = x / n; r.q[1] = y / n; r.q[2] = z / n; r.q[3] = w / n;
  return r;
}
static so3_t so3_load(const double* d) { return so3_norm(d[0], d[1], d[2], d[3]); }
static se3_t se3_load(const double* d) {
  se3_t g; g.t[0] = d[0]; g.t[1] = d[1]; g.t[2] = d[2]; g.r = so3_load(d + 3); return g;
}
static so3_t so3_mul(so3_t a, so3_t b) { /* Hamilton product, then normalise (so3.h:111-113) */
  const double* p = a.q; const double* q = b.q;
  return so3_norm(p[3] * q[0] + p[0] * q[3] + p[1] * q[2] - p[2] * q[1],
                  p[3] * q[1] + p[1] * q[3] + p[2] * q[0] - p[0] * q[2],
                  p[3] * q[2] + p[2] * q[3] + p[0] * q[1] - p[1] * q[0],
                  p[3] * q[3] - p[0] * q[0] - p[1] * q[1] - p[2] * q[2]);
}
static so3_t so3_inv(so3_t a) { return so3_norm(-a.q[0], -a.q[1], -a.q[2], a.q[3]); }
static void cross3(const double* a, const double* b, double* c) {
  c[0] = a[1] * b[2] - a[2] * b[1];
  c[1] = a[2] * b[0] - a[0] * b[2];
  c[2] = a[0] * b[1] - a[1] * b[0];
}
static void so3_act(so3_t a, const double* p, double* out) { /* so3.h:115-120 */
  double uv[3], uv2[3];
  cross3(a.q, p, uv);
  uv[0] += uv[0]; uv[1] += uv[1]; uv[2] += uv[2];
  cross3(a.q, uv, uv2);
  for (int i = 0; i < 3; i++) out[i] = p[i] + a.q[3] * uv[i] + uv2[i];
}
static void so3_matrix(so3_t a, double R[9]) { /* Eigen toRotationMatrix */
  const double x = a.q[0], y = a.q[1], z = a.q[2], w = a.q[3];
  const double tx = 2 * x, ty = 2 * y, tz = 2 * z;
  const double twx = tx * w, twy = ty * w, twz = tz * w;
  const double txx = tx * x, txy = ty * x, txz = tz * x;
  const double tyy = ty * y, tyz = tz * y, tzz = tz * z;
  R[0] = 1 - (tyy + tzz); R[1] = txy - twz; R[2] = txz + twy;
  R[3] = txy + twz; R[4] = 1 - (txx + tzz); R[5] = tyz - twx;
  R[6] = txz - twy; R[7] = tyz + twx; R[8] = 1 - (txx + tyy);
}
static void hat3(const double* p, double H[9]) { /* so3.h:161-169 */
  H[0] = 0; H[1] = -p[2]; H[2] = p[1];
  H[3] = p[2]; H[4] = 0; H[5] = -p[0];
  H[6] = -p[1]; H[7] = p[0]; H[8] = 0;
}
static void mm3(const double* A, const double* B, double* C) {
  for (int i = 0; i < 3; i++)
    for (int j = 0; j < 3; j++) {
      double s = 0;
      for (int k = 0; k < 3; k++) s += A[i * 3 + k] * B[k * 3 + j];
      C[i * 3 + j] = s;
    }
}
static void so3_log(so3_t a, double out[3]) { /* so3.h:175-211 */
  const double sq = a.q[0] * a.q[0] + a.q[1] * a.q[1] + a.q[2] * a.q[2];
  const double w = a.q[3];
  double f;
  if (sq < EPS * EPS) {
    f = 2.0 / w - (2.0 / 3.0) * sq / (w * w * w);
  } else {
    const double n = sqrt(sq);
    if (fabs(w) < EPS) f = (w > 0 ? PI_D : -PI_D) / n;
    else f = 2.0 * atan(n / w) / n;
  }
  for (int i = 0; i < 3; i++) out[i] = f * a.q[i];
}
static so3_t so3_exp(const double* phi) { /* so3.h:213-230 */
  const double t2 = phi[0] * phi[0] + phi[1] * phi[1] + phi[2] * phi[2];
  const double t = sqrt(t2);
  double im, re;
  if (t < EPS) {
    const double t4 = t2 * t2;
    im = 0.5 - (1.0 / 48.0) * t2 + (1.0 / 3840.0) * t4;
    re = 1.0 - (1.0 / 8.0) * t2 + (1.0 / 384.0) * t4;
  } else {
    im = sin(0.5 * t) / t;
    re = cos(0.5 * t);
  }
  return so3_norm(im * phi[0], im * phi[1], im * phi[2], re);
}
static void so3_left_jac(const double* phi, double J[9]) { /* so3.h:232-250 */
  double Ph[9], Ph2[9];
  hat3(phi, Ph);
  mm3(Ph, Ph, Ph2);
  const double t2 = phi[0] * phi[0] + phi[1] * phi[1] + phi[2] * phi[2], t = sqrt(t2);
  const double c1 = (t < EPS) ? 0.5 - (1.0 / 24.0) * t2 : (1.0 - cos(t)) / t2;
  const double c2 = (t < EPS) ? 1.0 / 6.0 - (1.0 / 120.0) * t2 : (t - sin(t)) / (t2 * t);
  for (int i = 0; i < 9; i++) J[i] = (i % 4 == 0 ? 1.0 : 0.0) + c1 * Ph[i] + c2 * Ph2[i];
}
static void so3_left_jac_inv(const double* phi, double J[9]) { /* so3.h:252-268 */
  double Ph[9], Ph2[9];
  hat3(phi, Ph);
  mm3(Ph, Ph, Ph2);
  const double t2 = phi[0] * phi[0] + phi[1] * phi[1] + phi[2] * phi[2], t = sqrt(t2);
  const double ht = 0.5 * t;
  const double c2 = (t < EPS) ? 1.0 / 12.0 : (1.0 - t * cos(ht) / (2.0 * sin(ht))) / (t * t);
  for (int i = 0; i < 9; i++) J[i] = (i % 4 == 0 ? 1.0 : 0.0) - 0.5 * Ph[i] + c2 * Ph2[i];
}
static void se3_calcQ(const double* xi, double Qm[9]) { /* se3.h:133-162 */
  double Ta[9], Ph[9];
  hat3(xi, Ta);
  hat3(xi + 3, Ph);
  const double t = sqrt(xi[3] * xi[3] + xi[4] * xi[4] + xi[5] * xi[5]);
  const double t2 = t * t, t4 = t2 * t2;
  const double c1 = (t < EPS) ? 1.0 / 6.0 - (1.0 / 120.0) * t2 : (t - sin(t)) / (t2 * t);
  const double c2 = (t < EPS) ? 1.0 / 24.0 - (1.0 / 720.0) * t2 : (t2 + 2 * cos(t) - 2) / (2 * t4);
  const double c3 = (t < EPS) ? 1.0 / 120.0 - (1.0 / 2520.0) * t2
                              : (2 * t - 3 * sin(t) + t * cos(t)) / (2 * t4 * t);
  double PT[9], TP[9], PTP[9], PPT[9], TPP[9], PTPP[9], PPTP[9];
  mm3(Ph, Ta, PT); mm3(Ta, Ph, TP); mm3(PT, Ph, PTP);
  mm3(Ph, PT, PPT); mm3(TP, Ph, TPP); mm3(PTP, Ph, PTPP); mm3(Ph, PTP, PPTP);
  for (int i = 0; i < 9; i++)
    Qm[i] = 0.5 * Ta[i] + c1 * (PT[i] + TP[i] + PTP[i]) + c2 * (PPT[i] + TPP[i] - 3 * PTP[i]) +
            c3 * (PTPP[i] + PPTP[i]);
}
/* 6x6 row-major helpers */
static void se3_Adj(se3_t g, double A[36]) { /* se3.h:58-67 (347-356) */
  double R[9], tx[9], tR[9];
  so3_matrix(g.r, R);
  hat3(g.t, tx);
  mm3(tx, R, tR);
  memset(A, 0, sizeof(double) * 36);
  for (int i = 0; i < 3; i++)
    for (int j = 0; j < 3; j++) {
      A[i * 6 + j] = R[i * 3 + j];
      A[i * 6 + 3 + j] = tR[i * 3 + j];
      A[(3 + i) * 6 + 3 + j] = R[i * 3 + j];
    }
}
static void se3_small_adj(const double* xi, double A[36]) { /* se3.h:389-401 */
  double Ta[9], Ph[9];
  hat3(xi, Ta);
  hat3(xi + 3, Ph);
  memset(A, 0, sizeof(double) * 36);
  for (int i = 0; i < 3; i++)
    for (int j = 0; j < 3; j++) {
      A[i * 6 + j] = Ph[i * 3 + j];
      A[i * 6 + 3 + j] = Ta[i * 3 + j];
      A[(3 + i) * 6 + 3 + j] = Ph[i * 3 + j];
    }
}
static void se3_exp(const double* xi, se3_t* g) { /* se3.h:423-431 */
  double J[9];
  g->r = so3_exp(xi + 3);
  so3_left_jac(xi + 3, J);
  for (int i = 0; i < 3; i++) g->t[i] = J[i * 3] * xi[0] + J[i * 3 + 1] * xi[1] + J[i * 3 + 2] * xi[2];
}
static void se3_log(se3_t g, double xi[6]) { /* se3.h:413-421 */
  double Vi[9];
  so3_log(g.r, xi + 3);
  so3_left_jac_inv(xi + 3, Vi);
  for (int i = 0; i < 3; i++) xi[i] = Vi[i * 3] * g.t[0] + Vi[i * 3 + 1] * g.t[1] + Vi[i * 3 + 2] * g.t[2];
}
static void se3_left_jac(const double* xi, double J[36]) { /* se3.h:464-475 */
  double Jr[9], Qm[9];
  so3_left_jac(xi + 3, Jr);
  se3_calcQ(xi, Qm);
  memset(J, 0, sizeof(double) * 36);
  for (int i = 0; i < 3; i++)
    for (int j = 0; j < 3; j++) {
      J[i * 6 + j] = Jr[i * 3 + j];
      J[i * 6 + 3 + j] = Qm[i * 3 + j];
      J[(3 + i) * 6 + 3 + j] = Jr[i * 3 + j];
    }
}
static void se3_left_jac_inv(const double* xi, double J[36]) { /* se3.h:477-490 */
  double Ji[9], Qm[9], T1[9], T2[9];
  so3_left_jac_inv(xi + 3, Ji);
  se3_calcQ(xi, Qm);
  mm3(Ji, Qm, T1);
  mm3(T1, Ji, T2);
  memset(J, 0, sizeof(double) * 36);
  for (int i = 0; i < 3; i++)
    for (int j = 0; j < 3; j++) {
      J[i * 6 + j] = Ji[i * 3 + j];
      J[i * 6 + 3 + j] = -T2[i * 3 + j];
      J[(3 + i) * 6 + 3 + j] = Ji[i * 3 + j];
    }
}
static void so3_store(so3_t r, double* d) { for (int i = 0; i < 4; i++) d[i] = r.q[i]; }
static void se3_store(se3_t g, double* d) {
  d[0] = g.t[0]; d[1] = g.t[1]; d[2] = g.t[2];
  so3_store(g.r, d + 3);
}
static se3_t se3_inv(se3_t g) { /* se3.h:325-327 */
  se3_t o;
  o.r = so3_inv(g.r);
  double t[3];
  so3_act(o.r, g.t, t);
  o.t[0] = -t[0]; o.t[1] = -t[1]; o.t[2] = -t[2];
  return o;
}
static se3_t se3_mul(se3_t a, se3_t b) { /* se3.h:334-336 */
  se3_t o;
  o.r = so3_mul(a.r, b.r);
  double t[3];
  so3_act(a.r, b.t, t);
  for (int i = 0; i < 3; i++) o.t[i] = a.t[i] + t[i];
  return o;
}
/* row-vector times matrix: out[j] = sum_i v[i] M[i][j] */
static void rowvec_mat(const double* v, const double* Mt, int n, int m, double* out) {
  for (int j = 0; j < m; j++) {
    double s = 0;
    for (int i = 0; i < n; i++) s += v[i] * Mt[i * m + j];
    out[j] = s;
  }
}
static void mat_vec(const double* Mt, const double* v, int n, int m, double* out) {
  for (int i = 0; i < n; i++) {
    double s = 0;
    for (int j = 0; j < m; j++) s += Mt[i * m + j] * v[j];
    out[i] = s;
  }
}

/* group ids (dispatch.h:24-45): 1 = SO3, 3 = SE3. */
enum { ORC_OP_EXP = 0, ORC_OP_LOG, ORC_OP_INV, ORC_OP_MUL, ORC_OP_ADJ, ORC_OP_ADJT, ORC_OP_ACT,
       ORC_OP_ACT4, ORC_OP_MATRIX, ORC_OP_PROJ, ORC_OP_JINV };

/* Forward ops over `n` elements.  Shapes (per element):
   EXP: a[K] -> X[N]; LOG: X[N] -> a[K]; INV: X -> Y; MUL: X,Y -> Z;
   ADJ/ADJT/JINV: X[N], a[K] -> b[K]; ACT: X, p[3] -> q[3]; ACT4: X, p[4] -> q[4];
   MATRIX: X -> T[16] (row-major 4x4); PROJ: X -> P[N*N] row-major. */
ORC_API int orc_lie_fwd(int group, int op, int n, const double* x, const double* y, double* out) {
  if (group != 1 && group != 3) return -2;
  const int K = group == 1 ? 3 : 6, N = group == 1 ? 4 : 7;
  for (int e = 0; e < n; e++) {
    if (group == 3) {
      const double* X = x + (size_t)e * (op == ORC_OP_EXP ? K : N);
      se3_t g, h;
      double A[36], Jm[36], b[6];
      switch (op) {
        case ORC_OP_EXP: se3_exp(X, &g); se3_store(g, out + (size_t)e * N); break;
        case ORC_OP_LOG: se3_log(se3_load(X), out + (size_t)e * K); break;
        case ORC_OP_INV: se3_store(se3_inv(se3_load(X)), out + (size_t)e * N); break;
        case ORC_OP_MUL:
          se3_store(se3_mul(se3_load(X), se3_load(y + (size_t)e * N)), out + (size_t)e * N);
          break;
        case ORC_OP_ADJ:
          se3_Adj(se3_load(X), A);
          mat_vec(A, y + (size_t)e * K, 6, 6, out + (size_t)e * K);
          break;
        case ORC_OP_ADJT:
          se3_Adj(se3_load(X), A);
          rowvec_mat(y + (size_t)e * K, A, 6, 6, out + (size_t)e * K);
          break;
        case ORC_OP_ACT: {
          g = se3_load(X);
          double p[3];
          so3_act(g.r, y + (size_t)e * 3, p);
          for (int i = 0; i < 3; i++) out[(size_t)e * 3 + i] = p[i] + g.t[i];
        } break;
        case ORC_OP_ACT4: {
          g = se3_load(X);
          const double* p = y + (size_t)e * 4;
          double q[3];
          so3_act(g.r, p, q);
          for (int i = 0; i < 3; i++) out[(size_t)e * 4 + i] = q[i] + g.t[i] * p[3];
          out[(size_t)e * 4 + 3] = p[3];
        } break;
        case ORC_OP_MATRIX: {
          g = se3_load(X);
          double R[9];
          so3_matrix(g.r, R);
          double* T = out + (size_t)e * 16;
          memset(T, 0, sizeof(double) * 16);
          for (int i = 0; i < 3; i++) {
            for (int j = 0; j < 3; j++) T[i * 4 + j] = R[i * 3 + j];
            T[i * 4 + 3] = g.t[i];
          }
          T[15] = 1.0;
        } break;
        case ORC_OP_PROJ: { /* se3.h:403-411, so3.h:141-151 */
          g = se3_load(X);
          double* Pm = out + (size_t)e * 49;
          memset(Pm, 0, sizeof(double) * 49);
          double H[9], mt[3] = {-g.t[0], -g.t[1], -g.t[2]};
          hat3(mt, H);
          for (int i = 0; i < 3; i++) {
            Pm[i * 7 + i] = 1.0;
            for (int j = 0; j < 3; j++) Pm[i * 7 + 3 + j] = H[i * 3 + j];
          }
          const double* q = g.r.q;
          double mv[3] = {-q[0], -q[1], -q[2]}, Hq[9];
          hat3(mv, Hq);
          for (int i = 0; i < 3; i++)
            for (int j = 0; j < 3; j++)
              Pm[(3 + i) * 7 + 3 + j] = 0.5 * ((i == j ? q[3] : 0.0) + Hq[i * 3 + j]);
          for (int j = 0; j < 3; j++) Pm[6 * 7 + 3 + j] = 0.5 * (-q[j]);
        } break;
        case ORC_OP_JINV: /* lietorch_gpu.cu:282-294 */
          se3_log(se3_load(X), b);
          se3_left_jac_inv(b, Jm);
          mat_vec(Jm, y + (size_t)e * K, 6, 6, out + (size_t)e * K);
          break;
        default: return -3;
      }
      (void)h;
    } else {
      const double* X = x + (size_t)e * (op == ORC_OP_EXP ? K : N);
      so3_t g;
      double R[9], b[3], Jm[9];
      switch (op) {
        case ORC_OP_EXP: so3_store(so3_exp(X), out + (size_t)e * N); break;
        case ORC_OP_LOG: so3_log(so3_load(X), out + (size_t)e * K); break;
        case ORC_OP_INV: so3_store(so3_inv(so3_load(X)), out + (size_t)e * N); break;
        case ORC_OP_MUL:
          so3_store(so3_mul(so3_load(X), so3_load(y + (size_t)e * N)), out + (size_t)e * N);
          break;
        case ORC_OP_ADJ:
          so3_matrix(so3_load(X), R);
          mat_vec(R, y + (size_t)e * K, 3, 3, out + (size_t)e * K);
          break;
        case ORC_OP_ADJT:
          so3_matrix(so3_load(X), R);
          rowvec_mat(y + (size_t)e * K, R, 3, 3, out + (size_t)e * K);
          break;
        case ORC_OP_ACT: so3_act(so3_load(X), y + (size_t)e * 3, out + (size_t)e * 3); break;
        case ORC_OP_ACT4:
          so3_act(so3_load(X), y + (size_t)e * 4, out + (size_t)e * 4);
          out[(size_t)e * 4 + 3] = y[(size_t)e * 4 + 3];
          break;
        case ORC_OP_MATRIX: {
          so3_matrix(so3_load(X), R);
          double* T = out + (size_t)e * 16;
          memset(T, 0, sizeof(double) * 16);
          for (int i = 0; i < 3; i++)
            for (int j = 0; j < 3; j++) T[i * 4 + j] = R[i * 3 + j];
          T[15] = 1.0;
        } break;
        case ORC_OP_PROJ: {
          g = so3_load(X);
          double* Pm = out + (size_t)e * 16;
          memset(Pm, 0, sizeof(double) * 16);
          double mv[3] = {-g.q[0], -g.q[1], -g.q[2]}, Hq[9];
          hat3(mv, Hq);
          for (int i = 0; i < 3; i++)
            for (int j = 0; j < 3; j++)
              Pm[i * 4 + j] = 0.5 * ((i == j ? g.q[3] : 0.0) + Hq[i * 3 + j]);
          for (int j = 0; j < 3; j++) Pm[3 * 4 + j] = 0.5 * (-g.q[j]);
        } break;
        case ORC_OP_JINV:
          so3_log(so3_load(X), b);
          so3_left_jac_inv(b, Jm);
          mat_vec(Jm, y + (size_t)e * K, 3, 3, out + (size_t)e * K);
          break;
        default: return -3;
      }
    }
  }
  return 0;
}

/* Backward ops (lietorch_gpu.cu:32-256).  grad rows use the tangent-padded
   convention of the reference: a gradient w.r.t. a group element is read as
   the first K entries of an N-strided row, and written as K entries into a
   zero-initialised N-strided row.
   EXP: grad[N], a[K] -> da[K]
   LOG: grad[K], X[N] -> dX[N]
   INV: grad[N], X[N] -> dX[N]
   MUL: grad[N], X, Y -> dX[N], dY[N]
   ADJ: grad[K], X, a[K] -> dX[N], da[K]
   ADJT: grad[K], X, a[K] -> dX[N], da[K]
   ACT: grad[3], X, p[3] -> dX[N], dp[3]
   ACT4: grad[4], X, p[4] -> dX[N], dp[4] */
ORC_API int orc_lie_bwd(int group, int op, int n, const double* grad, const double* x,
                        const double* y, double* out0, double* out1) {
  if (group != 3 && group != 1) return -2;
  const int K = group == 1 ? 3 : 6, N = group == 1 ? 4 : 7;
  for (int e = 0; e < n; e++) {
    double A[36], Jm[36], tmp[6], b[6];
    if (group == 3) {
      switch (op) {
        case ORC_OP_EXP:
          se3_left_jac(x + (size_t)e * K, Jm);
          rowvec_mat(grad + (size_t)e * N, Jm, 6, 6, out0 + (size_t)e * K);
          break;
        case ORC_OP_LOG:
          se3_log(se3_load(x + (size_t)e * N), b);
          se3_left_jac_inv(b, Jm);
          memset(out0 + (size_t)e * N, 0, sizeof(double) * N);
          rowvec_mat(grad + (size_t)e * K, Jm, 6, 6, out0 + (size_t)e * N);
          break;
        case ORC_OP_INV:
          se3_Adj(se3_inv(se3_load(x + (size_t)e * N)), A);
          memset(out0 + (size_t)e * N, 0, sizeof(double) * N);
          rowvec_mat(grad + (size_t)e * N, A, 6, 6, tmp);
          for (int i = 0; i < 6; i++) out0[(size_t)e * N + i] = -tmp[i];
          break;
        case ORC_OP_MUL:
          memset(out0 + (size_t)e * N, 0, sizeof(double) * N);
          memset(out1 + (size_t)e * N, 0, sizeof(double) * N);
          for (int i = 0; i < 6; i++) out0[(size_t)e * N + i] = grad[(size_t)e * N + i];
          se3_Adj(se3_load(x + (size_t)e * N), A);
          rowvec_mat(grad + (size_t)e * N, A, 6, 6, out1 + (size_t)e * N);
          break;
        case ORC_OP_ADJ: { /* lietorch_gpu.cu:140-157 */
          se3_Adj(se3_load(x + (size_t)e * N), A);
          mat_vec(A, y + (size_t)e * K, 6, 6, b);
          rowvec_mat(grad + (size_t)e * K, A, 6, 6, out1 + (size_t)e * K);
          se3_small_adj(b, Jm);
          memset(out0 + (size_t)e * N, 0, sizeof(double) * N);
          rowvec_mat(grad + (size_t)e * K, Jm, 6, 6, tmp);
          for (int i = 0; i < 6; i++) out0[(size_t)e * N + i] = -tmp[i];
        } break;
        case ORC_OP_ADJT: { /* lietorch_gpu.cu:173-188 */
          se3_Adj(se3_load(x + (size_t)e * N), A);
          mat_vec(A, grad + (size_t)e * K, 6, 6, b); /* X.Adj(db) */
          for (int i = 0; i < 6; i++) out1[(size_t)e * K + i] = b[i];
          se3_small_adj(b, Jm);
          memset(out0 + (size_t)e * N, 0, sizeof(double) * N);
          rowvec_mat(y + (size_t)e * K, Jm, 6, 6, tmp);
          for (int i = 0; i < 6; i++) out0[(size_t)e * N + i] = -tmp[i];
        } break;
        case ORC_OP_ACT: { /* lietorch_gpu.cu:204-221 */
          se3_t g = se3_load(x + (size_t)e * N);
          double R[9], q[3];
          so3_matrix(g.r, R);
          rowvec_mat(grad + (size_t)e * 3, R, 3, 3, out1 + (size_t)e * 3);
          so3_act(g.r, y + (size_t)e * 3, q);
          for (int i = 0; i < 3; i++) q[i] += g.t[i];
          double J[18], H[9], mq[3] = {-q[0], -q[1], -q[2]};
          hat3(mq, H);
          for (int i = 0; i < 3; i++)
            for (int j = 0; j < 3; j++) {
              J[i * 6 + j] = (i == j);
              J[i * 6 + 3 + j] = H[i * 3 + j];
            }
          memset(out0 + (size_t)e * N, 0, sizeof(double) * N);
          rowvec_mat(grad + (size_t)e * 3, J, 3, 6, out0 + (size_t)e * N);
        } break;
        case ORC_OP_ACT4: { /* lietorch_gpu.cu:238-256 */
          se3_t g = se3_load(x + (size_t)e * N);
          double R[9], T[16], q[4];
          so3_matrix(g.r, R);
          memset(T, 0, sizeof(T));
          for (int i = 0; i < 3; i++) {
            for (int j = 0; j < 3; j++) T[i * 4 + j] = R[i * 3 + j];
            T[i * 4 + 3] = g.t[i];
          }
          T[15] = 1;
          rowvec_mat(grad + (size_t)e * 4, T, 4, 4, out1 + (size_t)e * 4);
          const double* p = y + (size_t)e * 4;
          so3_act(g.r, p, q);
          for (int i = 0; i < 3; i++) q[i] += g.t[i] * p[3];
          q[3] = p[3];
          double J[24], H[9], mq[3] = {-q[0], -q[1], -q[2]};
          memset(J, 0, sizeof(J));
          hat3(mq, H);
          for (int i = 0; i < 3; i++)
            for (int j = 0; j < 3; j++) {
              J[i * 6 + j] = (i == j) ? q[3] : 0.0;
              J[i * 6 + 3 + j] = H[i * 3 + j];
            }
          memset(out0 + (size_t)e * N, 0, sizeof(double) * N);
          rowvec_mat(grad + (size_t)e * 4, J, 4, 6, out0 + (size_t)e * N);
        } break;
        default: return -3;
      }
    } else {
      double R[9], T3[9], r3[3], J3[9];
      switch (op) {
        case ORC_OP_EXP:
          so3_left_jac(x + (size_t)e * K, J3);
          rowvec_mat(grad + (size_t)e * N, J3, 3, 3, out0 + (size_t)e * K);
          break;
        case ORC_OP_LOG:
          so3_log(so3_load(x + (size_t)e * N), r3);
          so3_left_jac_inv(r3, J3);
          memset(out0 + (size_t)e * N, 0, sizeof(double) * N);
          rowvec_mat(grad + (size_t)e * K, J3, 3, 3, out0 + (size_t)e * N);
          break;
        case ORC_OP_INV:
          so3_matrix(so3_inv(so3_load(x + (size_t)e * N)), R);
          memset(out0 + (size_t)e * N, 0, sizeof(double) * N);
          rowvec_mat(grad + (size_t)e * N, R, 3, 3, r3);
          for (int i = 0; i < 3; i++) out0[(size_t)e * N + i] = -r3[i];
          break;
        case ORC_OP_MUL:
          memset(out0 + (size_t)e * N, 0, sizeof(double) * N);
          memset(out1 + (size_t)e * N, 0, sizeof(double) * N);
          for (int i = 0; i < 3; i++) out0[(size_t)e * N + i] = grad[(size_t)e * N + i];
          so3_matrix(so3_load(x + (size_t)e * N), R);
          rowvec_mat(grad + (size_t)e * N, R, 3, 3, out1 + (size_t)e * N);
          break;
        case ORC_OP_ADJ:
          so3_matrix(so3_load(x + (size_t)e * N), R);
          mat_vec(R, y + (size_t)e * K, 3, 3, r3);
          rowvec_mat(grad + (size_t)e * K, R, 3, 3, out1 + (size_t)e * K);
          hat3(r3, T3);
          memset(out0 + (size_t)e * N, 0, sizeof(double) * N);
          rowvec_mat(grad + (size_t)e * K, T3, 3, 3, tmp);
          for (int i = 0; i < 3; i++) out0[(size_t)e * N + i] = -tmp[i];
          break;
        case ORC_OP_ADJT:
          so3_matrix(so3_load(x + (size_t)e * N), R);
          mat_vec(R, grad + (size_t)e * K, 3, 3, r3);
          for (int i = 0; i < 3; i++) out1[(size_t)e * K + i] = r3[i];
          hat3(r3, T3);
          memset(out0 + (size_t)e * N, 0, sizeof(double) * N);
          rowvec_mat(y + (size_t)e * K, T3, 3, 3, tmp);
          for (int i = 0; i < 3; i++) out0[(size_t)e * N + i] = -tmp[i];
          break;
        case ORC_OP_ACT: {
          so3_t g = so3_load(x + (size_t)e * N);
          so3_matrix(g, R);
          rowvec_mat(grad + (size_t)e * 3, R, 3, 3, out1 + (size_t)e * 3);
          double q[3], mq[3];
          so3_act(g, y + (size_t)e * 3, q);
          for (int i = 0; i < 3; i++) mq[i] = -q[i];
          hat3(mq, T3);
          memset(out0 + (size_t)e * N, 0, sizeof(double) * N);
          rowvec_mat(grad + (size_t)e * 3, T3, 3, 3, out0 + (size_t)e * N);
        } break;
        case ORC_OP_ACT4: {
          so3_t g = so3_load(x + (size_t)e * N);
          so3_matrix(g, R);
          double T[16];
          memset(T, 0, sizeof(T));
          for (int i = 0; i < 3; i++)
            for (int j = 0; j < 3; j++) T[i * 4 + j] = R[i * 3 + j];
          T[15] = 1;
          rowvec_mat(grad + (size_t)e * 4, T, 4, 4, out1 + (size_t)e * 4);
          double q[3], mq[3], J[12];
          so3_act(g, y + (size_t)e * 4, q);
          for (int i = 0; i < 3; i++) mq[i] = -q[i];
          hat3(mq, T3);
          memset(J, 0, sizeof(J));
          for (int i = 0; i < 9; i++) J[i] = T3[i];
          memset(out0 + (size_t)e * N, 0, sizeof(double) * N);
          rowvec_mat(grad + (size_t)e * 4, J, 4, 3, out0 + (size_t)e * N);
        } break;
        default: return -3;
      }
    }
    (void)Jm; (void)b;
  }
  return 0;
}

/* ------------------------------------------------------------------------ */
/* F-FLOW: projective_ops.flow_mag (projective_ops.py:120-130) over          */
/* transform (:53-110) with lietorch's fp32 group ops (se3.h inv 325-327,    */
/* mul 334-336, act4; quaternion renormalised at every load, so3.h:95-97).   */
/* Op by op in fp32 (-std=c99: no contraction), as the reference's kernels.  */
/* ------------------------------------------------------------------------ */
typedef struct { float t[3], q[4]; } g7f;

static g7f g7_load(const float* d) {
  g7f g;
  float n;
  g.t[0] = d[0]; g.t[1] = d[1]; g.t[2] = d[2];
  n = sqrtf(d[3] * d[3] + d[4] * d[4] + d[5] * d[5] + d[6] * d[6]);
  g.q[0] = d[3] / n; g.q[1] = d[4] / n; g.q[2] = d[5] / n; g.q[3] = d[6] / n;
  return g;
}
static g7f g7_reload(g7f g) {
  float d[7] = {g.t[0], g.t[1], g.t[2], g.q[0], g.q[1], g.q[2], g.q[3]};
  return g7_load(d);
}
static void g7_qact(const float* q, const float* p, float* o) { /* so3.h:115-120 */
  float uv[3], c[3];
  uv[0] = q[1] * p[2] - q[2] * p[1];
  uv[1] = q[2] * p[0] - q[0] * p[2];
  uv[2] = q[0] * p[1] - q[1] * p[0];
  uv[0] += uv[0]; uv[1] += uv[1]; uv[2] += uv[2];
  c[0] = q[1] * uv[2] - q[2] * uv[1];
  c[1] = q[2] * uv[0] - q[0] * uv[2];
  c[2] = q[0] * uv[1] - q[1] * uv[0];
  for (int i = 0; i < 3; i++) o[i] = p[i] + q[3] * uv[i] + c[i];
}
static g7f g7_inv(g7f g) {
  g7f o;
  float t[3];
  const float n = sqrtf(g.q[0] * g.q[0] + g.q[1] * g.q[1] + g.q[2] * g.q[2] + g.q[3] * g.q[3]);
  o.q[0] = -g.q[0] / n; o.q[1] = -g.q[1] / n; o.q[2] = -g.q[2] / n; o.q[3] = g.q[3] / n;
  g7_qact(o.q, g.t, t);
  o.t[0] = -t[0]; o.t[1] = -t[1]; o.t[2] = -t[2];
  return o;
}
static g7f g7_mul(g7f a, g7f b) {
  g7f o;
  float t[3];
  const float x = a.q[3] * b.q[0] + a.q[0] * b.q[3] + a.q[1] * b.q[2] - a.q[2] * b.q[1];
  const float y = a.q[3] * b.q[1] + a.q[1] * b.q[3] + a.q[2] * b.q[0] - a.q[0] * b.q[2];
  const float z = a.q[3] * b.q[2] + a.q[2] * b.q[3] + a.q[0] * b.q[1] - a.q[1] * b.q[0];
  const float w = a.q[3] * b.q[3] - a.q[0] * b.q[0] - a.q[1] * b.q[1] - a.q[2] * b.q[2];
  const float n = sqrtf(x * x + y * y + z * z + w * w);
  o.q[0] = x / n; o.q[1] = y / n; o.q[2] = z / n; o.q[3] = w / n;
  g7_qact(a.q, b.t, t);
  for (int i = 0; i < 3; i++) o.t[i] = a.t[i] + t[i];
  return o;
}
/* transform of one pixel: Gij = poses[j] * poses[i].inv(), iproj, act4, proj */
static void transform_px(const float* Pi, const float* Pj, const float* Ki, const float* Kj,
                         float x, float y, float d, int tonly, float* out, float* Z) {
  g7f gij = g7_reload(g7_mul(g7_load(Pj), g7_reload(g7_inv(g7_load(Pi)))));
  float X0[4], p[3];
  if (tonly) { gij.q[0] = gij.q[1] = gij.q[2] = 0.0f; gij.q[3] = 1.0f; }
  X0[0] = (x - Ki[2]) / Ki[0];
  X0[1] = (y - Ki[3]) / Ki[1];
  X0[2] = 1.0f;
  X0[3] = d;
  g7_qact(gij.q, X0, p);
  {
    const float X = p[0] + gij.t[0] * X0[3], Y = p[1] + gij.t[1] * X0[3];
    const float Zz = p[2] + gij.t[2] * X0[3];
    const float inv = 1.0f / (Zz < 0.1f ? 0.1f : Zz);
    out[0] = Kj[0] * (inv * X) + Kj[2];
    out[1] = Kj[1] * (inv * Y) + Kj[3];
    *Z = Zz;
  }
}

/* flow[e * npx + p] = flow_mag of pixel p of patch kk[e] from frame ii[e] to
   jj[e]; valid = Z1 > 0.2.  px0 >= 0 selects one pixel (patches[..., r, c]
   with px0 = r * P + c, edges_loop), else all P*P pixels (motionmag). */
ORC_API int orc_flow_mag(const float* poses, const float* patches, const float* intr, int P,
                         const int64_t* ii, const int64_t* jj, const int64_t* kk, int E, int px0,
                         float beta, float* flow, uint8_t* valid) {
  const int PP = P * P, npx = px0 >= 0 ? 1 : PP;
  for (int e = 0; e < E; e++) {
    const int64_t a = ii[e], b = jj[e];
    const float* pk = patches + kk[e] * 3 * PP;
    for (int q = 0; q < npx; q++) {
      const int px = px0 >= 0 ? px0 : q;
      float c0[2], c1[2], c2[2], z0, z1, z2, a0, a1, b0, b1, f1, f2;
      transform_px(poses + 7 * a, poses + 7 * a, intr + 4 * a, intr + 4 * a, pk[px], pk[PP + px],
                   pk[2 * PP + px], 0, c0, &z0);
      transform_px(poses + 7 * a, poses + 7 * b, intr + 4 * a, intr + 4 * b, pk[px], pk[PP + px],
                   pk[2 * PP + px], 0, c1, &z1);
      transform_px(poses + 7 * a, poses + 7 * b, intr + 4 * a, intr + 4 * b, pk[px], pk[PP + px],
                   pk[2 * PP + px], 1, c2, &z2);
      a0 = c1[0] - c0[0]; a1 = c1[1] - c0[1];
      b0 = c2[0] - c0[0]; b1 = c2[1] - c0[1];
      f1 = sqrtf(a0 * a0 + a1 * a1);
      f2 = sqrtf(b0 * b0 + b1 * b1);
      flow[(size_t)e * npx + q] = beta * f1 + (1.0f - beta) * f2;
      valid[(size_t)e * npx + q] = z1 > 0.2f;
    }
  }
  return 0;
}

/* SE3(a) * SE3(b).inv() in fp32 (dpvo.py:630, pg.delta) */
ORC_API int orc_se3_mul_inv(const float* a, const float* b, float* out) {
  g7f g = g7_mul(g7_load(a), g7_reload(g7_inv(g7_load(b))));
  for (int i = 0; i < 3; i++) out[i] = g.t[i];
  for (int i = 0; i < 4; i++) out[3 + i] = g.q[i];
  return 0;
}
