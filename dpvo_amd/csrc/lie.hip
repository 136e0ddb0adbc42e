// lie.hip -- lietorch SO3 (group 1) / SE3 (group 3) on gfx950 (L-SE3).
//
// Reference semantics: dpvo/lietorch/include/so3.h, se3.h and the kernels of
// dpvo/lietorch/src/lietorch_gpu.cu:20-294 (one thread per group element,
// Eigen math).  Restated here without Eigen: plain fixed-size register math,
// templated on float/double, quaternion (x, y, z, w) normalised on load
// (so3.h:95-97), tangent ordering (tau, phi).
#include "common.hpp"

namespace dpvo {
namespace lie {

template <typename S>
struct Q4 { S x, y, z, w; };

template <typename S>
__device__ __forceinline__ Q4<S> qnorm(S x, S y, S z, S w) {
  const S n = sqrt(x * x + y * y + z * z + w * w);
  return {x / n, y / n, z / n, w / n};
}
template <typename S>
__device__ __forceinline__ Q4<S> qmul(const Q4<S>& p, const Q4<S>& q) {  // then normalise
  return qnorm<S>(p.w * q.x + p.x * q.w + p.y * q.z - p.z * q.y,
                  p.w * q.y + p.y * q.w + p.z * q.x - p.x * q.z,
                  p.w * q.z + p.z * q.w + p.x * q.y - p.y * q.x,
                  p.w * q.w - p.x * q.x - p.y * q.y - p.z * q.z);
}
template <typename S>
__device__ __forceinline__ void cross(const S* a, const S* b, S* c) {
  c[0] = a[1] * b[2] - a[2] * b[1];
  c[1] = a[2] * b[0] - a[0] * b[2];
  c[2] = a[0] * b[1] - a[1] * b[0];
}
template <typename S>
__device__ __forceinline__ void qact(const Q4<S>& q, const S* p, S* o) {  // so3.h:115-120
  const S v[3] = {q.x, q.y, q.z};
  S uv[3], uv2[3];
  cross(v, p, uv);
  uv[0] += uv[0]; uv[1] += uv[1]; uv[2] += uv[2];
  cross(v, uv, uv2);
  for (int i = 0; i < 3; i++) o[i] = p[i] + q.w * uv[i] + uv2[i];
}
template <typename S>
__device__ __forceinline__ void qmat(const Q4<S>& q, S* R) {  // Eigen toRotationMatrix
  const S tx = 2 * q.x, ty = 2 * q.y, tz = 2 * q.z;
  const S twx = tx * q.w, twy = ty * q.w, twz = tz * q.w;
  const S txx = tx * q.x, txy = ty * q.x, txz = tz * q.x;
  const S tyy = ty * q.y, tyz = tz * q.y, tzz = tz * q.z;
  R[0] = 1 - (tyy + tzz); R[1] = txy - twz; R[2] = txz + twy;
  R[3] = txy + twz; R[4] = 1 - (txx + tzz); R[5] = tyz - twx;
  R[6] = txz - twy; R[7] = tyz + twx; R[8] = 1 - (txx + tyy);
}
template <typename S>
__device__ __forceinline__ void hat(const S* p, S* H) {  // so3.h:161-169
  H[0] = 0; H[1] = -p[2]; H[2] = p[1];
  H[3] = p[2]; H[4] = 0; H[5] = -p[0];
  H[6] = -p[1]; H[7] = p[0]; H[8] = 0;
}
template <typename S>
__device__ __forceinline__ void mm3(const S* A, const S* B, S* C) {
  for (int i = 0; i < 3; i++)
    for (int j = 0; j < 3; j++)
      C[i * 3 + j] = A[i * 3] * B[j] + A[i * 3 + 1] * B[3 + j] + A[i * 3 + 2] * B[6 + j];
}
template <typename S>
__device__ __forceinline__ S eps() { return S(1e-6); }  // common.h:7

template <typename S>
__device__ __forceinline__ void so3_log(const Q4<S>& q, S* o) {  // so3.h:175-211
  const S sq = q.x * q.x + q.y * q.y + q.z * q.z;
  const S w = q.w;
  S f;
  if (sq < eps<S>() * eps<S>()) {
    f = S(2) / w - S(2.0 / 3.0) * sq / (w * w * w);
  } else {
    const S n = sqrt(sq);
    if (fabs(w) < eps<S>())
      f = (w > S(0) ? S(3.14159265358979323846) : -S(3.14159265358979323846)) / n;
    else
      f = S(2) * atan(n / w) / n;
  }
  o[0] = f * q.x; o[1] = f * q.y; o[2] = f * q.z;
}
template <typename S>
__device__ __forceinline__ Q4<S> so3_exp(const S* phi) {  // so3.h:213-230
  const S t2 = phi[0] * phi[0] + phi[1] * phi[1] + phi[2] * phi[2];
  const S t = sqrt(t2);
  S im, re;
  if (t < eps<S>()) {
    const S t4 = t2 * t2;
    im = S(0.5) - S(1.0 / 48.0) * t2 + S(1.0 / 3840.0) * t4;
    re = S(1) - S(1.0 / 8.0) * t2 + S(1.0 / 384.0) * t4;
  } else {
    im = sin(S(0.5) * t) / t;
    re = cos(S(0.5) * t);
  }
  return qnorm<S>(im * phi[0], im * phi[1], im * phi[2], re);
}
template <typename S>
__device__ __forceinline__ void so3_jl(const S* phi, S* J) {  // so3.h:232-250
  S Ph[9], Ph2[9];
  hat(phi, Ph);
  mm3(Ph, Ph, Ph2);
  const S t2 = phi[0] * phi[0] + phi[1] * phi[1] + phi[2] * phi[2], t = sqrt(t2);
  const S c1 = (t < eps<S>()) ? S(0.5) - S(1.0 / 24.0) * t2 : (S(1) - cos(t)) / t2;
  const S c2 = (t < eps<S>()) ? S(1.0 / 6.0) - S(1.0 / 120.0) * t2 : (t - sin(t)) / (t2 * t);
  for (int i = 0; i < 9; i++) J[i] = (i % 4 == 0 ? S(1) : S(0)) + c1 * Ph[i] + c2 * Ph2[i];
}
template <typename S>
__device__ __forceinline__ void so3_jl_inv(const S* phi, S* J) {  // so3.h:252-268
  S Ph[9], Ph2[9];
  hat(phi, Ph);
  mm3(Ph, Ph, Ph2);
  const S t2 = phi[0] * phi[0] + phi[1] * phi[1] + phi[2] * phi[2], t = sqrt(t2);
  const S ht = S(0.5) * t;
  const S c2 = (t < eps<S>()) ? S(1.0 / 12.0) : (S(1) - t * cos(ht) / (S(2) * sin(ht))) / (t * t);
  for (int i = 0; i < 9; i++) J[i] = (i % 4 == 0 ? S(1) : S(0)) + S(-0.5) * Ph[i] + c2 * Ph2[i];
}
template <typename S>
__device__ __forceinline__ void se3_Q(const S* xi, S* Qm) {  // se3.h:133-162
  S Ta[9], Ph[9];
  hat(xi, Ta);
  hat(xi + 3, Ph);
  const S t = sqrt(xi[3] * xi[3] + xi[4] * xi[4] + xi[5] * xi[5]);
  const S t2 = t * t, t4 = t2 * t2;
  const S c1 = (t < eps<S>()) ? S(1.0 / 6.0) - S(1.0 / 120.0) * t2 : (t - sin(t)) / (t2 * t);
  const S c2 = (t < eps<S>()) ? S(1.0 / 24.0) - S(1.0 / 720.0) * t2
                              : (t2 + 2 * cos(t) - 2) / (2 * t4);
  const S c3 = (t < eps<S>()) ? S(1.0 / 120.0) - S(1.0 / 2520.0) * t2
                              : (2 * t - 3 * sin(t) + t * cos(t)) / (2 * t4 * t);
  S PT[9], TP[9], PTP[9], PPT[9], TPP[9], PTPP[9], PPTP[9];
  mm3(Ph, Ta, PT); mm3(Ta, Ph, TP); mm3(PT, Ph, PTP);
  mm3(Ph, PT, PPT); mm3(TP, Ph, TPP); mm3(PTP, Ph, PTPP); mm3(Ph, PTP, PPTP);
  for (int i = 0; i < 9; i++)
    Qm[i] = S(0.5) * Ta[i] + c1 * (PT[i] + TP[i] + PTP[i]) + c2 * (PPT[i] + TPP[i] - 3 * PTP[i]) +
            c3 * (PTPP[i] + PPTP[i]);
}

// 6x6 row-major helpers
template <typename S>
__device__ __forceinline__ void blocks6(const S* A, const S* B, const S* D, S* M) {
  // M = [[A, B], [0, D]]
  for (int i = 0; i < 3; i++)
    for (int j = 0; j < 3; j++) {
      M[i * 6 + j] = A[i * 3 + j];
      M[i * 6 + 3 + j] = B[i * 3 + j];
      M[(3 + i) * 6 + j] = 0;
      M[(3 + i) * 6 + 3 + j] = D[i * 3 + j];
    }
}
template <typename S>
__device__ __forceinline__ void rowvec_mat(const S* v, const S* M, int n, int m, S* o) {
  for (int j = 0; j < m; j++) {
    S s = 0;
    for (int i = 0; i < n; i++) s += v[i] * M[i * m + j];
    o[j] = s;
  }
}
template <typename S>
__device__ __forceinline__ void mat_vec(const S* M, const S* v, int n, int m, S* o) {
  for (int i = 0; i < n; i++) {
    S s = 0;
    for (int j = 0; j < m; j++) s += M[i * m + j] * v[j];
    o[i] = s;
  }
}

template <typename S>
struct SE3g {
  S t[3];
  Q4<S> q;
};
template <typename S>
__device__ __forceinline__ SE3g<S> se3_load(const S* d) {
  SE3g<S> g;
  g.t[0] = d[0]; g.t[1] = d[1]; g.t[2] = d[2];
  g.q = qnorm<S>(d[3], d[4], d[5], d[6]);
  return g;
}
template <typename S>
__device__ __forceinline__ void se3_store(const SE3g<S>& g, S* d) {
  d[0] = g.t[0]; d[1] = g.t[1]; d[2] = g.t[2];
  d[3] = g.q.x; d[4] = g.q.y; d[5] = g.q.z; d[6] = g.q.w;
}
template <typename S>
__device__ __forceinline__ SE3g<S> se3_inv(const SE3g<S>& g) {  // se3.h:325-327
  SE3g<S> o;
  o.q = qnorm<S>(-g.q.x, -g.q.y, -g.q.z, g.q.w);
  S t[3];
  qact(o.q, g.t, t);
  o.t[0] = -t[0]; o.t[1] = -t[1]; o.t[2] = -t[2];
  return o;
}
template <typename S>
__device__ __forceinline__ SE3g<S> se3_mul(const SE3g<S>& a, const SE3g<S>& b) {  // :334-336
  SE3g<S> o;
  o.q = qmul(a.q, b.q);
  S t[3];
  qact(a.q, b.t, t);
  for (int i = 0; i < 3; i++) o.t[i] = a.t[i] + t[i];
  return o;
}
template <typename S>
__device__ __forceinline__ void se3_Adj(const SE3g<S>& g, S* A) {  // se3.h:347-356
  S R[9], tx[9], tR[9];
  qmat(g.q, R);
  hat(g.t, tx);
  mm3(tx, R, tR);
  blocks6(R, tR, R, A);
}
template <typename S>
__device__ __forceinline__ void se3_adj_small(const S* xi, S* A) {  // se3.h:389-401
  S Ta[9], Ph[9];
  hat(xi, Ta);
  hat(xi + 3, Ph);
  blocks6(Ph, Ta, Ph, A);
}
template <typename S>
__device__ __forceinline__ SE3g<S> se3_exp(const S* xi) {  // se3.h:423-431
  SE3g<S> g;
  g.q = so3_exp(xi + 3);
  S J[9];
  so3_jl(xi + 3, J);
  for (int i = 0; i < 3; i++) g.t[i] = J[i * 3] * xi[0] + J[i * 3 + 1] * xi[1] + J[i * 3 + 2] * xi[2];
  return g;
}
template <typename S>
__device__ __forceinline__ void se3_log(const SE3g<S>& g, S* xi) {  // se3.h:413-421
  so3_log(g.q, xi + 3);
  S Vi[9];
  so3_jl_inv(xi + 3, Vi);
  for (int i = 0; i < 3; i++) xi[i] = Vi[i * 3] * g.t[0] + Vi[i * 3 + 1] * g.t[1] + Vi[i * 3 + 2] * g.t[2];
}
template <typename S>
__device__ __forceinline__ void se3_jl(const S* xi, S* J) {  // se3.h:464-475
  S Jr[9], Qm[9];
  so3_jl(xi + 3, Jr);
  se3_Q(xi, Qm);
  blocks6(Jr, Qm, Jr, J);
}
template <typename S>
__device__ __forceinline__ void se3_jl_inv(const S* xi, S* J) {  // se3.h:477-490
  S Ji[9], Qm[9], T1[9], T2[9];
  so3_jl_inv(xi + 3, Ji);
  se3_Q(xi, Qm);
  mm3(Ji, Qm, T1);
  mm3(T1, Ji, T2);
  for (int i = 0; i < 9; i++) T2[i] = -T2[i];
  blocks6(Ji, T2, Ji, J);
}

enum { OP_EXP = 0, OP_LOG, OP_INV, OP_MUL, OP_ADJ, OP_ADJT, OP_ACT, OP_ACT4, OP_MATRIX, OP_PROJ,
       OP_JINV };

// ---- SE3 forward, one element (lietorch_gpu.cu:20-294) ----
template <typename S>
__device__ void se3_fwd(int op, const S* X, const S* Y, S* out) {
  switch (op) {
    case OP_EXP: se3_store(se3_exp(X), out); break;
    case OP_LOG: se3_log(se3_load(X), out); break;
    case OP_INV: se3_store(se3_inv(se3_load(X)), out); break;
    case OP_MUL: se3_store(se3_mul(se3_load(X), se3_load(Y)), out); break;
    case OP_ADJ: { S A[36]; se3_Adj(se3_load(X), A); mat_vec(A, Y, 6, 6, out); } break;
    case OP_ADJT: { S A[36]; se3_Adj(se3_load(X), A); rowvec_mat(Y, A, 6, 6, out); } break;
    case OP_ACT: {
      const SE3g<S> g = se3_load(X);
      S p[3];
      qact(g.q, Y, p);
      for (int i = 0; i < 3; i++) out[i] = p[i] + g.t[i];
    } break;
    case OP_ACT4: {
      const SE3g<S> g = se3_load(X);
      S p[3];
      qact(g.q, Y, p);
      for (int i = 0; i < 3; i++) out[i] = p[i] + g.t[i] * Y[3];
      out[3] = Y[3];
    } break;
    case OP_MATRIX: {
      const SE3g<S> g = se3_load(X);
      S R[9];
      qmat(g.q, R);
      for (int i = 0; i < 3; i++) {
        for (int j = 0; j < 3; j++) out[i * 4 + j] = R[i * 3 + j];
        out[i * 4 + 3] = g.t[i];
        out[12 + i] = 0;
      }
      out[15] = 1;
    } break;
    case OP_PROJ: {  // se3.h:403-411, so3.h:141-151
      const SE3g<S> g = se3_load(X);
      for (int i = 0; i < 49; i++) out[i] = 0;
      S mt[3] = {-g.t[0], -g.t[1], -g.t[2]}, H[9];
      hat(mt, H);
      for (int i = 0; i < 3; i++) {
        out[i * 7 + i] = 1;
        for (int j = 0; j < 3; j++) out[i * 7 + 3 + j] = H[i * 3 + j];
      }
      S mv[3] = {-g.q.x, -g.q.y, -g.q.z}, Hq[9];
      hat(mv, Hq);
      for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++)
          out[(3 + i) * 7 + 3 + j] = S(0.5) * ((i == j ? g.q.w : S(0)) + Hq[i * 3 + j]);
      out[6 * 7 + 3] = S(0.5) * -g.q.x;
      out[6 * 7 + 4] = S(0.5) * -g.q.y;
      out[6 * 7 + 5] = S(0.5) * -g.q.z;
    } break;
    case OP_JINV: {
      S a[6], J[36];
      se3_log(se3_load(X), a);
      se3_jl_inv(a, J);
      mat_vec(J, Y, 6, 6, out);
    } break;
  }
}

// ---- SE3 backward, one element (lietorch_gpu.cu:32-256) ----
template <typename S>
__device__ void se3_bwd(int op, const S* g, const S* X, const S* Y, S* o0, S* o1) {
  S A[36], T[6], b[6];
  switch (op) {
    case OP_EXP: se3_jl(X, A); rowvec_mat(g, A, 6, 6, o0); break;
    case OP_LOG:
      se3_log(se3_load(X), b);
      se3_jl_inv(b, A);
      rowvec_mat(g, A, 6, 6, o0);
      o0[6] = 0;
      break;
    case OP_INV:
      se3_Adj(se3_inv(se3_load(X)), A);
      rowvec_mat(g, A, 6, 6, T);
      for (int i = 0; i < 6; i++) o0[i] = -T[i];
      o0[6] = 0;
      break;
    case OP_MUL:
      for (int i = 0; i < 6; i++) o0[i] = g[i];
      o0[6] = 0;
      se3_Adj(se3_load(X), A);
      rowvec_mat(g, A, 6, 6, o1);
      o1[6] = 0;
      break;
    case OP_ADJ:
      se3_Adj(se3_load(X), A);
      mat_vec(A, Y, 6, 6, b);
      rowvec_mat(g, A, 6, 6, o1);
      se3_adj_small(b, A);
      rowvec_mat(g, A, 6, 6, T);
      for (int i = 0; i < 6; i++) o0[i] = -T[i];
      o0[6] = 0;
      break;
    case OP_ADJT:
      se3_Adj(se3_load(X), A);
      mat_vec(A, g, 6, 6, b);
      for (int i = 0; i < 6; i++) o1[i] = b[i];
      se3_adj_small(b, A);
      rowvec_mat(Y, A, 6, 6, T);
      for (int i = 0; i < 6; i++) o0[i] = -T[i];
      o0[6] = 0;
      break;
    case OP_ACT: {
      const SE3g<S> G = se3_load(X);
      S R[9], q[3];
      qmat(G.q, R);
      rowvec_mat(g, R, 3, 3, o1);
      qact(G.q, Y, q);
      for (int i = 0; i < 3; i++) q[i] = -(q[i] + G.t[i]);
      S H[9], J[18];
      hat(q, H);
      for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) {
          J[i * 6 + j] = (i == j) ? S(1) : S(0);
          J[i * 6 + 3 + j] = H[i * 3 + j];
        }
      rowvec_mat(g, J, 3, 6, o0);
      o0[6] = 0;
    } break;
    case OP_ACT4: {
      const SE3g<S> G = se3_load(X);
      S R[9], M4[16], q[3];
      qmat(G.q, R);
      for (int i = 0; i < 3; i++) {
        for (int j = 0; j < 3; j++) M4[i * 4 + j] = R[i * 3 + j];
        M4[i * 4 + 3] = G.t[i];
        M4[12 + i] = 0;
      }
      M4[15] = 1;
      rowvec_mat(g, M4, 4, 4, o1);
      qact(G.q, Y, q);
      for (int i = 0; i < 3; i++) q[i] = -(q[i] + G.t[i] * Y[3]);
      S H[9], J[24];
      hat(q, H);
      for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) {
          J[i * 6 + j] = (i == j) ? Y[3] : S(0);
          J[i * 6 + 3 + j] = H[i * 3 + j];
        }
      for (int j = 0; j < 6; j++) J[18 + j] = 0;
      rowvec_mat(g, J, 4, 6, o0);
      o0[6] = 0;
    } break;
  }
}

// ---- SO3 forward / backward, one element ----
template <typename S>
__device__ void so3_fwd(int op, const S* X, const S* Y, S* out) {
  auto ld = [](const S* d) { return qnorm<S>(d[0], d[1], d[2], d[3]); };
  auto st = [](const Q4<S>& q, S* d) { d[0] = q.x; d[1] = q.y; d[2] = q.z; d[3] = q.w; };
  S R[9];
  switch (op) {
    case OP_EXP: st(so3_exp(X), out); break;
    case OP_LOG: so3_log(ld(X), out); break;
    case OP_INV: { const Q4<S> q = ld(X); st(qnorm<S>(-q.x, -q.y, -q.z, q.w), out); } break;
    case OP_MUL: st(qmul(ld(X), ld(Y)), out); break;
    case OP_ADJ: qmat(ld(X), R); mat_vec(R, Y, 3, 3, out); break;
    case OP_ADJT: qmat(ld(X), R); rowvec_mat(Y, R, 3, 3, out); break;
    case OP_ACT: qact(ld(X), Y, out); break;
    case OP_ACT4: qact(ld(X), Y, out); out[3] = Y[3]; break;
    case OP_MATRIX:
      qmat(ld(X), R);
      for (int i = 0; i < 16; i++) out[i] = 0;
      for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) out[i * 4 + j] = R[i * 3 + j];
      out[15] = 1;
      break;
    case OP_PROJ: {
      const Q4<S> q = ld(X);
      for (int i = 0; i < 16; i++) out[i] = 0;
      S mv[3] = {-q.x, -q.y, -q.z}, H[9];
      hat(mv, H);
      for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) out[i * 4 + j] = S(0.5) * ((i == j ? q.w : S(0)) + H[i * 3 + j]);
      out[12] = S(0.5) * -q.x; out[13] = S(0.5) * -q.y; out[14] = S(0.5) * -q.z;
    } break;
    case OP_JINV: {
      S a[3], J[9];
      so3_log(ld(X), a);
      so3_jl_inv(a, J);
      mat_vec(J, Y, 3, 3, out);
    } break;
  }
}

template <typename S>
__device__ void so3_bwd(int op, const S* g, const S* X, const S* Y, S* o0, S* o1) {
  auto ld = [](const S* d) { return qnorm<S>(d[0], d[1], d[2], d[3]); };
  S R[9], J[9], a[3], T[3];
  switch (op) {
    case OP_EXP: so3_jl(X, J); rowvec_mat(g, J, 3, 3, o0); break;
    case OP_LOG: so3_log(ld(X), a); so3_jl_inv(a, J); rowvec_mat(g, J, 3, 3, o0); o0[3] = 0; break;
    case OP_INV: {
      const Q4<S> q = ld(X);
      qmat(qnorm<S>(-q.x, -q.y, -q.z, q.w), R);
      rowvec_mat(g, R, 3, 3, T);
      for (int i = 0; i < 3; i++) o0[i] = -T[i];
      o0[3] = 0;
    } break;
    case OP_MUL:
      for (int i = 0; i < 3; i++) o0[i] = g[i];
      o0[3] = 0;
      qmat(ld(X), R);
      rowvec_mat(g, R, 3, 3, o1);
      o1[3] = 0;
      break;
    case OP_ADJ:
      qmat(ld(X), R);
      mat_vec(R, Y, 3, 3, a);
      rowvec_mat(g, R, 3, 3, o1);
      hat(a, J);
      rowvec_mat(g, J, 3, 3, T);
      for (int i = 0; i < 3; i++) o0[i] = -T[i];
      o0[3] = 0;
      break;
    case OP_ADJT:
      qmat(ld(X), R);
      mat_vec(R, g, 3, 3, a);
      for (int i = 0; i < 3; i++) o1[i] = a[i];
      hat(a, J);
      rowvec_mat(Y, J, 3, 3, T);
      for (int i = 0; i < 3; i++) o0[i] = -T[i];
      o0[3] = 0;
      break;
    case OP_ACT: {
      const Q4<S> q = ld(X);
      qmat(q, R);
      rowvec_mat(g, R, 3, 3, o1);
      qact(q, Y, a);
      for (int i = 0; i < 3; i++) a[i] = -a[i];
      hat(a, J);
      rowvec_mat(g, J, 3, 3, o0);
      o0[3] = 0;
    } break;
    case OP_ACT4: {
      const Q4<S> q = ld(X);
      qmat(q, R);
      S M4[16];
      for (int i = 0; i < 16; i++) M4[i] = 0;
      for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) M4[i * 4 + j] = R[i * 3 + j];
      M4[15] = 1;
      rowvec_mat(g, M4, 4, 4, o1);
      qact(q, Y, a);
      for (int i = 0; i < 3; i++) a[i] = -a[i];
      S J4[12];
      hat(a, J);
      for (int i = 0; i < 9; i++) J4[i] = J[i];
      J4[9] = J4[10] = J4[11] = 0;
      rowvec_mat(g, J4, 4, 3, o0);
      o0[3] = 0;
    } break;
  }
}

struct Dims {
  int xin, yin, out, gin, o0, o1;
};

__host__ __device__ constexpr Dims fwd_dims(int group, int op) {
  const int K = group == 1 ? 3 : 6, N = group == 1 ? 4 : 7;
  return op == OP_EXP    ? Dims{K, 0, N, 0, 0, 0}
         : op == OP_LOG  ? Dims{N, 0, K, 0, 0, 0}
         : op == OP_INV  ? Dims{N, 0, N, 0, 0, 0}
         : op == OP_MUL  ? Dims{N, N, N, 0, 0, 0}
         : op == OP_ACT  ? Dims{N, 3, 3, 0, 0, 0}
         : op == OP_ACT4 ? Dims{N, 4, 4, 0, 0, 0}
         : op == OP_MATRIX ? Dims{N, 0, 16, 0, 0, 0}
         : op == OP_PROJ ? Dims{N, 0, N * N, 0, 0, 0}
                         : Dims{N, K, K, 0, 0, 0};  // ADJ, ADJT, JINV
}
__host__ __device__ constexpr Dims bwd_dims(int group, int op) {
  const int K = group == 1 ? 3 : 6, N = group == 1 ? 4 : 7;
  return op == OP_EXP    ? Dims{K, 0, 0, N, K, 0}
         : op == OP_LOG  ? Dims{N, 0, 0, K, N, 0}
         : op == OP_INV  ? Dims{N, 0, 0, N, N, 0}
         : op == OP_MUL  ? Dims{N, N, 0, N, N, N}
         : op == OP_ACT  ? Dims{N, 3, 0, 3, N, 3}
         : op == OP_ACT4 ? Dims{N, 4, 0, 4, N, 4}
                         : Dims{N, K, 0, K, N, K};  // ADJ, ADJT
}

// One thread per group element; (group, op) are template parameters so every
// loop bound is a compile-time constant and the operands stay in registers.
template <typename S, int G, int OP>
__global__ void __launch_bounds__(256)
    lie_fwd_kernel(int n, const S* __restrict__ X, const S* __restrict__ Y, S* __restrict__ out) {
  constexpr Dims d = fwd_dims(G, OP);
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    S x[7], y[7], o[49];
#pragma unroll
    for (int k = 0; k < d.xin; k++) x[k] = X[(size_t)i * d.xin + k];
#pragma unroll
    for (int k = 0; k < d.yin; k++) y[k] = Y[(size_t)i * d.yin + k];
    if constexpr (G == 3)
      se3_fwd<S>(OP, x, y, o);
    else
      so3_fwd<S>(OP, x, y, o);
#pragma unroll
    for (int k = 0; k < d.out; k++) out[(size_t)i * d.out + k] = o[k];
  }
}

template <typename S, int G, int OP>
__global__ void __launch_bounds__(256)
    lie_bwd_kernel(int n, const S* __restrict__ Gr, const S* __restrict__ X,
                   const S* __restrict__ Y, S* __restrict__ o0, S* __restrict__ o1) {
  constexpr Dims d = bwd_dims(G, OP);
  constexpr int K = G == 1 ? 3 : 6;
  // gradient rows of group elements are N-strided, their first K entries used
  constexpr int gread = (OP == OP_EXP || OP == OP_INV || OP == OP_MUL) ? K : d.gin;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    S x[7], y[7], g[7], a[7], b[7];
#pragma unroll
    for (int k = 0; k < d.xin; k++) x[k] = X[(size_t)i * d.xin + k];
#pragma unroll
    for (int k = 0; k < d.yin; k++) y[k] = Y[(size_t)i * d.yin + k];
#pragma unroll
    for (int k = 0; k < gread; k++) g[k] = Gr[(size_t)i * d.gin + k];
#pragma unroll
    for (int k = 0; k < 7; k++) a[k] = b[k] = 0;
    if constexpr (G == 3)
      se3_bwd<S>(OP, g, x, y, a, b);
    else
      so3_bwd<S>(OP, g, x, y, a, b);
#pragma unroll
    for (int k = 0; k < d.o0; k++) o0[(size_t)i * d.o0 + k] = a[k];
#pragma unroll
    for (int k = 0; k < d.o1; k++) o1[(size_t)i * d.o1 + k] = b[k];
  }
}

template <typename S, int G>
int launch_fwd(int op, int n, const void* X, const void* Y, void* out, hipStream_t s,
               unsigned grid) {
#define DPVO_LIE_F(OPV)                                                                        \
  case OPV:                                                                                    \
    hipLaunchKernelGGL((lie_fwd_kernel<S, G, OPV>), dim3(grid), dim3(256), 0, s, n,            \
                       (const S*)X, (const S*)Y, (S*)out);                                     \
    break;
  switch (op) {
    DPVO_LIE_F(OP_EXP) DPVO_LIE_F(OP_LOG) DPVO_LIE_F(OP_INV) DPVO_LIE_F(OP_MUL)
    DPVO_LIE_F(OP_ADJ) DPVO_LIE_F(OP_ADJT) DPVO_LIE_F(OP_ACT) DPVO_LIE_F(OP_ACT4)
    DPVO_LIE_F(OP_MATRIX) DPVO_LIE_F(OP_PROJ) DPVO_LIE_F(OP_JINV)
    default: return DPVO_ERR_INVALID;
  }
#undef DPVO_LIE_F
  return launch_status();
}

template <typename S, int G>
int launch_bwd(int op, int n, const void* Gr, const void* X, const void* Y, void* o0, void* o1,
               hipStream_t s, unsigned grid) {
#define DPVO_LIE_B(OPV)                                                                        \
  case OPV:                                                                                    \
    hipLaunchKernelGGL((lie_bwd_kernel<S, G, OPV>), dim3(grid), dim3(256), 0, s, n,            \
                       (const S*)Gr, (const S*)X, (const S*)Y, (S*)o0, (S*)o1);                \
    break;
  switch (op) {
    DPVO_LIE_B(OP_EXP) DPVO_LIE_B(OP_LOG) DPVO_LIE_B(OP_INV) DPVO_LIE_B(OP_MUL)
    DPVO_LIE_B(OP_ADJ) DPVO_LIE_B(OP_ADJT) DPVO_LIE_B(OP_ACT) DPVO_LIE_B(OP_ACT4)
    default: return DPVO_ERR_INVALID;
  }
#undef DPVO_LIE_B
  return launch_status();
}

}  // namespace lie
}  // namespace dpvo

using namespace dpvo;

static unsigned lie_grid(int n) {
  int g = (n + 255) / 256;
  if (g > 65536) g = 65536;
  return g > 0 ? g : 1;
}

DPVO_EXPORT int dpvo_lie_forward(int group, int op, int dtype, int n, const void* X, const void* Y,
                                 void* out, void* stream) {
  if (group != 1 && group != 3) return DPVO_ERR_UNSUPPORTED;
  if (op < 0 || op > lie::OP_JINV || n < 0) return DPVO_ERR_INVALID;
  if (n == 0) return DPVO_OK;
  hipStream_t s = as_stream(stream);
  const unsigned g = lie_grid(n);
  if (dtype == DPVO_F32)
    return group == 3 ? lie::launch_fwd<float, 3>(op, n, X, Y, out, s, g)
                      : lie::launch_fwd<float, 1>(op, n, X, Y, out, s, g);
  if (dtype == DPVO_F64)
    return group == 3 ? lie::launch_fwd<double, 3>(op, n, X, Y, out, s, g)
                      : lie::launch_fwd<double, 1>(op, n, X, Y, out, s, g);
  return DPVO_ERR_UNSUPPORTED;
}

DPVO_EXPORT int dpvo_lie_backward(int group, int op, int dtype, int n, const void* grad,
                                  const void* X, const void* Y, void* out0, void* out1,
                                  void* stream) {
  if (group != 1 && group != 3) return DPVO_ERR_UNSUPPORTED;
  if (op < 0 || op > lie::OP_ACT4 || n < 0) return DPVO_ERR_INVALID;
  if (n == 0) return DPVO_OK;
  hipStream_t s = as_stream(stream);
  const unsigned g = lie_grid(n);
  if (dtype == DPVO_F32)
    return group == 3 ? lie::launch_bwd<float, 3>(op, n, grad, X, Y, out0, out1, s, g)
                      : lie::launch_bwd<float, 1>(op, n, grad, X, Y, out0, out1, s, g);
  if (dtype == DPVO_F64)
    return group == 3 ? lie::launch_bwd<double, 3>(op, n, grad, X, Y, out0, out1, s, g)
                      : lie::launch_bwd<double, 1>(op, n, grad, X, Y, out0, out1, s, g);
  return DPVO_ERR_UNSUPPORTED;
}

DPVO_EXPORT const char* dpvo_status_string(int status) {
  switch (status) {
    case DPVO_OK: return "ok";
    case DPVO_ERR_INVALID: return "invalid argument";
    case DPVO_ERR_LAUNCH: return "kernel launch failed";
    case DPVO_ERR_UNSUPPORTED: return "unsupported configuration";
    case DPVO_ERR_WORKSPACE: return "workspace too small";
  }
  return "unknown status";
}

#ifndef DPVO_GIT_REV
#define DPVO_GIT_REV "dev"
#endif
DPVO_EXPORT const char* dpvo_version(void) { return "dpvo_hot gfx950 " DPVO_GIT_REV; }
