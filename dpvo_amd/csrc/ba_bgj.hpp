// ba_bgj.hpp -- in-workgroup dense SPD inverse of the large-graph BA's
// superblocks (ba_large.hip, block cyclic reduction), shared with the solver
// micro-benchmark (scripts/micro/bgj_bench.hip).
#pragma once

#include "common.hpp"

// per-phase shader-clock stamps (micro-benchmark builds only)
#ifndef BGJ_STAMP
#define BGJ_STAMP(k)
#endif

namespace dpvo {
namespace gba {

constexpr int kGCap = 16;  // superblock poses (band half-width limit)
constexpr int kMaxM = 6 * kGCap;

__device__ __forceinline__ double rcp_f64(double p) {
  double r = __builtin_amdgcn_rcp(p);  // ~2^-26, then two Newton steps
  double e = fma(-p, r, 1.0);
  r = fma(r, e, r);
  e = fma(-p, r, 1.0);
  return fma(r, e, r);
}

// Block Gauss-Jordan inverse (no pivoting; SPD), 6 x 6 pivot blocks, of the
// n x n matrix src (n = 6 nb <= kMaxM, row stride lda) into dst (row stride n;
// global or LDS; may alias src: every load happens before the first barrier).
// 1024 threads; thread (ty, tx) keeps entries (ty + 32 p, tx + 32 q) in
// registers.  Three barriers per block step (a scalar Gauss-Jordan needs one
// per pivot, six per block, each on the pivot's dependency chain): (1) the
// owners publish the raw block rows Rw (6 x n) and block columns Cw (n x 6)
// (parity double-buffered); (2a) wave 0 inverts the pivot P = A[b, b] (one
// entry per lane, pivot row / column by shuffles); (2b) every thread forms one
// entry of W = P^-1 Rw and of V = Cw P^-1; (3) every entry outside the block
// gets a -= Cw_i . W_j (6 FMAs), block rows W, block columns -V, the pivot P^-1.
// BGJ_THREAD_PIVOT (experiment): (2a) + (2b) replaced by right-hand-side
// solves from a per-thread Cholesky of P, one barrier less -- measured equal
// (78.0k vs 79.0k cycles at m = 72: the per-thread fp64 sqrt / reciprocal
// chain costs what the barrier and the wave-0 chain did).
// W, V, P^-1 are single-buffered: their writers of step K + 1 have passed
// barrier (1) of K + 1, so every reader of step K is done.
// vbuf: 2 (Rw + Cw) + W + V + P^-1 = 2 * 12 kMaxM + 12 kMaxM + 36 doubles.
constexpr size_t kBgjDoubles = 36 * (size_t)kMaxM + 40;
__device__ __forceinline__ bool wg_bgj_inverse(const double* src, int n, int lda, double* dst, double* vbuf) {
  __shared__ int bad;
  const int tid = threadIdx.x, ty = tid >> 5, tx = tid & 31;
  double a[3][3];
#pragma unroll
  for (int p = 0; p < 3; p++)
#pragma unroll
    for (int q = 0; q < 3; q++) {
      const int i = ty + 32 * p, j = tx + 32 * q;
      const double v = src[(size_t)min(i, n - 1) * lda + min(j, n - 1)];  // unconditional
      a[p][q] = (i < n && j < n) ? v : 0.0;
    }
  if (tid == 0) bad = 0;
  double* W = vbuf + 24 * kMaxM;  // [6][kMaxM]
  double* V = W + 6 * kMaxM;      // [kMaxM][6]
  double* Pi = V + 6 * kMaxM;     // [36]
  const int nb = n / 6;
  BGJ_STAMP(0);
  for (int K = 0; K < nb; K++) {
    const int b0 = 6 * K;
    double* Rw = vbuf + (K & 1) * 12 * kMaxM;  // [6][kMaxM]
    double* Cw = Rw + 6 * kMaxM;                // [kMaxM][6]
    // (1) publish: a thread owns at most one row and one column of the block
    const int dr = (ty - b0) & 31, dc = (tx - b0) & 31;
    if (dr < 6) {
      const int r = b0 + dr, rp = r >> 5;
#pragma unroll
      for (int q = 0; q < 3; q++) {
        const int j = tx + 32 * q;
        const double v = rp == 0 ? a[0][q] : rp == 1 ? a[1][q] : a[2][q];
        if (j < n) Rw[dr * kMaxM + j] = v;
      }
    }
    if (dc < 6) {
      const int c = b0 + dc, cq = c >> 5;
#pragma unroll
      for (int p = 0; p < 3; p++) {
        const int i = ty + 32 * p;
        const double v = cq == 0 ? a[p][0] : cq == 1 ? a[p][1] : a[p][2];
        if (i < n) Cw[i * 6 + dc] = v;
      }
    }
    __syncthreads();
    BGJ_STAMP(1 + 4 * K);
#ifndef BGJ_THREAD_PIVOT  // wave 0 inverts P, then W and V by products
    // (2a) wave 0: P^-1
    if (tid < kWave) {
      // lane 6 r + c holds P[r][c]; pivot row / column by lane shuffles
      const int lr = min(tid, 35) / 6, lc = min(tid, 35) % 6;
      double x = Rw[lr * kMaxM + b0 + lc];
      bool ok = true;
#pragma unroll
      for (int t = 0; t < 6; t++) {
        const double piv = __shfl(x, 7 * t, 64);
        const double rowv = __shfl(x, 6 * t + lc, 64);
        const double colv = __shfl(x, 6 * lr + t, 64);
        ok = ok && piv > 0.0;
        const double ip = piv > 0.0 ? rcp_f64(piv) : 0.0;
        if (lr != t && lc != t) x = fma(-colv, rowv * ip, x);
        else if (lr == t && lc != t) x = rowv * ip;
        else if (lr != t) x = -colv * ip;
        else x = ip;
      }
      if (!ok && tid == 0) bad = 1;
      if (tid < 36) Pi[tid] = x;
    }
    __syncthreads();
    BGJ_STAMP(2 + 4 * K);
    // (2b) W = P^-1 Rw and V = Cw P^-1, one entry of each per thread
    for (int q = tid; q < 6 * n; q += blockDim.x) {
      const int d = q / n, j = q - d * n;  // W[d][j]
      const int i = q / 6, e = q - i * 6;  // V[i][e]
      double sw = 0.0, sv = 0.0;
#pragma unroll
      for (int u = 0; u < 6; u++) {
        sw = fma(Pi[d * 6 + u], Rw[u * kMaxM + j], sw);
        sv = fma(Cw[i * 6 + u], Pi[u * 6 + e], sv);
      }
      W[d * kMaxM + j] = sw;
      V[i * 6 + e] = sv;
    }
    __syncthreads();
    BGJ_STAMP(3 + 4 * K);
#else
    // (2) W = P^-1 Rw, V = Cw P^-1 (= (P^-1 Cw^T)^T, P symmetric) and P^-1 by
    // right-hand sides: n columns of Rw, n rows of Cw, 6 unit vectors, one per
    // thread, each thread factoring P = L L^T itself in registers (P is an SPD
    // Schur complement).  No wave-0 pivot chain and one barrier per block step
    // less than inverting P first (profiles/r04_cfg4_bgj_phases.txt).
    for (int q = tid; q < 2 * n + 6; q += blockDim.x) {
      double l[21];  // lower triangle, packed by rows: l[i (i + 1) / 2 + j]
#pragma unroll
      for (int i = 0; i < 6; i++)
#pragma unroll
        for (int j = 0; j <= i; j++) l[i * (i + 1) / 2 + j] = Rw[i * kMaxM + b0 + j];
      double x[6];
#pragma unroll
      for (int u = 0; u < 6; u++) {  // unconditional reads, then select
        const double r = Rw[u * kMaxM + min(q, n - 1)];
        const double c = Cw[min(max(q - n, 0), n - 1) * 6 + u];
        x[u] = q < n ? r : (q < 2 * n ? c : (u == q - 2 * n ? 1.0 : 0.0));
      }
      bool ok = true;
      double rd[6];
#pragma unroll
      for (int j = 0; j < 6; j++) {
        double d = l[j * (j + 1) / 2 + j];
#pragma unroll
        for (int k = 0; k < j; k++) d = fma(-l[j * (j + 1) / 2 + k], l[j * (j + 1) / 2 + k], d);
        ok = ok && d > 0.0;
        const double sd = sqrt(d > 0.0 ? d : 1.0);
        rd[j] = rcp_f64(sd);
#pragma unroll
        for (int i = j + 1; i < 6; i++) {
          double v = l[i * (i + 1) / 2 + j];
#pragma unroll
          for (int k = 0; k < j; k++) v = fma(-l[i * (i + 1) / 2 + k], l[j * (j + 1) / 2 + k], v);
          l[i * (i + 1) / 2 + j] = v * rd[j];
        }
      }
#pragma unroll
      for (int i = 0; i < 6; i++) {  // L z = x
        double v = x[i];
#pragma unroll
        for (int k = 0; k < i; k++) v = fma(-l[i * (i + 1) / 2 + k], x[k], v);
        x[i] = v * rd[i];
      }
#pragma unroll
      for (int i = 5; i >= 0; i--) {  // L^T w = z
        double v = x[i];
#pragma unroll
        for (int k = i + 1; k < 6; k++) v = fma(-l[k * (k + 1) / 2 + i], x[k], v);
        x[i] = v * rd[i];
      }
      if (!ok) bad = 1;
      if (q < n) {
#pragma unroll
        for (int u = 0; u < 6; u++) W[u * kMaxM + q] = x[u];
      } else if (q < 2 * n) {
#pragma unroll
        for (int u = 0; u < 6; u++) V[(q - n) * 6 + u] = x[u];
      } else {
#pragma unroll
        for (int u = 0; u < 6; u++) Pi[u * 6 + (q - 2 * n)] = x[u];
      }
    }
    __syncthreads();
    BGJ_STAMP(2 + 4 * K);
    BGJ_STAMP(3 + 4 * K);
#endif
    // (3) update, branch-free except for the few waves holding block rows
    // (padding entries i, j >= n are computed from clamped rows and never
    // published or stored)
    double wj[3][6];
#pragma unroll
    for (int q = 0; q < 3; q++) {
      const int j = min(tx + 32 * q, n - 1);
#pragma unroll
      for (int u = 0; u < 6; u++) wj[q][u] = W[u * kMaxM + j];
    }
#pragma unroll
    for (int p = 0; p < 3; p++) {
      const int i = min(ty + 32 * p, n - 1);
      double ci[6];
#pragma unroll
      for (int u = 0; u < 6; u++) ci[u] = Cw[i * 6 + u];
#pragma unroll
      for (int q = 0; q < 3; q++) {
        double v = a[p][q];
#pragma unroll
        for (int u = 0; u < 6; u++) v = fma(-ci[u], wj[q][u], v);
        a[p][q] = v;
      }
    }
    // block columns (entry (i, b0 + dc), i outside the block): -V
    const int ps = (b0 + dr) >> 5, qs = (b0 + dc) >> 5;
    {
      double vv[3];
#pragma unroll
      for (int p = 0; p < 3; p++) vv[p] = V[min(ty + 32 * p, n - 1) * 6 + min(dc, 5)];
#pragma unroll
      for (int p = 0; p < 3; p++)
#pragma unroll
        for (int q = 0; q < 3; q++)
          if (dc < 6 && q == qs && !(dr < 6 && p == ps)) a[p][q] = -vv[p];
    }
    // block rows (entry (b0 + dr, j)): W, and P^-1 inside the block
    if (dr < 6) {
      const double pv = Pi[dr * 6 + min(dc, 5)];
#pragma unroll
      for (int q = 0; q < 3; q++) {
        const double wv = W[dr * kMaxM + min(tx + 32 * q, n - 1)];
        const double v = (dc < 6 && q == qs) ? pv : wv;
#pragma unroll
        for (int p = 0; p < 3; p++)
          if (p == ps) a[p][q] = v;
      }
    }
    BGJ_STAMP(4 + 4 * K);
  }
  __syncthreads();
#pragma unroll
  for (int p = 0; p < 3; p++)
#pragma unroll
    for (int q = 0; q < 3; q++) {
      const int i = ty + 32 * p, j = tx + 32 * q;
      if (i < n && j < n) dst[(size_t)i * n + j] = a[p][q];
    }
  __syncthreads();
  return bad == 0;
}


}  // namespace gba
}  // namespace dpvo
