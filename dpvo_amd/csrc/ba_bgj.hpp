// ba_bgj.hpp -- in-workgroup dense SPD inverse of the large-graph BA's
// superblocks (ba_large.hip, block cyclic reduction), shared with the solver
// micro-benchmark (scripts/micro/bgj_bench.hip).
#pragma once

#include "common.hpp"


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
// (A per-thread Cholesky of P instead of (2a) + (2b), one barrier less,
// measured equal: 78.0k vs 79.0k cycles at m = 72; DESIGN.md.)
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
    // wave 0 inverts P, then W and V by products
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
