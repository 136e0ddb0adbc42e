// EXPERIMENT (not in the product build; scripts/micro/gj_bench.hip measures it):
// measured 2.2-3.4x slower than ba_solve.hpp's blocked Cholesky at N = 10-16
// (profiles/r04_solver_gj/), so the window kernel keeps wsolve.
//
// ba_gjsolve.hpp -- dense solve of the damped pose Schur complement of a
// DPVO window, S dX = y (ba_cuda.cu:560-562: L = chol(S); dX =
// cholesky_solve(y, L)), by ONE 256-thread workgroup, as an explicit inverse.
//
// Why an inverse: the time of a window solve is its dependency chain, not its
// ~1e5 flops.  A Cholesky factor has a serial chain in the factorisation AND
// in every triangular sweep (forward + backward, again for each refinement
// step).  Block Gauss-Jordan inversion has the factorisation's chain only
// (N block steps, one workgroup barrier each); afterwards every solve is a
// matrix-vector product -- all 256 threads, one barrier.
//
//   * S^-1 in fp32, in registers: thread t owns row i = t / Q, columns
//     [seg L, seg L + L) with seg = t % Q (Q = 256 / n threads per row, L =
//     ceil(n / Q)); n = 6N <= 96.  A block step k (pivot rows / columns
//     K = [6k, 6k + 6)) publishes row block K (transposed, rb) and column
//     block K (cb) through LDS, double-buffered by step parity, so one
//     barrier per step suffices.  Every lane then inverts the 6x6 pivot
//     block P itself (Cholesky in registers; a non-positive pivot = failure)
//     and updates its entries with ONE 6-term dot each:
//        i in K:  a_ij <- (P^-1)_q . A_Kj      (j not in K),  (P^-1)_q,j-6k (j in K)
//        i not:   a_ij <- a_ij - V_i . A_Kj    (j not in K),  -V_i,j-6k    (j in K)
//     with V_i = A_iK P^-1 (six values per lane) -- the in-place block
//     Gauss-Jordan recurrence; both cases are one code path (coefficients
//     and a keep factor selected per lane).
//   * fp64 iterative refinement: x = S^-1 (float) y, then x += S^-1 (y - S x)
//     with the fp64 S (residual64, ba_solve.hpp).  Host emulation on the
//     cfg2 systems (condition ~2e5): ||x - x64|| / ||x64|| 7e-5 -> 2e-8 after
//     one refinement (the blocked Cholesky of ba_solve.hpp: 3e-8).
// No pivoting: every pivot block of an SPD matrix under Gauss-Jordan is a
// Schur complement of it, hence SPD.
#pragma once

#include "ba_solve.hpp"

namespace dpvo {
namespace bad {

struct GJSolve {
  const double* S;  // [NB][36] damped S (fp64), lower 6x6 blocks (lblk), row-major blocks
  const double* y;  // [n]
  double* x;        // [n] solution (fp64)
  float* rhs;       // [n] fp32 right-hand side of the current solve
  float* red;       // [n][4] partial row dots
  float* cb;        // [2][n][8] column block K of every row, by step parity
  float* rb;        // [2][n][8] row block K, transposed (rb[j][q] = A[6k + q][j])
};

// fp32 work buffers for N free poses (S, y, x are the caller's): rhs [n4],
// red [4 n4], cb [16 n4], rb [16 n4] with n4 = 6N rounded up to 4 (16-B
// aligned sub-buffers when the base is)
__host__ __device__ constexpr size_t gj_n4(int N) { return ((size_t)6 * N + 3) & ~(size_t)3; }
__host__ __device__ constexpr size_t gjsolve_floats(int N) { return 37 * gj_n4(N); }
// carve the buffers out of `f` (16-B aligned, gjsolve_floats(N) floats)
__device__ __forceinline__ void gj_carve(GJSolve& s, float* f, int N) {
  const size_t n4 = gj_n4(N);
  s.rhs = f;
  s.red = f + n4;
  s.cb = f + 5 * n4;
  s.rb = f + 21 * n4;
}

// threads per row and columns per thread for n = 6N
__host__ __device__ constexpr int gj_q(int n) { return n >= 256 ? 1 : (256 / n > 4 ? 4 : 256 / n); }
__host__ __device__ constexpr int gj_l(int n) { return (n + gj_q(n) - 1) / gj_q(n); }

// P^-1 of a 6x6 SPD block (lower entries of P used) in registers.  False if
// a Cholesky pivot is not positive (NaN included).
__device__ __forceinline__ bool inv6_spd(const float P[6][6], float Pi[6][6]) {
  float m[6][6], L[6][6], ri[6];
#pragma unroll
  for (int r = 0; r < 6; r++)
#pragma unroll
    for (int c = 0; c <= r; c++) m[r][c] = P[r][c];
  const bool ok = chol6_m(m, L, ri);  // L strictly lower, ri = 1 / L_qq
  // Linv (lower): Linv_ii = ri_i; Linv_ij = -ri_i sum_{j<=k<i} L_ik Linv_kj
  float Li[6][6];
#pragma unroll
  for (int j = 0; j < 6; j++) {
    Li[j][j] = ri[j];
#pragma unroll
    for (int i = j + 1; i < 6; i++) {
      float s = 0.0f;
#pragma unroll
      for (int k = j; k < i; k++) s += L[i][k] * Li[k][j];
      Li[i][j] = -ri[i] * s;
    }
  }
  // P^-1 = Linv^T Linv: (i, j) = sum_{k >= max(i, j)} Linv_ki Linv_kj
#pragma unroll
  for (int i = 0; i < 6; i++)
#pragma unroll
    for (int j = 0; j <= i; j++) {
      float s = 0.0f;
#pragma unroll
      for (int k = i; k < 6; k++) s += Li[k][i] * Li[k][j];
      Pi[i][j] = s;
      Pi[j][i] = s;
    }
  return ok;
}

template <int NN>
// not inlined: sixteen inlined instances push the window kernel past 256 VGPRs
// (spills); as calls each instance allocates its own registers
__device__ __noinline__ bool gjsolve_n(const GJSolve& s, int refine, int* fail) {
  constexpr int n = 6 * NN, Q = gj_q(n), L = gj_l(n);
  const int tid = threadIdx.x;
  const int i = tid / Q, seg = tid % Q, j0 = seg * L;
  const bool act = i < n;
  const int ic = act ? i : n - 1;  // clamped row (inactive lanes compute on a copy)
  const int I = ic / 6, xi = ic % 6;
  // row segment of S in fp32 registers (symmetric: upper blocks from the lower ones)
  float a[L];
#pragma unroll
  for (int c = 0; c < L; c++) {
    const int j = min(j0 + c, n - 1), J = j / 6, xj = j % 6;
    const double v = (I >= J) ? s.S[36 * lblk(I, J) + 6 * xi + xj] : s.S[36 * lblk(J, I) + 6 * xj + xi];
    a[c] = (float)v;
  }
  if (tid == 0) *fail = 0;
  bool ok = true;
  for (int k = 0; k < NN; k++) {
    const int par = k & 1, k6 = 6 * k;
    float* cb = s.cb + par * 8 * n;
    float* rb = s.rb + par * 8 * n;
    const int q = ic - k6;
    const bool inK = act && (unsigned)q < 6u;
    // (1) publish row block K (transposed) and this row's column block K
#pragma unroll
    for (int c = 0; c < L; c++) {
      const int j = j0 + c;
      if (inK && j < n) rb[8 * j + q] = a[c];
      if (act && (unsigned)(j - k6) < 6u) cb[8 * ic + (j - k6)] = a[c];
    }
    __syncthreads();
    // (2) pivot block P = A_KK (rows of rb at columns K), its inverse in every lane
    float P[6][6], Pi[6][6];
#pragma unroll
    for (int p = 0; p < 6; p++) {
      const float4 lo = *reinterpret_cast<const float4*>(rb + 8 * (k6 + p));
      const float2 hi = *reinterpret_cast<const float2*>(rb + 8 * (k6 + p) + 4);
      P[0][p] = lo.x; P[1][p] = lo.y; P[2][p] = lo.z; P[3][p] = lo.w; P[4][p] = hi.x; P[5][p] = hi.y;
    }
    __builtin_amdgcn_sched_barrier(0);
    ok = inv6_spd(P, Pi) && ok;
    // coefficients: i in K -> row q of P^-1 (V of the unit row e_q), keep 0;
    // else -V_i = -(A_iK P^-1), keep 1
    float ci[6];
    {
      const float4 lo = *reinterpret_cast<const float4*>(cb + 8 * ic);
      const float2 hi = *reinterpret_cast<const float2*>(cb + 8 * ic + 4);
      ci[0] = lo.x; ci[1] = lo.y; ci[2] = lo.z; ci[3] = lo.w; ci[4] = hi.x; ci[5] = hi.y;
    }
    const float sg = inK ? 1.0f : -1.0f, keep = inK ? 0.0f : 1.0f;
#pragma unroll
    for (int r = 0; r < 6; r++) ci[r] = inK ? ((r == q) ? 1.0f : 0.0f) : ci[r];
    float co[6];
#pragma unroll
    for (int p = 0; p < 6; p++) {
      float v = 0.0f;
#pragma unroll
      for (int r = 0; r < 6; r++) v += ci[r] * Pi[r][p];
      co[p] = sg * v;
    }
    // (3) one 6-term dot per owned entry; the scheduler may not hoist the
    // column loads above the pivot inverse (their registers would spill)
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int c = 0; c < L; c++) {
      if (c % 4 == 0) __builtin_amdgcn_sched_barrier(0);
      const int j = min(j0 + c, n - 1);
      const float4 lo = *reinterpret_cast<const float4*>(rb + 8 * j);
      const float2 hi = *reinterpret_cast<const float2*>(rb + 8 * j + 4);
      float v = keep * a[c];
      v += co[0] * lo.x;
      v += co[1] * lo.y;
      v += co[2] * lo.z;
      v += co[3] * lo.w;
      v += co[4] * hi.x;
      v += co[5] * hi.y;
      const int jk = j - k6;
      float w = co[0];
      w = (jk == 1) ? co[1] : w;
      w = (jk == 2) ? co[2] : w;
      w = (jk == 3) ? co[3] : w;
      w = (jk == 4) ? co[4] : w;
      w = (jk == 5) ? co[5] : w;
      a[c] = ((unsigned)jk < 6u) ? w : v;
    }
  }
  if (!ok) atomicOr(fail, 1);
  // x = S^-1 y, then `refine` steps x += S^-1 (y - S x) (fp64 residual)
  for (int k = tid; k < n; k += blockDim.x) s.rhs[k] = (float)s.y[k];
  __syncthreads();
  const bool okall = *fail == 0;
  for (int it = 0; it <= refine; it++) {
    if (it > 0) {
      if (!okall) break;
      residual64(s.S, s.y, s.x, s.rhs, NN);
      __syncthreads();
    }
    float d = 0.0f;
#pragma unroll
    for (int c = 0; c < L; c++) {
      const int j = j0 + c;
      d += (j < n) ? a[c] * s.rhs[min(j, n - 1)] : 0.0f;
    }
    if (act) s.red[4 * i + seg] = d;
    __syncthreads();
    if (tid < n) {
      float t = s.red[4 * tid];
#pragma unroll
      for (int g = 1; g < Q; g++) t += s.red[4 * tid + g];
      s.x[tid] = (it ? s.x[tid] : 0.0) + (double)t;
    }
    __syncthreads();
  }
  if (!okall) {
    for (int k = tid; k < n; k += blockDim.x) s.x[k] = 0.0;
    __syncthreads();
  }
  return okall;
}

// Whole workgroup (blockDim.x == 256, 1 <= N <= 16).  Solves S x = y into s.x
// (fp64); false (x = 0) if a pivot block was not positive definite.  Every
// thread returns after a workgroup barrier.  `fail` is an LDS int.
__device__ inline bool gjsolve(const GJSolve& s, int N, int refine, int* fail) {
  switch (N) {
#define DPVO_GJ_CASE(NN) \
  case NN:               \
    return gjsolve_n<NN>(s, refine, fail);
    DPVO_GJ_CASE(1)
    DPVO_GJ_CASE(2)
    DPVO_GJ_CASE(3)
    DPVO_GJ_CASE(4)
    DPVO_GJ_CASE(5)
    DPVO_GJ_CASE(6)
    DPVO_GJ_CASE(7)
    DPVO_GJ_CASE(8)
    DPVO_GJ_CASE(9)
    DPVO_GJ_CASE(10)
    DPVO_GJ_CASE(11)
    DPVO_GJ_CASE(12)
    DPVO_GJ_CASE(13)
    DPVO_GJ_CASE(14)
    DPVO_GJ_CASE(15)
    DPVO_GJ_CASE(16)
#undef DPVO_GJ_CASE
    default:
      return false;
  }
}

}  // namespace bad
}  // namespace dpvo
