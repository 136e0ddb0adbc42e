// ba_solve.hpp -- dense solve of the damped pose Schur complement of a DPVO
// window, S dX = y (ba_cuda.cu:560-562: L = chol(S); dX = cholesky_solve),
// by ONE 256-thread workgroup, latency-first.
//
// S is at most 96 x 96 (N <= 16 free poses, 6 x 6 blocks).  The work is tiny
// (~1e5 flops); the time is the dependency chain of N pivot steps.  Design
// (DESIGN.md "F-BA solve"):
//   * fp32 blocked right-looking Cholesky with look-ahead.  Wave 0 owns the
//     critical path of step k: update block column k+1 with panel k, factor
//     the 6 x 6 pivot k+1 in registers (redundantly in every lane: no
//     cross-lane traffic), and form panel column k+1 with that factor still
//     in registers.  Waves 1-3 meanwhile apply panel k to the rest of the
//     trailing matrix.  One workgroup barrier per block step.
//   * The explicit inverse factor Z = L^-1 is accumulated alongside by waves
//     1-3 (T_ij -= L_ik Z_kj, one step behind), so the triangular solves
//     after the factorisation are dense matvecs (no N-step chains).
//   * fp64 iterative refinement: r = y - S x with the fp64 S, x += Z^T Z r.
//     A dependent fp64 FMA costs ~36 cycles on gfx950 against ~8 for fp32, so
//     the chain runs in fp32 and the accuracy comes back from the
//     (parallel) fp64 residual: ||dx - dx_64|| / ||dx_64|| ~ kappa eps32^2.
// Storage (LDS, lower 6x6 blocks, block (a, b), a >= b, at lblk(a, b),
// row-major, diagonal blocks full):
//   A: fp32 copy of S -> L (diag block k: L_kk lower, 1/L_qq on its diagonal)
//   Z: fp32, T accumulators -> Z = L^-1 (block (i, j), i >= j), each block
//      stored TRANSPOSED (column c of Z_ij contiguous: the triangular solves
//      of step k produce and consume columns)
#pragma once

#include "ba_device.hpp"

namespace dpvo {
namespace bad {

struct WSolve {
  const double* S;  // [NB][36] damped S (fp64)
  const double* y;  // [n]
  float* A;         // [NB][36]
  float* Z;         // [NB][36]
  float* v0;        // [n] fp32 work vector
  float* v1;        // [n] fp32 work vector
  double* x;        // [n] solution (fp64)
  double* r;        // unused (layout compatibility)
};

__host__ __device__ constexpr size_t wsolve_bytes(int N) {
  return sizeof(float) * 2 * 36 * (size_t)(N * (N + 1) / 2) + sizeof(float) * 2 * 6 * (size_t)N +
         sizeof(double) * 2 * 6 * (size_t)N;
}

// Wide LDS accesses: a 6x6 block is 144 B (9 x 16 B) at a 16-B aligned
// base, a row 24 B (3 x 8 B).  Few, wide DS instructions keep each step
// inside the 15 outstanding LDS requests a wave may have.
__device__ __forceinline__ void ld_row(const float* p, float v[6]) {
  const float2* q = reinterpret_cast<const float2*>(p);
#pragma unroll
  for (int k = 0; k < 3; k++) {
    const float2 t = q[k];
    v[2 * k] = t.x;
    v[2 * k + 1] = t.y;
  }
}
__device__ __forceinline__ void st_row(float* p, const float v[6]) {
  float2* q = reinterpret_cast<float2*>(p);
#pragma unroll
  for (int k = 0; k < 3; k++) q[k] = make_float2(v[2 * k], v[2 * k + 1]);
}
__device__ __forceinline__ void ld_blk(const float* p, float B[36]) {
  const float4* q = reinterpret_cast<const float4*>(p);
#pragma unroll
  for (int k = 0; k < 9; k++) {
    const float4 t = q[k];
    B[4 * k] = t.x;
    B[4 * k + 1] = t.y;
    B[4 * k + 2] = t.z;
    B[4 * k + 3] = t.w;
  }
}

// Cholesky factor of the 6x6 pivot (lower entries of `a`, row-major) in
// registers of the calling lane: L strictly lower, ri[q] = 1 / L_qq.  False if
// a pivot is not positive (NaN included).
__device__ __forceinline__ bool chol6_reg(const float* a, float L[6][6], float ri[6]) {
  float m[6][6], B[36];
  ld_blk(a, B);
#pragma unroll
  for (int r = 0; r < 6; r++)
#pragma unroll
    for (int c = 0; c <= r; c++) m[r][c] = B[6 * r + c];
  bool ok = true;
#pragma unroll
  for (int c = 0; c < 6; c++) {
    const float d = m[c][c];
    ok = ok && (d > 0.0f);
    const float rs = __builtin_amdgcn_rsqf(d);
    ri[c] = rs;
#pragma unroll
    for (int i = c + 1; i < 6; i++) L[i][c] = m[i][c] * rs;
#pragma unroll
    for (int i = c + 1; i < 6; i++)
#pragma unroll
      for (int j = c + 1; j <= i; j++) m[i][j] -= L[i][c] * L[j][c];
  }
  return ok;
}

// z = L^-1 t (forward substitution), L strictly lower + ri
__device__ __forceinline__ void fwd6(const float L[6][6], const float ri[6], const float t[6],
                                     float z[6]) {
#pragma unroll
  for (int q = 0; q < 6; q++) {
    float s = t[q];
#pragma unroll
    for (int p = 0; p < q; p++) s -= L[q][p] * z[p];
    z[q] = s * ri[q];
  }
}

// load a factored pivot block (lower L, 1/L_qq on the diagonal) from LDS
__device__ __forceinline__ void load_piv(const float* b, float L[6][6], float ri[6]) {
  float B[36];
  ld_blk(b, B);
#pragma unroll
  for (int r = 0; r < 6; r++) {
#pragma unroll
    for (int c = 0; c < r; c++) L[r][c] = B[6 * r + c];
    ri[r] = B[7 * r];
  }
}

// lanes 0..20 write the 21 lower entries of a register-resident factor
// (1/L_qq on the diagonal).  Fully unrolled selects: indexing the register
// arrays with a lane-dependent index would put them in scratch memory.
__device__ __forceinline__ void store_piv(float* pv, const float L[6][6], const float ri[6],
                                          int lane) {
  float v = 0.0f;
  int off = 0;
#pragma unroll
  for (int r = 0, idx = 0; r < 6; r++)
#pragma unroll
    for (int c = 0; c <= r; c++, idx++)
      if (lane == idx) {
        v = (r == c) ? ri[r] : L[r][c];
        off = 6 * r + c;
      }
  if (lane < 21) pv[off] = v;
}

// out[x][:] -= a[x][:] . B^T   (row x of a 6x6 block times the transpose of B)
__device__ __forceinline__ void row_sub_abt(float* out, const float* arow, const float* Bp) {
  float a[6], o[6], B[36];
  ld_row(arow, a);
  ld_row(out, o);
  ld_blk(Bp, B);
#pragma unroll
  for (int z = 0; z < 6; z++) {
    float s = o[z];
#pragma unroll
    for (int q = 0; q < 6; q++) s -= a[q] * B[6 * z + q];
    o[z] = s;
  }
  st_row(out, o);
}

// rows x and x+1 of a block at once: B (36 values) loaded once for both
__device__ __forceinline__ void row2_sub_abt(float* out, const float* arow, const float* Bp) {
  float a0[6], a1[6], o0[6], o1[6], B[36];
  ld_row(arow, a0);
  ld_row(arow + 6, a1);
  ld_row(out, o0);
  ld_row(out + 6, o1);
  ld_blk(Bp, B);
#pragma unroll
  for (int z = 0; z < 6; z++) {
    float s0 = o0[z], s1 = o1[z];
#pragma unroll
    for (int q = 0; q < 6; q++) {
      s0 -= a0[q] * B[6 * z + q];
      s1 -= a1[q] * B[6 * z + q];
    }
    o0[z] = s0;
    o1[z] = s1;
  }
  st_row(out, o0);
  st_row(out + 6, o1);
}

// quad (4 adjacent lanes) sum
__device__ __forceinline__ float quad_sum(float v) {
  v += __shfl_xor(v, 1, 64);
  v += __shfl_xor(v, 2, 64);
  return v;
}
__device__ __forceinline__ double quad_sum(double v) {
  v += __shfl_xor(v, 1, 64);
  v += __shfl_xor(v, 2, 64);
  return v;
}

// Dense matvecs after the factorisation: one pass of the workgroup, LPR
// lanes per row (4 for n <= 64, else 2; adjacent lanes, reduced by xor
// shuffles), fixed summation order.
__device__ __forceinline__ int lanes_per_row(int n) { return n <= 64 ? 4 : 2; }

template <typename T>
__device__ __forceinline__ T row_sum(T v, int lpr) {
  v += __shfl_xor(v, 1, 64);
  if (lpr == 4) v += __shfl_xor(v, 2, 64);
  return v;
}

// out = Z in  (Z lower block triangular, blocks stored transposed)
__device__ __forceinline__ void z_mul(const float* Z, const float* in, float* out, int N) {
  const int n = 6 * N, lpr = lanes_per_row(n);
  const int t = threadIdx.x, row = t / lpr, part = t % lpr;
  float s = 0.0f;
  if (row < n) {
    const int i = row / 6, x = row % 6;
    for (int j = part; j <= i; j += lpr) {
      const float* b = Z + 36 * lblk(i, j) + x;
      float v[6];
      ld_row(in + 6 * j, v);
#pragma unroll
      for (int c = 0; c < 6; c++) s += b[6 * c] * v[c];
    }
  }
  s = row_sum(s, lpr);
  if (row < n && part == 0) out[row] = s;
}

// x (+)= Z^T in, accumulated into the fp64 x
__device__ __forceinline__ void zt_mul(const float* Z, const float* in, double* x, bool add, int N) {
  const int n = 6 * N, lpr = lanes_per_row(n);
  const int t = threadIdx.x, row = t / lpr, part = t % lpr;
  float s = 0.0f;
  if (row < n) {
    const int j = row / 6, c = row % 6;
    for (int i = j + part; i < N; i += lpr) {
      float b[6], v[6];
      ld_row(Z + 36 * lblk(i, j) + 6 * c, b);
      ld_row(in + 6 * i, v);
#pragma unroll
      for (int xx = 0; xx < 6; xx++) s += b[xx] * v[xx];
    }
  }
  s = row_sum(s, lpr);
  if (row < n && part == 0) x[row] = (add ? x[row] : 0.0) + (double)s;
}

// v = (float) (y - S x) in fp64 (S lower blocks, symmetric)
__device__ __forceinline__ void residual64(const double* S, const double* y, const double* x,
                                           float* v, int N) {
  const int n = 6 * N, lpr = lanes_per_row(n);
  const int t = threadIdx.x, row = t / lpr, part = t % lpr;
  double s0 = 0.0, s1 = 0.0;
  if (row < n) {
    const int i = row / 6, xr = row % 6;
    for (int j = part; j < N; j += lpr) {
      const double* b = (i >= j) ? S + 36 * lblk(i, j) + 6 * xr : S + 36 * lblk(j, i) + xr;
      const int st = (i >= j) ? 1 : 6;
      const double* xv = x + 6 * j;
      s0 += b[0] * xv[0] + b[st] * xv[1] + b[2 * st] * xv[2];
      s1 += b[3 * st] * xv[3] + b[4 * st] * xv[4] + b[5 * st] * xv[5];
    }
  }
  const double s = row_sum(s0 + s1, lpr);
  if (row < n && part == 0) v[row] = (float)(y[row] - s);
}

// Whole workgroup (blockDim.x == 256, 1 <= N <= 16).  Solves S x = y into s.x
// (fp64).  Returns false (x = 0) if a pivot was not positive.  Every thread
// returns after a workgroup barrier.  `fail` is an LDS int.
__device__ __forceinline__ void wstamp(long long* st, int slot) {
  if (st && threadIdx.x == 0) st[slot] = (long long)__builtin_amdgcn_s_memtime();
}

// st (instrumentation, may be null): shader-clock stamps by thread 0 --
// [0] start, [1] pivot 0, [2 + k] block step k done, [40] factored,
// [41] first solve, [42 + it] refinement step it
__device__ inline bool wsolve(const WSolve& s, int N, int refine, int* fail,
                              long long* st = nullptr) {
  const int tid = threadIdx.x, wid = tid >> 6, lane = tid & 63;
  const int NB = N * (N + 1) / 2, n = 6 * N;
  wstamp(st, 0);
  // wave 0 carries the pivot chain: let it win issue / LDS arbitration
  if (wid == 0) __builtin_amdgcn_s_setprio(3);
  for (int k = tid; k < 36 * NB; k += blockDim.x) {
    s.A[k] = (float)s.S[k];
    s.Z[k] = 0.0f;
  }
  for (int k = tid; k < n; k += blockDim.x) s.v1[k] = (float)s.y[k];
  if (tid == 0) *fail = 0;
  __syncthreads();
  if (wid == 0) {  // pivot 0 and panel column 0
    float L[6][6], ri[6];
    const bool ok = chol6_reg(s.A, L, ri);
    store_piv(s.A, L, ri, lane);
    if (!ok && lane == 0) *fail = 1;
    for (int t = lane; t < 6 * (N - 1); t += 64) {
      const int i = 1 + t / 6, x = t % 6;
      float* a = s.A + 36 * lblk(i, 0) + 6 * x;
      float av[6], lv[6];
      ld_row(a, av);
      fwd6(L, ri, av, lv);
      st_row(a, lv);
    }
  }
  __syncthreads();
  wstamp(st, 1);
  for (int k = 0; k < N; k++) {
    if (wid == 0) {
      if (k + 1 < N) {
        const int c1 = k + 1;
        // (1) block column k+1 -= L_ik L_{k+1,k}^T, i >= k+1
        const float* Lk1 = s.A + 36 * lblk(c1, k);
        for (int t = lane; t < 6 * (N - c1); t += 64) {
          const int i = c1 + t / 6, x = t % 6;
          row_sub_abt(s.A + 36 * lblk(i, c1) + 6 * x, s.A + 36 * lblk(i, k) + 6 * x, Lk1);
        }
        wave_lds_sync();
        if (st && k == 2 && lane == 0) st[50] = (long long)__builtin_amdgcn_s_memtime();
        // (3) factor pivot k+1 in registers; (4) panel column k+1 with it
        float L[6][6], ri[6];
        float* pv = s.A + 36 * lblk(c1, c1);
        const bool ok = chol6_reg(pv, L, ri);
        wave_lds_sync();
        if (st && k == 2 && lane == 0) st[51] = (long long)__builtin_amdgcn_s_memtime();
        store_piv(pv, L, ri, lane);
        if (!ok && lane == 0) *fail = 1;
        for (int t = lane; t < 6 * (N - c1 - 1); t += 64) {
          const int i = c1 + 1 + t / 6, x = t % 6;
          float* a = s.A + 36 * lblk(i, c1) + 6 * x;
          float av[6], lv[6];
          ld_row(a, av);
          fwd6(L, ri, av, lv);
          st_row(a, lv);
        }
        if (st && k == 2 && lane == 0) st[52] = (long long)__builtin_amdgcn_s_memtime();
      }
    } else {
      const int t0 = tid - 64, T3 = blockDim.x - 64;
      // (5) trailing A_ij -= L_ik L_jk^T, k+2 <= j <= i
      const int m = N - k - 2;
      const int n5 = m > 0 ? 3 * (m * (m + 1) / 2) : 0;  // row pairs
      // (6) Z_kj = L_kk^-1 (T_kj - L_{k,k-1} Z_{k-1,j}) (j < k), Z_kk = L_kk^-1: column tasks
      const int n6 = 6 * (k + 1);
      // (7) T_ij -= L_{i,k-1} Z_{k-1,j}, i >= k+1, j <= k-1
      const int n7 = (k >= 1) ? 6 * (N - k - 1) * k : 0;
      for (int t = t0; t < n5 + n6 + n7; t += T3) {
        if (t < n5) {
          const int x = 2 * (t % 3);
          int a, b;
          tri_of(t / 3, a, b);
          const int i = k + 2 + a, j = k + 2 + b;
          row2_sub_abt(s.A + 36 * lblk(i, j) + 6 * x, s.A + 36 * lblk(i, k) + 6 * x,
                       s.A + 36 * lblk(j, k));
        } else if (t < n5 + n6) {
          const int u = t - n5, j = u / 6, c = u % 6;
          float tv[6], zv[6];
          if (j == k) {
#pragma unroll
            for (int q = 0; q < 6; q++) tv[q] = (q == c) ? 1.0f : 0.0f;
          } else {
            float T[6], zc[6], Lp[36];
            ld_row(s.Z + 36 * lblk(k, j) + 6 * c, T);
            ld_row(s.Z + 36 * lblk(k - 1, j) + 6 * c, zc);
            ld_blk(s.A + 36 * lblk(k, k - 1), Lp);
#pragma unroll
            for (int x = 0; x < 6; x++) {
              float v = T[x];
#pragma unroll
              for (int q = 0; q < 6; q++) v -= Lp[6 * x + q] * zc[q];
              tv[x] = v;
            }
          }
          float L[6][6], ri[6];
          load_piv(s.A + 36 * lblk(k, k), L, ri);
          fwd6(L, ri, tv, zv);
          st_row(s.Z + 36 * lblk(k, j) + 6 * c, zv);
        } else {
          const int u = t - n5 - n6, c = u % 6, blk = u / 6;
          const int i = k + 1 + blk / k, j = blk % k;
          // (transposed storage) T_ij[x][c] -= sum_q L_{i,k-1}[x][q] Z_{k-1,j}[q][c]
          row_sub_abt(s.Z + 36 * lblk(i, j) + 6 * c, s.Z + 36 * lblk(k - 1, j) + 6 * c,
                      s.A + 36 * lblk(i, k - 1));
        }
      }
      if (st && k == 2 && tid == 64) st[53] = (long long)__builtin_amdgcn_s_memtime();
    }
    __syncthreads();
    wstamp(st, 2 + k);
  }
  wstamp(st, 40);
  if (wid == 0) __builtin_amdgcn_s_setprio(0);
  const bool ok = *fail == 0;
  // x = Z^T Z y, then refinement x += Z^T Z (y - S x); v1 = (float) y since the start
  z_mul(s.Z, s.v1, s.v0, N);
  __syncthreads();
  zt_mul(s.Z, s.v0, s.x, false, N);
  __syncthreads();
  wstamp(st, 41);
  for (int it = 0; ok && it < refine; it++) {
    residual64(s.S, s.y, s.x, s.v1, N);
    __syncthreads();
    z_mul(s.Z, s.v1, s.v0, N);
    __syncthreads();
    zt_mul(s.Z, s.v0, s.x, true, N);
    __syncthreads();
    wstamp(st, 42 + it);
  }
  if (!ok) {
    for (int k = tid; k < n; k += blockDim.x) s.x[k] = 0.0;
    __syncthreads();
  }
  return ok;
}

}  // namespace bad
}  // namespace dpvo
