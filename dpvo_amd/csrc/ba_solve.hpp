// ba_solve.hpp -- dense solve of the damped pose Schur complement of a DPVO
// window, S dX = y (ba_cuda.cu:560-562: L = chol(S); dX = cholesky_solve),
// by ONE 256-thread workgroup, latency-first.
//
// S is at most 96 x 96 (N <= 16 free poses, 6 x 6 blocks).  The work is tiny
// (~1e5 flops); the time is the dependency chain of N pivot steps.  Design
// (DESIGN.md "F-BA solve"):
//   * fp32 blocked right-looking Cholesky with look-ahead.  Wave 0 owns the
//     critical path of step k: block column k+1 is updated with panel k in
//     registers (rows lane, lane + 64), the 6 x 6 pivot k+1 is broadcast by
//     v_readlane and factored redundantly in every lane, its inverse Linv
//     written by lanes 0-5, and panel column k+1 formed from the rows still
//     in registers -- one LDS round trip per step.  Waves 1-3 meanwhile apply
//     panel k to the rest of the trailing matrix.  One workgroup barrier per
//     block step.  The chain is instruction issue on one wave, so its 6-term
//     dots (column update, sweeps) are packed fp32 (v_pk_fma_f32).
//   * The factor is turned into block LDL^T form, A = Lt D Lt^T with
//     Lt_ik = L_ik Linv_kk and D_k^-1 = Linv_kk^T Linv_kk (ldl_task, by wave 3
//     while the trailing update leaves it idle), so a block step of the
//     triangular sweeps is 6 v_readlane broadcasts and ONE 6-term dot per lane
//     (wave 0 alone, right-hand side in registers, no barrier inside a sweep).
//   * fp64 iterative refinement: r = y - S x with the fp64 S, x += A^-1 r.
//     A dependent fp64 FMA costs ~36 cycles on gfx950 against ~8 for fp32, so
//     the chain runs in fp32 and the accuracy comes back from the
//     (parallel) fp64 residual: ||dx - dx_64|| / ||dx_64|| ~ kappa eps32^2.
// Storage (LDS, lower 6x6 blocks, block (a, b), a >= b, at lblk(a, b),
// row-major, diagonal blocks full):
//   A: fp32 copy of S -> L (diag block k: L_kk lower, 1/L_qq on its
//      diagonal) -> D_k^-1 on the diagonal blocks after ldl_task
//   Z: diag block k: Linv_kk (lower, zeros above); off-diagonal (i, k): Lt_ik
#pragma once

#include "ba_device.hpp"

namespace dpvo {
namespace bad {

struct WSolve {
  const double* S;  // [NB][36] damped S (fp64), 16-B aligned (read in pairs)
  const double* y;  // [n]
  float* A;         // [NB][36], 8-B aligned
  float* Z;         // [NB][36]
  float* v0;        // [n] unused (layout compatibility)
  float* v1;        // [n] fp32 work vector
  double* x;        // [n] solution (fp64)
  double* r;        // unused (layout compatibility)
};

__host__ __device__ constexpr size_t wsolve_bytes(int N) {
  return sizeof(float) * 2 * 36 * (size_t)(N * (N + 1) / 2) + sizeof(float) * 2 * 6 * (size_t)N +
         sizeof(double) * 2 * 6 * (size_t)N;
}

typedef float f32x2 __attribute__((ext_vector_type(2)));  // packed fp32 (v_pk_fma_f32)

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
__device__ __forceinline__ void ld_col(const float* c, float v[6]) {  // stride-6 column
#pragma unroll
  for (int q = 0; q < 6; q++) v[q] = c[6 * q];
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
__device__ __forceinline__ bool chol6_m(float m[6][6], float L[6][6], float ri[6]) {
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
__device__ __forceinline__ bool chol6_reg(const float* a, float L[6][6], float ri[6]) {
  float m[6][6], B[36];
  ld_blk(a, B);
#pragma unroll
  for (int r = 0; r < 6; r++)
#pragma unroll
    for (int c = 0; c <= r; c++) m[r][c] = B[6 * r + c];
  return chol6_m(m, L, ri);
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

// lanes 0-5 store column `lane` of Linv = L^-1 of a register-resident pivot
// factor into a row-major 6x6 block (zeros above the diagonal included)
__device__ __forceinline__ void store_linv(float* out, const float L[6][6], const float ri[6],
                                           int lane) {
  if (lane < 6) {
    float e[6], z[6];
#pragma unroll
    for (int q = 0; q < 6; q++) e[q] = (q == lane) ? 1.0f : 0.0f;
    fwd6(L, ri, e, z);
#pragma unroll
    for (int x = 0; x < 6; x++) out[6 * x + lane] = z[x];
  }
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
    // rows x and x + 1 as one packed pair (v_pk_fma_f32), B broadcast
    f32x2 s = f32x2{o0[z], o1[z]};
#pragma unroll
    for (int q = 0; q < 6; q++)
      s = __builtin_elementwise_fma(f32x2{-a0[q], -a1[q]}, f32x2{B[6 * z + q], B[6 * z + q]}, s);
    o0[z] = s.x;
    o1[z] = s.y;
  }
  st_row(out, o0);
  st_row(out + 6, o1);
}

// lanes per row (4 for n <= 64, else 2; adjacent lanes, reduced by xor
// shuffles), fixed summation order.
__device__ __forceinline__ int lanes_per_row(int n) { return n <= 64 ? 4 : 2; }

template <typename T>
__device__ __forceinline__ T row_sum(T v, int lpr) {
  v += __shfl_xor(v, 1, 64);
  if (lpr == 4) v += __shfl_xor(v, 2, 64);
  return v;
}

// v = (float) (y - S x) in fp64 (S lower blocks, symmetric)
__device__ __forceinline__ void residual64(const double* S, const double* y, const double* x,
                                           float* v, int N) {
  const int n = 6 * N, lpr = lanes_per_row(n);
  int t = threadIdx.x;
  asm volatile("" : "+v"(t));  // not loop-invariant for the caller (see wsolve)
  const int row = t / lpr, part = t % lpr;
  double s0 = 0.0, s1 = 0.0;
  if (row < n) {
    const int i = row / 6, xr = row % 6;
    // unrolled: the loads of later blocks issue before the fp64 FMA chains of
    // the first (one LDS wait for several blocks instead of one per block)
#pragma unroll 4
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

__device__ __forceinline__ void wstamp(long long* st, int slot) {
  if (st && threadIdx.x == 0) st[slot] = (long long)__builtin_amdgcn_s_memtime();
}

// broadcast rows 6k .. 6k+5 of the lane-distributed vector (b0: rows 0..63,
// b1: rows 64..) to every lane
__device__ __forceinline__ void bcast6(float b0, float b1, int k, float out[6]) {
  if (6 * k + 5 < 64) {  // wave-uniform branches (resolved at compile time for constant k)
#pragma unroll
    for (int q = 0; q < 6; q++)
      out[q] = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(b0), 6 * k + q));
  } else if (6 * k >= 64) {
#pragma unroll
    for (int q = 0; q < 6; q++)
      out[q] = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(b1), 6 * k + q - 64));
  } else {
#pragma unroll
    for (int q = 0; q < 6; q++) {
      const int r = 6 * k + q;
      const float lo = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(b0), min(r, 63)));
      const float hi = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(b1), max(r - 64, 0)));
      out[q] = (r < 64) ? lo : hi;
    }
  }
}

// Block LDL^T form of the factor, A = Lt D Lt^T with Lt_ik = L_ik Linv_kk
// (unit diagonal blocks) and D_k^-1 = Linv_kk^T Linv_kk: a block step of a
// sweep is then 6 v_readlane broadcasts, ONE 6-term dot per lane and a select
// (no per-step 6x6 triangular solve on the chain).  Storage after the
// factorisation (ldl_task):
// Z off-diagonal block (i, k) = Lt_ik (row-major), A diagonal block k = D_k^-1.
// task u of block column kc (u < 6 (N - kc)): u < 6 row u of D_kc^-1, else
// row u % 6 of Lt_{kc + u / 6, kc}.  Needs panel column kc and Linv_kc final.
__device__ __forceinline__ void ldl_task(const WSolve& s, int kc, int u) {
  const int i = kc + u / 6, x = u % 6;
  const float* Lip = s.Z + 36 * lblk(kc, kc);
  float Li[36], o[6];
  ld_blk(Lip, Li);
  if (i > kc) {  // Lt_ik[x][q] = sum_{p >= q} L_ik[x][p] Linv_kk[p][q]
    float l[6];
    ld_row(s.A + 36 * lblk(i, kc) + 6 * x, l);
#pragma unroll
    for (int q = 0; q < 6; q++) {
      float v = 0.0f;
#pragma unroll
      for (int p = q; p < 6; p++) v += l[p] * Li[6 * p + q];
      o[q] = v;
    }
  } else {  // D^-1[x][q] = sum_p Linv[p][x] Linv[p][q] (Linv stored with its zeros)
    float lx[6];
    ld_col(Lip + x, lx);
#pragma unroll
    for (int q = 0; q < 6; q++) {
      float v = 0.0f;
#pragma unroll
      for (int p = q; p < 6; p++) v += lx[p] * Li[6 * p + q];
      o[q] = v;
    }
  }
  st_row((i > kc ? s.Z + 36 * lblk(i, kc) : s.A + 36 * lblk(kc, kc)) + 6 * x, o);
}

// b := A^-1 b = Lt^-T D^-1 Lt^-1 b by wave 0 (rows lane and lane + 64 of b in
// b0 / b1).  Compile-time N (one instance per N <= 11, DPVO's windows): both
// sweeps fully unrolled, the loads (which do not depend on b) for step k+1
// issued before step k's readlane chain, no register copies between steps.
__device__ __forceinline__ const float* fwd_row(const float* A, const float* Z, int i, int x, int k,
                                                int N) {
  return (i > k && i < N) ? Z + 36 * lblk(i, k) + 6 * x : A + 36 * lblk(k, k) + 6 * x;
}
__device__ __forceinline__ const float* bwd_col(const float* Z, int i, int x, int k) {
  return Z + 36 * lblk(k, (i < k) ? i : 0) + x;
}
// packed fp32 (v_pk_fma_f32: two products per instruction): (even, odd)
// partial sums, then one add
__device__ __forceinline__ float dot6(const float l[6], const float v[6]) {
  f32x2 s = f32x2{l[0], l[1]} * f32x2{v[0], v[1]};
  s = __builtin_elementwise_fma(f32x2{l[2], l[3]}, f32x2{v[2], v[3]}, s);
  s = __builtin_elementwise_fma(f32x2{l[4], l[5]}, f32x2{v[4], v[5]}, s);
  return s.x + s.y;
}

template <int NN>
__device__ __forceinline__ void ldl_sweeps(const float* A, const float* Z, int lane, float& b0,
                                           float& b1) {
  constexpr int N = NN, n = 6 * N;
  constexpr bool two = n > 64;
  const int r0 = lane, r1 = lane + 64;
  const int i0 = r0 / 6, x0 = r0 % 6, i1 = r1 / 6, x1 = r1 % 6;
  // forward: y_k = b_k (final at step k), b_i -= Lt_ik y_k (i > k); block k
  // lanes turn y_k into w_k = D_k^-1 y_k with the same dot
  float l0[N][6], l1[N][6];
  ld_row(fwd_row(A, Z, i0, x0, 0, N), l0[0]);
  if (two) ld_row(fwd_row(A, Z, i1, x1, 0, N), l1[0]);
#pragma unroll
  for (int k = 0; k < N; k++) {
    float bk[6];
    if (k + 1 < N) {
      ld_row(fwd_row(A, Z, i0, x0, k + 1, N), l0[k + 1]);
      if (two) ld_row(fwd_row(A, Z, i1, x1, k + 1, N), l1[k + 1]);
    }
    bcast6(b0, b1, k, bk);
    {
      const float d = dot6(l0[k], bk);
      b0 = (i0 == k) ? d : (i0 > k && r0 < n) ? b0 - d : b0;
    }
    if (two) {
      const float d = dot6(l1[k], bk);
      b1 = (i1 == k) ? d : (i1 > k && r1 < n) ? b1 - d : b1;
    }
  }
  // backward: x_k (final at step k), b_j -= Lt_kj^T x_k (j < k)
  if (N > 1) {
    ld_col(bwd_col(Z, i0, x0, N - 1), l0[N - 1]);
    if (two) ld_col(bwd_col(Z, i1, x1, N - 1), l1[N - 1]);
  }
#pragma unroll
  for (int k = N - 1; k > 0; k--) {
    float xk[6];
    if (k > 1) {
      ld_col(bwd_col(Z, i0, x0, k - 1), l0[k - 1]);
      if (two) ld_col(bwd_col(Z, i1, x1, k - 1), l1[k - 1]);
    }
    bcast6(b0, b1, k, xk);
    {
      const float d = dot6(l0[k], xk);
      b0 = (i0 < k) ? b0 - d : b0;
    }
    if (two) {
      const float d = dot6(l1[k], xk);
      b1 = (i1 < k) ? b1 - d : b1;
    }
  }
}

// the same for a run-time N (every N but 10 and 11)
__device__ __forceinline__ void ldl_sweeps_rt(const float* A, const float* Z, int N, int lane,
                                           float& b0, float& b1) {
  const int n = 6 * N;
  const int r0 = lane, r1 = lane + 64;
  const int i0 = r0 / 6, x0 = r0 % 6, i1 = r1 / 6, x1 = r1 % 6;
  for (int k = 0; k < N; k++) {
    float l0[6], l1[6], bk[6];
    ld_row(fwd_row(A, Z, i0, x0, k, N), l0);
    ld_row(fwd_row(A, Z, i1, x1, k, N), l1);
    bcast6(b0, b1, k, bk);
    const float d0 = dot6(l0, bk), d1 = dot6(l1, bk);
    b0 = (i0 == k) ? d0 : (i0 > k && r0 < n) ? b0 - d0 : b0;
    b1 = (i1 == k) ? d1 : (i1 > k && r1 < n) ? b1 - d1 : b1;
  }
  for (int k = N - 1; k > 0; k--) {
    float l0[6], l1[6], xk[6];
    ld_col(bwd_col(Z, i0, x0, k), l0);
    ld_col(bwd_col(Z, i1, x1, k), l1);
    bcast6(b0, b1, k, xk);
    const float d0 = dot6(l0, xk), d1 = dot6(l1, xk);
    b0 = (i0 < k) ? b0 - d0 : b0;
    b1 = (i1 < k) ? b1 - d1 : b1;
  }
}

__device__ __forceinline__ void sweeps(const float* A, const float* Z, int N, int lane, float& b0,
                                       float& b1) {
  // Unrolled for DPVO's window sizes only (N = 10: the fork's window of free
  // poses, N = 11: cfg2).  Inside the window kernel's BA iteration loop the
  // compiler hoists the per-lane row addresses and selects of every unrolled
  // case before the loop (they are loop-invariant) and keeps them live in
  // spilled registers: with all of N = 1..11 unrolled that was ~2000
  // instructions (2.5 us) at the loop entry.  Other N take the loop form.
  switch (N) {
    case 10:
      ldl_sweeps<10>(A, Z, lane, b0, b1);
      break;
    case 11:
      ldl_sweeps<11>(A, Z, lane, b0, b1);
      break;
    default:
      ldl_sweeps_rt(A, Z, N, lane, b0, b1);
  }
}

// block column k-1's LDL^T tasks go to wave 3 during factor step k when the
// step's trailing update (n5 row pairs) leaves it idle
__device__ __forceinline__ bool ldl_early(int N, int k) {
  const int m = N - k - 2, n5 = m > 0 ? 3 * (m * (m + 1) / 2) : 0;
  return k >= 1 && n5 <= 128;
}

// Whole workgroup (blockDim.x == 256, 1 <= N <= 16).  Solves S x = y into s.x
// (fp64).  Returns false (x = 0) if a pivot was not positive.  Every thread
// returns after a workgroup barrier.  `fail` is an LDS int.
// st (instrumentation, may be null): shader-clock stamps by thread 0 --
// [0] start, [1] pivot 0, [2 + k] block step k done, [40] factored,
// [41] first solve, [42 + it] refinement step it; step 2: [50] wave 0 done,
// [51 + w] wave w's trailing update done, [55] wave 3's ldl_task done
__device__ inline bool wsolve(const WSolve& s, int N, int refine, int* fail,
                              long long* st = nullptr) {
  const int tid = threadIdx.x, wid = tid >> 6, lane = tid & 63;
  const int NB = N * (N + 1) / 2, n = 6 * N;
  wstamp(st, 0);
  if (wid == 0) __builtin_amdgcn_s_setprio(3);
  // pairs: one 16-B read and one 8-B write per two entries (S 16-B, A 8-B aligned)
  for (int k = tid; k < 18 * NB; k += blockDim.x) {
    const double2 v = reinterpret_cast<const double2*>(s.S)[k];
    reinterpret_cast<float2*>(s.A)[k] = make_float2((float)v.x, (float)v.y);
  }
  for (int k = tid; k < n; k += blockDim.x) s.v1[k] = (float)s.y[k];
  if (tid == 0) *fail = 0;
  __syncthreads();
  if (wid == 0) {  // pivot 0 and panel column 0
    float L[6][6], ri[6];
    const bool ok = chol6_reg(s.A, L, ri);
    store_linv(s.Z, L, ri, lane);
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
        // block column k+1 in registers (row t = lane, lane + 64 of it:
        // block c1 + t / 6, row t % 6): update with panel k, broadcast the
        // pivot rows (lanes 0-5) by v_readlane, factor the pivot in every lane,
        // and form the panel rows -- one LDS round trip per step
        const int c1 = k + 1, nr = 6 * (N - c1);
        float B[36], v0[6], v1[6];
        ld_blk(s.A + 36 * lblk(c1, k), B);
        const int ta = min(lane, nr - 1), tb = min(lane + 64, nr - 1);
        const int ia = c1 + ta / 6, xa = ta % 6, ib = c1 + tb / 6, xb = tb % 6;
        {
          float a[6];
          ld_row(s.A + 36 * lblk(ia, k) + 6 * xa, a);
          ld_row(s.A + 36 * lblk(ia, c1) + 6 * xa, v0);
#pragma unroll
          for (int z = 0; z < 6; z++) v0[z] -= dot6(a, B + 6 * z);
        }
        if (nr > 64) {
          float a[6];
          ld_row(s.A + 36 * lblk(ib, k) + 6 * xb, a);
          ld_row(s.A + 36 * lblk(ib, c1) + 6 * xb, v1);
#pragma unroll
          for (int z = 0; z < 6; z++) v1[z] -= dot6(a, B + 6 * z);
        }
        float m[6][6], L[6][6], ri[6];
        // the 21 lower pivot entries (row r = lane r's v0) to every lane by
        // v_readlane: 33.1k vs 34.9k cycles per N = 11 solve against a store
        // of the rows to LDS, a wave LDS fence and a 144-B block load (nothing
        // else reads the updated pivot rows: only Linv is kept of the block)
#pragma unroll
        for (int r = 0; r < 6; r++)
#pragma unroll
          for (int c = 0; c <= r; c++)
            m[r][c] = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v0[c]), r));
        const bool ok = chol6_m(m, L, ri);
        if (!ok && lane == 0) *fail = 1;
        {
          // ONE forward substitution per lane: lanes 0-5 solve for unit vectors
          // (column `lane` of Linv = L^-1, stored with its zeros into Z), the
          // other lanes for their panel row (L^-1 v0, stored into A); two
          // back-to-back substitutions (store_linv, then the panel) were two
          // dependent 21-FMA chains on the critical path of every block step
          float rhs[6], z[6];
#pragma unroll
          for (int q = 0; q < 6; q++) rhs[q] = (lane < 6) ? ((q == lane) ? 1.0f : 0.0f) : v0[q];
          fwd6(L, ri, rhs, z);
          if (lane < 6) {
            float* out = s.Z + 36 * lblk(c1, c1);
#pragma unroll
            for (int x = 0; x < 6; x++) out[6 * x + lane] = z[x];
          } else if (lane < nr) {
            st_row(s.A + 36 * lblk(ia, c1) + 6 * xa, z);
          }
        }
        if (lane + 64 < nr) {
          float lv[6];
          fwd6(L, ri, v1, lv);
          st_row(s.A + 36 * lblk(ib, c1) + 6 * xb, lv);
        }
        if (st && k == 2 && lane == 0) st[50] = (long long)__builtin_amdgcn_s_memtime();
      }
    } else {
      const int t0 = tid - 64, T3 = blockDim.x - 64;
      // trailing A_ij -= L_ik L_jk^T, k+2 <= j <= i
      const int m = N - k - 2;
      const int n5 = m > 0 ? 3 * (m * (m + 1) / 2) : 0;  // row pairs
      for (int t = t0; t < n5; t += T3) {
        const int x = 2 * (t % 3);
        int a, b;
        tri_of(t / 3, a, b);
        const int i = k + 2 + a, j = k + 2 + b;
        row2_sub_abt(s.A + 36 * lblk(i, j) + 6 * x, s.A + 36 * lblk(i, k) + 6 * x,
                     s.A + 36 * lblk(j, k));
      }
      if (k == N - 1 && t0 < 6) ldl_task(s, k, t0);  // D_{N-1}^-1 (no Lt below it)
      // LDL^T form of block column k-1 (ldl_task) by wave 3 when the tasks
      // above leave it idle; the remaining columns after the factorisation
      if (st && k == 2 && (tid & 63) == 0) st[51 + wid] = (long long)__builtin_amdgcn_s_memtime();
      if (wid == 3 && ldl_early(N, k))
        for (int u = lane; u < 6 * (N - k + 1); u += 64) ldl_task(s, k - 1, u);
      if (st && k == 2 && tid == 192) st[55] = (long long)__builtin_amdgcn_s_memtime();
    }
    __syncthreads();
    wstamp(st, 2 + k);
  }
  {  // the block columns ldl_early left over (D_{N-1}^-1 is done in step N-1)
    int tot = 0;
    for (int kc = 0; kc + 1 < N; kc++)
      if (!ldl_early(N, kc + 1)) tot += 6 * (N - kc);
    for (int t = tid; t < tot; t += blockDim.x) {
      int r = t, kc = 0;
      for (; kc + 1 < N; kc++) {
        if (ldl_early(N, kc + 1)) continue;
        if (r < 6 * (N - kc)) break;
        r -= 6 * (N - kc);
      }
      ldl_task(s, kc, r);
    }
    if (tot) __syncthreads();
  }
  wstamp(st, 40);
  const bool ok = *fail == 0;
  // x = A^-1 y by wave 0, then refinement x += A^-1 (y - S x); one call site
  // of the sweeps (their code is large)
  for (int it = 0; it <= refine; it++) {
    if (it > 0) {
      if (!ok) break;
      residual64(s.S, s.y, s.x, s.v1, N);
      __syncthreads();
    }
    if (wid == 0) {
      float b0 = (lane < n) ? s.v1[lane] : 0.0f, b1 = (lane + 64 < n) ? s.v1[lane + 64] : 0.0f;
      sweeps(s.A, s.Z, N, lane, b0, b1);
      if (lane < n) s.x[lane] = (it ? s.x[lane] : 0.0) + (double)b0;
      if (lane + 64 < n) s.x[lane + 64] = (it ? s.x[lane + 64] : 0.0) + (double)b1;
    }
    __syncthreads();
    wstamp(st, 41 + it);
  }
  if (wid == 0) __builtin_amdgcn_s_setprio(0);
  if (!ok) {
    for (int k = tid; k < n; k += blockDim.x) s.x[k] = 0.0;
    __syncthreads();
  }
  return ok;
}

}  // namespace bad
}  // namespace dpvo
