// ba_ldl.hpp -- dense solve of the damped pose Schur complement of a DPVO
// window, S dX = y (ba_cuda.cu:560-562: L = chol(S); dX = cholesky_solve),
// by ONE 256-thread workgroup, latency-first.
//
// S is at most 96 x 96 (N <= 16 free poses).  The flops are few (n^3/6 ~ 5e4
// at N = 11); the time is the dependency chain of n pivots.  Design
// (DESIGN.md "F-BA solve"):
//   * fp32 LDL^T (no square roots), right-looking by 6-column panels with
//     look-ahead.  Wave 0 owns the chain: a panel lives in its registers, one
//     matrix row per lane (rows 64.. in a second register set), and a column
//     step is readlane(pivot) -> rcp -> readlane(row entries) -> FMAs: no LDS
//     round trip and no barrier inside a panel.  At step k wave 0 applies
//     panel k to column block k+1 and factors it; waves 1-3 meanwhile apply
//     panel k to the trailing matrix with v_mfma_f32_16x16x4_f32 (a rank-6
//     update per 16x16 tile, exact fp32 FMA chains).  One workgroup barrier
//     per panel.
//   * y rides along as row n of the matrix, so the factorisation also leaves
//     u = L^-1 y (unit-lower L) in that row: no separate forward pass.
//   * Triangular chains (x = L^-T D^-1 u, and the refinement's forward and
//     backward passes) are one wave, one pivot per step: readlane + FMA, the
//     factor entries of the next 6 steps prefetched from LDS.
//   * One fp64 refinement step: r = y - S x with the fp64 S (all waves), then
//     x += S~^-1 r through the same factor.  A dependent fp64 FMA costs ~36
//     cycles on gfx950 against ~8 for fp32, so the chains run in fp32 and the
//     accuracy comes back from the (parallel) fp64 residual:
//     ||dx - dx_64|| / ||dx_64|| ~ (kappa eps32)^2.
// Storage (LDS): A = fp32 [(n + 1) rows][ls], row-major; column blocks < k hold
// U = L D (the un-scaled factor; L = U D^-1), the rest the matrix being
// reduced; rd = 1 / D.  The row stride ls is = 2 (mod 4), so 32 lanes reading
// 8 B of 32 consecutive rows hit 64 distinct banks.
#pragma once

#include "ba_device.hpp"

namespace dpvo {
namespace bad {

__host__ __device__ constexpr int ldl_stride(int n) { return ((n + 2) & 3) == 0 ? n + 4 : n + 2; }

// scratch bytes of ldl_solve for N free poses (16-B aligned base)
__host__ __device__ constexpr size_t ldl_bytes(int N) {
  return sizeof(float) * ((size_t)(6 * N + 1) * ldl_stride(6 * N) + 2 * (size_t)(6 * N + 64)) +
         sizeof(double) * (size_t)(6 * N) + 16;
}

struct LSolve {
  const double* S;  // [NB][36] damped S, lower 6x6 blocks (a >= b) at lblk(a, b), row-major
  const double* y;  // [n]
  float* A;         // [(n + 1) * ls]
  float* rd;        // [n + 64] 1 / D
  float* rv;        // [n + 64] fp32 residual
  double* x;        // [n] solution (fp64)
  int* fail;        // LDS int
};

__device__ __forceinline__ LSolve ldl_view(const double* S, const double* y, char* scratch, int N,
                                           int* fail) {
  const int n = 6 * N, ls = ldl_stride(n);
  LSolve v;
  v.S = S;
  v.y = y;
  v.A = reinterpret_cast<float*>(scratch);
  v.rd = v.A + (size_t)(n + 1) * ls;
  v.rv = v.rd + n + 64;
  v.x = reinterpret_cast<double*>(v.rv + n + 64);
  v.fail = fail;
  return v;
}

__device__ __forceinline__ float rlane(float v, int l) {
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), l));
}

// 6 consecutive floats at an 8-B aligned LDS address
__device__ __forceinline__ void ld6(const float* p, float v[6]) {
  const float2* q = reinterpret_cast<const float2*>(p);
#pragma unroll
  for (int k = 0; k < 3; k++) {
    const float2 t = q[k];
    v[2 * k] = t.x;
    v[2 * k + 1] = t.y;
  }
}
__device__ __forceinline__ void st6(float* p, const float v[6]) {
  float2* q = reinterpret_cast<float2*>(p);
#pragma unroll
  for (int k = 0; k < 3; k++) q[k] = make_float2(v[2 * k], v[2 * k + 1]);
}

// LDL^T of a 6-column panel held one row per lane (p0: rows R0 + lane, p1:
// rows R0 + 64 + lane); the panel's first 6 rows are its diagonal block, in
// lanes 0..5.  On return p holds U = L D of the rows (entries above the
// diagonal of the diagonal block are don't-care) and rdv[c] = 1 / D_c.
template <bool TWO>
__device__ __forceinline__ bool ldl_panel(float p0[6], float p1[6], float rdv[6]) {
  bool ok = true;
#pragma unroll
  for (int c = 0; c < 6; c++) {
    const float d = rlane(p0[c], c);
    ok = ok && (d > 0.0f);
    const float r = __builtin_amdgcn_rcpf(d);
    rdv[c] = r;
    const float l0 = p0[c] * r;
    const float l1 = TWO ? p1[c] * r : 0.0f;
#pragma unroll
    for (int c2 = c + 1; c2 < 6; c2++) {
      const float s = rlane(p0[c], c2);  // A[R0 + c2][c], current
      p0[c2] -= l0 * s;
      if (TWO) p1[c2] -= l1 * s;
    }
  }
  return ok;
}

// wave 0: apply panel k (k < 0: none) to column block kn = k + 1, rows
// 6 kn .. n (row n = y), factor it and store U and rd.  rdk: rd of panel k.
template <bool TWO>
__device__ __forceinline__ bool ldl_lookahead(const LSolve& v, int n, int ls, int k,
                                              const float rdk[6], float rdn[6], int lane) {
  const int kn = k + 1, R0 = 6 * kn, cnt = n + 1 - R0;
  const int row0 = R0 + min(lane, cnt - 1);
  const int row1 = R0 + min(64 + lane, cnt - 1);
  float a0[6], a1[6];
  ld6(v.A + (size_t)row0 * ls + R0, a0);
  if (TWO) ld6(v.A + (size_t)row1 * ls + R0, a1);
  if (k >= 0) {
    const int c0 = 6 * k;
    float u0[6], u1[6], K[36];
    ld6(v.A + (size_t)row0 * ls + c0, u0);
    if (TWO) ld6(v.A + (size_t)row1 * ls + c0, u1);
#pragma unroll
    for (int z = 0; z < 6; z++) ld6(v.A + (size_t)(R0 + z) * ls + c0, K + 6 * z);  // broadcast
#pragma unroll
    for (int c = 0; c < 6; c++) {
      u0[c] *= rdk[c];  // L = U D^-1
      if (TWO) u1[c] *= rdk[c];
    }
#pragma unroll
    for (int z = 0; z < 6; z++)
#pragma unroll
      for (int c = 0; c < 6; c++) {
        a0[z] -= u0[c] * K[6 * z + c];
        if (TWO) a1[z] -= u1[c] * K[6 * z + c];
      }
  }
  const bool ok = ldl_panel<TWO>(a0, a1, rdn);
  if (lane < cnt) st6(v.A + (size_t)row0 * ls + R0, a0);
  if (TWO && 64 + lane < cnt) st6(v.A + (size_t)row1 * ls + R0, a1);
  float r = rdn[0];
#pragma unroll
  for (int c = 1; c < 6; c++) r = (lane == c) ? rdn[c] : r;
  if (lane < 6) v.rd[R0 + lane] = r;
  return ok;
}

typedef float f32x4 __attribute__((ext_vector_type(4)));

// waves 1..3: apply panel k to the trailing matrix, rows r0 .. n (row n = y),
// columns r0 .. n-1, r0 = 6 (k + 2): A -= U_k D^-1 U_k^T over lower 16x16
// tiles (a diagonal tile is computed whole; its upper half is don't-care).
// Tiles are dealt round-robin to the three waves; a wave loads the operands
// of up to 4 tiles before its first MFMA.
__device__ __forceinline__ void ldl_trailing(const LSolve& v, int n, int ls, int k, int w,
                                             int lane) {
  const int r0 = 6 * (k + 2);
  const int nc = n - r0;
  if (nc <= 0) return;
  const int nr = nc + 1;
  const int tr = (nr + 15) >> 4, tc = (nc + 15) >> 4;
  const int i = lane & 15, kq = lane >> 4, c0 = 6 * k;
  const float rdA = v.rd[c0 + kq];
  const float rdB = (kq < 2) ? v.rd[c0 + 4 + kq] : 0.0f;
  // this wave's tiles, in order
  int tl[8];
  int nt = 0, t = 0;
  for (int a = 0; a < tr; a++)
    for (int b = 0; b <= a && b < tc; b++, t++)
      if (t % 3 == w && nt < 8) tl[nt++] = (a << 8) | b;
  for (int t0 = 0; t0 < nt; t0 += 4) {
    float af0[4], af1[4], bf0[4], bf1[4];
    f32x4 acc[4];
#pragma unroll
    for (int q = 0; q < 4; q++) {
      const bool live = t0 + q < nt;
      const int a = live ? (tl[t0 + q] >> 8) : 0, b = live ? (tl[t0 + q] & 0xff) : 0;
      const int rb = r0 + 16 * a, cb = r0 + 16 * b;
      const bool av = live && rb + i <= n, bv = live && cb + i < n;
      const float* ar = v.A + (size_t)min(rb + i, n) * ls + c0;
      const float* bc = v.A + (size_t)min(cb + i, n - 1) * ls + c0;
      af0[q] = av ? -ar[kq] : 0.0f;
      af1[q] = (av && kq < 2) ? -ar[4 + kq] : 0.0f;
      bf0[q] = bv ? bc[kq] * rdA : 0.0f;
      bf1[q] = (bv && kq < 2) ? bc[4 + kq] * rdB : 0.0f;
      const int col = cb + i;
#pragma unroll
      for (int j = 0; j < 4; j++) {
        const int row = rb + 4 * kq + j;
        acc[q][j] = (live && row <= n && col < n) ? v.A[(size_t)row * ls + col] : 0.0f;
      }
    }
#pragma unroll
    for (int q = 0; q < 4; q++) {
      acc[q] = __builtin_amdgcn_mfma_f32_16x16x4f32(af0[q], bf0[q], acc[q], 0, 0, 0);
      acc[q] = __builtin_amdgcn_mfma_f32_16x16x4f32(af1[q], bf1[q], acc[q], 0, 0, 0);
    }
#pragma unroll
    for (int q = 0; q < 4; q++) {
      if (t0 + q >= nt) break;
      const int a = tl[t0 + q] >> 8, b = tl[t0 + q] & 0xff;
      const int rb = r0 + 16 * a, col = r0 + 16 * b + i;
#pragma unroll
      for (int j = 0; j < 4; j++) {
        const int row = rb + 4 * kq + j;
        if (row <= n && col < n) v.A[(size_t)row * ls + col] = acc[q][j];
      }
    }
  }
}

// wave 0: backward pass L^T x = w in place (w0: entry lane, w1: entry 64 + lane).
// Step k: x_k = w_k; w_i -= L[k][i] x_k (i < k), L[k][i] = U[k][i] rd[i].
template <bool TWO>
__device__ __forceinline__ void ldl_back(const LSolve& v, int N, int ls, float& w0, float& w1,
                                         int lane) {
  const int n = 6 * N;
  const float rd0 = (lane < n) ? v.rd[lane] : 0.0f;
  const float rd1 = (TWO && 64 + lane < n) ? v.rd[64 + lane] : 0.0f;
  float c0[6], c1[6], m0[6], m1[6];
  auto load = [&](int b, float* q0, float* q1) {
#pragma unroll
    for (int j = 0; j < 6; j++) {
      const int kx = 6 * b + j;
      const float* row = v.A + (size_t)kx * ls;
      q0[j] = (lane < kx) ? row[lane] * rd0 : 0.0f;
      if (TWO) q1[j] = (64 + lane < kx) ? row[64 + lane] * rd1 : 0.0f;
    }
  };
  load(N - 1, c0, c1);
  for (int b = N - 1; b >= 0; b--) {
    if (b > 0) load(b - 1, m0, m1);
#pragma unroll
    for (int j = 5; j >= 0; j--) {
      const int kx = 6 * b + j;
      float x;
      if (TWO)
        x = (kx >= 64) ? rlane(w1, (kx - 64) & 63) : rlane(w0, kx & 63);
      else
        x = rlane(w0, kx & 63);
      w0 -= c0[j] * x;
      if (TWO) w1 -= c1[j] * x;
    }
#pragma unroll
    for (int j = 0; j < 6; j++) {
      c0[j] = m0[j];
      if (TWO) c1[j] = m1[j];
    }
  }
}

// wave 0: forward pass L u = r in place.  Step k: u_k = r_k; r_i -= L[i][k] u_k
// (i > k), L[i][k] = U[i][k] rd[k]: a lane's own row, 6 entries per block.
template <bool TWO>
__device__ __forceinline__ void ldl_fwd(const LSolve& v, int N, int ls, float& r0, float& r1,
                                        int lane) {
  const int n = 6 * N;
  const int i0 = min(lane, n - 1), i1 = min(64 + lane, n - 1);
  float c0[6], c1[6], m0[6], m1[6];
  auto load = [&](int b, float* q0, float* q1) {
    float rdb[6], u0[6], u1[6];
    ld6(v.rd + 6 * b, rdb);  // broadcast
    ld6(v.A + (size_t)i0 * ls + 6 * b, u0);
    if (TWO) ld6(v.A + (size_t)i1 * ls + 6 * b, u1);
#pragma unroll
    for (int j = 0; j < 6; j++) {
      const int kx = 6 * b + j;
      q0[j] = (lane > kx && lane < n) ? u0[j] * rdb[j] : 0.0f;
      if (TWO) q1[j] = (64 + lane > kx && 64 + lane < n) ? u1[j] * rdb[j] : 0.0f;
    }
  };
  load(0, c0, c1);
  for (int b = 0; b < N; b++) {
    if (b + 1 < N) load(b + 1, m0, m1);
#pragma unroll
    for (int j = 0; j < 6; j++) {
      const int kx = 6 * b + j;
      float u;
      if (TWO)
        u = (kx >= 64) ? rlane(r1, (kx - 64) & 63) : rlane(r0, kx & 63);
      else
        u = rlane(r0, kx & 63);
      r0 -= c0[j] * u;
      if (TWO) r1 -= c1[j] * u;
    }
#pragma unroll
    for (int j = 0; j < 6; j++) {
      c0[j] = m0[j];
      if (TWO) c1[j] = m1[j];
    }
  }
}

// out = (float) (y - S x) in fp64, whole workgroup (S lower blocks, symmetric)
__device__ __forceinline__ void ldl_residual(const double* S, const double* y, const double* x,
                                             float* out, int N) {
  const int n = 6 * N, lpr = n <= 64 ? 4 : 2;
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
  double s = s0 + s1;
  s += __shfl_xor(s, 1, 64);
  if (lpr == 4) s += __shfl_xor(s, 2, 64);
  if (row < n && part == 0) out[row] = (float)(y[row] - s);
}

template <bool TWO>
__device__ __forceinline__ void ldl_chains(const LSolve& v, int N, int ls, int refine, int lane) {
  const int n = 6 * N;
  // x0 = L^-T D^-1 u, u = row n of the factor
  const float* un = v.A + (size_t)n * ls;
  float w0 = (lane < n) ? un[lane] * v.rd[lane] : 0.0f;
  float w1 = (TWO && 64 + lane < n) ? un[64 + lane] * v.rd[64 + lane] : 0.0f;
  ldl_back<TWO>(v, N, ls, w0, w1, lane);
  if (lane < n) v.x[lane] = (double)w0;
  if (TWO && 64 + lane < n) v.x[64 + lane] = (double)w1;
  (void)refine;
}

template <bool TWO>
__device__ __forceinline__ void ldl_refine_chain(const LSolve& v, int N, int ls, int lane) {
  const int n = 6 * N;
  float r0 = (lane < n) ? v.rv[lane] : 0.0f;
  float r1 = (TWO && 64 + lane < n) ? v.rv[64 + lane] : 0.0f;
  ldl_fwd<TWO>(v, N, ls, r0, r1, lane);
  r0 *= (lane < n) ? v.rd[lane] : 0.0f;
  if (TWO) r1 *= (64 + lane < n) ? v.rd[64 + lane] : 0.0f;
  ldl_back<TWO>(v, N, ls, r0, r1, lane);
  if (lane < n) v.x[lane] += (double)r0;
  if (TWO && 64 + lane < n) v.x[64 + lane] += (double)r1;
}

// Whole workgroup (blockDim.x == 256, 1 <= N <= 16).  Solves S x = y into
// v.x (fp64).  Returns false (x = 0) if a pivot was not positive (NaN
// included).  Every thread returns after a workgroup barrier.
__device__ inline bool ldl_solve(const LSolve& v, int N, int refine) {
  const int tid = threadIdx.x, wid = tid >> 6, lane = tid & 63;
  const int n = 6 * N, ls = ldl_stride(n), NB = N * (N + 1) / 2;
  const bool two = n + 1 > 64;  // rows 64.. live in a second register set
  // fp32 copy of S (lower blocks) and y as row n
  for (int t = tid; t < 36 * NB; t += blockDim.x) {
    const int blk = t / 36, e = t % 36;
    int a, b;
    tri_of(blk, a, b);
    v.A[(size_t)(6 * a + e / 6) * ls + 6 * b + e % 6] = (float)v.S[t];
  }
  for (int t = tid; t < n; t += blockDim.x) v.A[(size_t)n * ls + t] = (float)v.y[t];
  if (tid == 0) *v.fail = 0;
  __syncthreads();
  // wave 0 carries the pivot chain: let it win issue / LDS arbitration
  if (wid == 0) __builtin_amdgcn_s_setprio(3);
  float rdk[6] = {0, 0, 0, 0, 0, 0};
  bool ok = true;
  if (wid == 0) {  // panel 0
    ok = two ? ldl_lookahead<true>(v, n, ls, -1, rdk, rdk, lane)
             : ldl_lookahead<false>(v, n, ls, -1, rdk, rdk, lane);
  }
  __syncthreads();
  for (int k = 0; k < N; k++) {
    if (wid == 0) {
      if (k + 1 < N) {
        float rdn[6];
        const bool two_k = n + 1 - 6 * (k + 1) > 64;
        ok = (two_k ? ldl_lookahead<true>(v, n, ls, k, rdk, rdn, lane)
                    : ldl_lookahead<false>(v, n, ls, k, rdk, rdn, lane)) &&
             ok;
#pragma unroll
        for (int c = 0; c < 6; c++) rdk[c] = rdn[c];
      }
    } else {
      ldl_trailing(v, n, ls, k, wid - 1, lane);
    }
    __syncthreads();
  }
  if (wid == 0) {
    if (!ok && lane == 0) *v.fail = 1;
    if (n > 64)
      ldl_chains<true>(v, N, ls, refine, lane);
    else
      ldl_chains<false>(v, N, ls, refine, lane);
    __builtin_amdgcn_s_setprio(0);
  }
  __syncthreads();
  const bool good = *v.fail == 0;
  for (int it = 0; good && it < refine; it++) {
    ldl_residual(v.S, v.y, v.x, v.rv, N);
    __syncthreads();
    if (wid == 0) {
      if (n > 64)
        ldl_refine_chain<true>(v, N, ls, lane);
      else
        ldl_refine_chain<false>(v, N, ls, lane);
    }
    __syncthreads();
  }
  if (!good) {
    for (int t = tid; t < n; t += blockDim.x) v.x[t] = 0.0;
    __syncthreads();
  }
  return good;
}

}  // namespace bad
}  // namespace dpvo
