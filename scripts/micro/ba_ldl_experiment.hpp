// ba_ldl_experiment.hpp -- EXPERIMENT, not shipped (round 3): an alternative
// to dpvo_amd/csrc/ba_solve.hpp, measured slower and kept for the record.
// scripts/micro/ldl_bench.hip / chain_bench.hip time it (build with
// -I scripts/micro -I dpvo_amd/csrc -I include).  Measured on MI355X, N = 11,
// s_memtime cycles: factorisation steps 2.1-3.2k each (look-ahead alone 1.3k,
// the three-wave trailing update the bottleneck), one-wave block chains
// 600-800 per 6-step block (instruction-issue bound: ~50 VALU per block for
// one wave), whole solve 67k against 44k for ba_solve.hpp.
//
// Dense solve of the damped pose Schur complement of a DPVO
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
constexpr int kLdlPad = 16;  // zero rows below row n: 16x16 tiles read past it unmasked
__host__ __device__ constexpr size_t ldl_bytes(int N) {
  return sizeof(float) * ((size_t)(6 * N + 1 + kLdlPad) * ldl_stride(6 * N) +
                          2 * (size_t)(6 * N + 64) + 36 * (size_t)N) +
         sizeof(double) * (size_t)(6 * N) + 16;
}

struct LSolve {
  const double* S;  // [NB][36] damped S, lower 6x6 blocks (a >= b) at lblk(a, b), row-major
  const double* y;  // [n]
  float* A;         // [(n + 1 + kLdlPad) * ls]
  float* rd;        // [n + 64] 1 / D
  float* rv;        // [n + 64] fp32 residual
  double* x;        // [n] solution (fp64)
  float* db;        // [N][36] strictly-lower diagonal blocks of L (chains)
  int* fail;        // LDS int
};

__device__ __forceinline__ LSolve ldl_view(const double* S, const double* y, char* scratch, int N,
                                           int* fail) {
  const int n = 6 * N, ls = ldl_stride(n);
  LSolve v;
  v.S = S;
  v.y = y;
  v.A = reinterpret_cast<float*>(scratch);
  v.rd = v.A + (size_t)(n + 1 + kLdlPad) * ls;
  v.rv = v.rd + n + 64;
  v.x = reinterpret_cast<double*>(v.rv + n + 64);
  v.db = reinterpret_cast<float*>(v.x + n);
  v.fail = fail;
  return v;
}

// s_waitcnt lgkmcnt(0): a loop's first prefetch must land before the loop, or
// the waitcnt pass (which merges the pending state at the loop header)
// waits for every later prefetch at the top of every iteration
__device__ __forceinline__ void lgkm_drain() { __builtin_amdgcn_s_waitcnt(0xc07f); }

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
                                             int lane, long long* st = nullptr) {
  auto stamp = [&](int slot) {
    if (st && w == 0 && lane == 0 && k == 7) st[slot] = (long long)__builtin_amdgcn_s_memtime();
  };
  stamp(50);
  const int r0 = 6 * (k + 2);
  const int nc = n - r0;
  if (nc <= 0) return;
  const int nr = nc + 1;
  const int tr = (nr + 15) >> 4, tc = (nc + 15) >> 4;
  const int i = lane & 15, kq = lane >> 4, c0 = 6 * k;
  const int kq2 = kq < 2 ? 4 + kq : kq;  // k of the second MFMA (6, 7 are zero)
  // lane constants: no clamps anywhere -- rows past n are the zero padding
  // rows (their products are never stored), columns past n - 1 are finite
  // entries whose results are never stored either
  const float rdA = v.rd[c0 + kq];
  const float rdB = (kq < 2) ? v.rd[c0 + kq2] : 0.0f;
  const float mA2 = (kq < 2) ? -1.0f : 0.0f;
  const int offA = i * ls + c0 + kq, offA2 = i * ls + c0 + kq2, offC = 4 * kq * ls + i;
  // lower tiles row by row: rows a < tc hold a + 1 tiles (triangular
  // numbering), row tc (present when tr = tc + 1) holds tc.  This wave takes
  // tiles w, w + 3, ...; closed-form coordinates, no data-dependent loops.
  const int ntri = tc * (tc + 1) / 2;
  const int ntot = ntri + (tr > tc ? tc : 0);
  for (int t0 = w; t0 < ntot; t0 += 12) {
    float xa0[4], xa1[4], xb0[4], xb1[4];
    f32x4 acc[4];
    int rb[4], cb[4];
#pragma unroll
    for (int q = 0; q < 4; q++) {  // tile coordinates (uniform)
      const int t = min(t0 + 3 * q, ntot - 1);
      // row of triangular index t < 21 (tc <= 6): count of triangular numbers <= t
      const int a = (t >= 1) + (t >= 3) + (t >= 6) + (t >= 10) + (t >= 15);
      const bool tail = t >= ntri;
      rb[q] = r0 + 16 * (tail ? tc : a);
      cb[q] = r0 + 16 * (tail ? t - ntri : t - a * (a + 1) / 2);
    }
    // every load of the batch before any use (raw values; scaling below)
#pragma unroll
    for (int q = 0; q < 4; q++) {
      const float* ta = v.A + (size_t)rb[q] * ls;
      const float* tb = v.A + (size_t)cb[q] * ls;
      xa0[q] = ta[offA];
      xa1[q] = ta[offA2];
      xb0[q] = tb[offA];
      xb1[q] = tb[offA2];
#pragma unroll
      for (int j = 0; j < 4; j++) acc[q][j] = ta[offC + j * ls + cb[q]];
    }
    stamp(51);
    // masks are multiplied in, never `c ? load : 0`: clang turns a select of
    // a single-use load into a branch around it, with its own lgkmcnt(0)
#pragma unroll
    for (int q = 0; q < 4; q++) {
      acc[q] = __builtin_amdgcn_mfma_f32_16x16x4f32(-xa0[q], xb0[q] * rdA, acc[q], 0, 0, 0);
      acc[q] = __builtin_amdgcn_mfma_f32_16x16x4f32(xa1[q] * mA2, xb1[q] * rdB, acc[q], 0, 0, 0);
    }
    stamp(52);
#pragma unroll
    for (int q = 0; q < 4; q++) {
      if (t0 + 3 * q >= ntot) break;
      const int col = cb[q] + i;
      float* ta = v.A + (size_t)rb[q] * ls;
#pragma unroll
      for (int j = 0; j < 4; j++) {
        const int row = rb[q] + 4 * kq + j;
        if (row <= n && col < n) ta[offC + j * ls + cb[q]] = acc[q][j];
      }
    }
  }
  stamp(53);
}

// Chains: one wave; entry i of a vector lives in lane i (i < 60, w0) or lane
// i - 60 (i >= 60, w1), so every 6-entry block lives in one register set.
// Before the chains, ldl_prepare_chains stores L = U rd in both triangles of A
// (A[i][k] = L[max(i,k)][min(i,k)]), so the forward pass (row i of L) and the
// backward pass (column i of L) both read a lane's own row: 3 8-B loads per
// block, plus the block's diagonal 6x6 from the compact db (9 16-B loads) --
// few enough LDS loads in flight that waiting for one never waits for the
// next block's prefetch.  A block is one step of the chain: its 6 current
// entries are read with 6 independent readlanes, the 6x6 unit-triangular
// block system is solved redundantly in every lane's registers (5 dependent
// FMAs deep), and every lane applies the block's 6 columns to its own entry
// with the same masked formula, which also leaves each block lane holding
// its own solution.  Block loops stay rolled: the solve runs from a cold
// i-cache, and straight-line code is fetch-bound.
constexpr int kS1 = 60;

// all threads, after the factorisation: L = U rd into both triangles, db
__device__ __forceinline__ void ldl_prepare_chains(const LSolve& v, int N, int ls) {
  const int n = 6 * N;
  // wave index through readfirstlane: the compiler then knows it is uniform
  // (scalar loop control instead of exec-mask loops)
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  const int nw = blockDim.x >> 6;
  for (int k = 1 + wid; k < n; k += nw)  // pairs (k, i), k > i: wave per row, lane per column
    for (int i = lane; i < k; i += 64) {
      const float l = v.A[(size_t)k * ls + i] * v.rd[i];
      v.A[(size_t)k * ls + i] = l;
      v.A[(size_t)i * ls + k] = l;
      if (k / 6 == i / 6) v.db[36 * (k / 6) + 6 * (k % 6) + i % 6] = l;
    }
  for (int t = threadIdx.x; t < 36 * N; t += blockDim.x)
    if ((t % 6) >= (t % 36) / 6) v.db[t] = 0.0f;  // diagonal and upper entries
}

__device__ __forceinline__ void ld36(const float* p, float v[36]) {
  const float4* q = reinterpret_cast<const float4*>(p);
#pragma unroll
  for (int k = 0; k < 9; k++) {
    const float4 t = q[k];
    v[4 * k] = t.x;
    v[4 * k + 1] = t.y;
    v[4 * k + 2] = t.z;
    v[4 * k + 3] = t.w;
  }
}

// wave 0: backward pass L^T x = w in place.  Block b (descending): x_k = w_k -
// sum_{k' > k in b} L[k'][k] x_k'; every w_i (i < 6b + j) -= L[6b + j][i] x_j.
template <bool TWO>
__device__ __forceinline__ void ldl_back(const LSolve& v, int N, int ls, float& w0_io,
                                         float& w1_io, int lane) {
  // values, not references: `hi ? w1 : w0` on references put both in scratch
  float w0 = w0_io, w1 = w1_io;
  const int n = 6 * N;
  const int i0 = min(lane, n - 1), i1 = min(kS1 + lane, n - 1);
  float c0[6], c1[6], m0[6], m1[6], Ld[36], Lm[36];
  auto load = [&](int b, float* q0, float* q1, float* Lq) {
    ld6(v.A + (size_t)i0 * ls + 6 * b, q0);
    if (TWO) ld6(v.A + (size_t)i1 * ls + 6 * b, q1);
    ld36(v.db + 36 * b, Lq);
  };
  load(N - 1, c0, c1, Ld);
  lgkm_drain();
  for (int b = N - 1; b >= 0; b--) {
    if (b > 0) load(b - 1, m0, m1, Lm);
    const bool hi = TWO && 6 * b >= kS1;
    const int base = hi ? 6 * b - kS1 : 6 * b;
    const float src = hi ? w1 : w0;
    float x[6];
#pragma unroll
    for (int j = 0; j < 6; j++) x[j] = rlane(src, base + j);
#pragma unroll
    for (int j = 5; j >= 0; j--)
#pragma unroll
      for (int p = j + 1; p < 6; p++) x[j] -= Ld[6 * p + j] * x[p];
#pragma unroll
    for (int j = 5; j >= 0; j--) {
      const int kx = 6 * b + j;
      w0 -= (lane < kx && lane < kS1 ? c0[j] : 0.0f) * x[j];
      if (TWO && hi) w1 -= (kS1 + lane < kx ? c1[j] : 0.0f) * x[j];
    }
#pragma unroll
    for (int j = 0; j < 6; j++) {
      c0[j] = m0[j];
      if (TWO) c1[j] = m1[j];
    }
#pragma unroll
    for (int j = 0; j < 36; j++) Ld[j] = Lm[j];
  }
  w0_io = w0;
  w1_io = w1;
}

// wave 0: forward pass L u = r in place.  Block b (ascending): u_k = r_k -
// sum_{k' < k in b} L[k][k'] u_k'; every r_i (i > 6b + j) -= L[i][6b + j] u_j.
template <bool TWO>
__device__ __forceinline__ void ldl_fwd(const LSolve& v, int N, int ls, float& r0_io,
                                        float& r1_io, int lane) {
  float r0 = r0_io, r1 = r1_io;
  const int n = 6 * N;
  const int i0 = min(lane, n - 1), i1 = min(kS1 + lane, n - 1);
  const bool l0 = lane < n && lane < kS1, l1 = kS1 + lane < n;
  float c0[6], c1[6], m0[6], m1[6], Ld[36], Lm[36];
  auto load = [&](int b, float* q0, float* q1, float* Lq) {
    ld6(v.A + (size_t)i0 * ls + 6 * b, q0);
    if (TWO) ld6(v.A + (size_t)i1 * ls + 6 * b, q1);
    ld36(v.db + 36 * b, Lq);
  };
  load(0, c0, c1, Ld);
  lgkm_drain();
  for (int b = 0; b < N; b++) {
    if (b + 1 < N) load(b + 1, m0, m1, Lm);
    const bool hi = TWO && 6 * b >= kS1;
    const int base = hi ? 6 * b - kS1 : 6 * b;
    const float src = hi ? r1 : r0;
    float u[6];
#pragma unroll
    for (int j = 0; j < 6; j++) u[j] = rlane(src, base + j);
#pragma unroll
    for (int j = 0; j < 6; j++)
#pragma unroll
      for (int p = 0; p < j; p++) u[j] -= Ld[6 * j + p] * u[p];
#pragma unroll
    for (int j = 0; j < 6; j++) {
      const int kx = 6 * b + j;
      if (!hi) r0 -= (l0 && lane > kx ? c0[j] : 0.0f) * u[j];
      if (TWO) r1 -= (l1 && kS1 + lane > kx ? c1[j] : 0.0f) * u[j];
    }
#pragma unroll
    for (int j = 0; j < 6; j++) {
      c0[j] = m0[j];
      if (TWO) c1[j] = m1[j];
    }
#pragma unroll
    for (int j = 0; j < 36; j++) Ld[j] = Lm[j];
  }
  r0_io = r0;
  r1_io = r1;
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
__device__ __forceinline__ void ldl_chains(const LSolve& v, int N, int ls, int lane) {
  const int n = 6 * N;
  // x0 = L^-T D^-1 u, u = row n of the factor
  const float* un = v.A + (size_t)n * ls;
  const bool e0 = lane < n && lane < kS1, e1 = TWO && kS1 + lane < n;
  float w0 = e0 ? un[lane] * v.rd[lane] : 0.0f;
  float w1 = e1 ? un[kS1 + lane] * v.rd[kS1 + lane] : 0.0f;
  ldl_back<TWO>(v, N, ls, w0, w1, lane);
  if (e0) v.x[lane] = (double)w0;
  if (e1) v.x[kS1 + lane] = (double)w1;
}

template <bool TWO>
__device__ __forceinline__ void ldl_refine_chain(const LSolve& v, int N, int ls, int lane) {
  const int n = 6 * N;
  const bool e0 = lane < n && lane < kS1, e1 = TWO && kS1 + lane < n;
  float r0 = e0 ? v.rv[lane] : 0.0f;
  float r1 = e1 ? v.rv[kS1 + lane] : 0.0f;
  ldl_fwd<TWO>(v, N, ls, r0, r1, lane);
  r0 = e0 ? r0 * v.rd[lane] : 0.0f;
  r1 = e1 ? r1 * v.rd[kS1 + lane] : 0.0f;
  ldl_back<TWO>(v, N, ls, r0, r1, lane);
  if (e0) v.x[lane] += (double)r0;
  if (e1) v.x[kS1 + lane] += (double)r1;
}

// Whole workgroup (blockDim.x == 256, 1 <= N <= 16).  Solves S x = y into
// v.x (fp64).  Returns false (x = 0) if a pivot was not positive (NaN
// included).  Every thread returns after a workgroup barrier.
__device__ __forceinline__ void lstamp(long long* st, int slot) {
  if (st && threadIdx.x == 0) st[slot] = (long long)__builtin_amdgcn_s_memtime();
}

// st (instrumentation, may be null): shader-clock stamps by thread 0 --
// [0] start, [1] copied, [2] panel 0, [3 + k] step k, [40] back chain,
// [41 + 2 it] residual, [42 + 2 it] refinement chains
__device__ inline bool ldl_solve(const LSolve& v, int N, int refine, long long* st = nullptr,
                                 int dbg = 0) {
  const int tid = threadIdx.x, wid = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
  const int n = 6 * N, ls = ldl_stride(n), NB = N * (N + 1) / 2;
  const bool two = n + 1 > 64;  // rows 64.. live in a second register set
  lstamp(st, 0);
  // fp32 copy of S (lower blocks) and y as row n
  // fp32 copy of S (lower blocks), y as row n, and zeros everywhere else (every
  // entry of A finite: the masked loads below multiply by 0).  Task = (row r,
  // 6-column chunk b); chunk N is the row's tail [6N, ls).
  for (int t = tid; t < (n + 1 + kLdlPad) * (N + 1); t += blockDim.x) {
    const int r = t / (N + 1), b = t % (N + 1), a = r / 6, x = r % 6;
    float2* dst = reinterpret_cast<float2*>(v.A + (size_t)r * ls + 6 * b);
    float2 o[3] = {make_float2(0.f, 0.f), make_float2(0.f, 0.f), make_float2(0.f, 0.f)};
    if (b < N && r == n) {
      const double2* src = reinterpret_cast<const double2*>(v.y + 6 * b);
#pragma unroll
      for (int h = 0; h < 3; h++) {
        const double2 d = src[h];
        o[h] = make_float2((float)d.x, (float)d.y);
      }
    } else if (b <= a && b < N) {
      const double2* src = reinterpret_cast<const double2*>(v.S + 36 * lblk(a, b) + 6 * x);
#pragma unroll
      for (int h = 0; h < 3; h++) {
        const double2 d = src[h];
        o[h] = make_float2((float)d.x, (float)d.y);
      }
    }
    const int nw = (b < N) ? 3 : (ls - 6 * N) / 2;
#pragma unroll
    for (int h = 0; h < 3; h++)
      if (h < nw) dst[h] = o[h];
  }
  if (tid == 0) *v.fail = 0;
  __syncthreads();
  lstamp(st, 1);
  // wave 0 carries the pivot chain: let it win issue / LDS arbitration
  if (wid == 0) __builtin_amdgcn_s_setprio(3);
  float rdk[6] = {0, 0, 0, 0, 0, 0};
  bool ok = true;
  if (wid == 0) {  // panel 0
    ok = two ? ldl_lookahead<true>(v, n, ls, -1, rdk, rdk, lane)
             : ldl_lookahead<false>(v, n, ls, -1, rdk, rdk, lane);
  }
  __syncthreads();
  lstamp(st, 2);
  for (int k = 0; k < N; k++) {
    if (wid == 0) {
      if (k + 1 < N && !(dbg & 2)) {
        float rdn[6];
        const bool two_k = n + 1 - 6 * (k + 1) > 64;
        ok = (two_k ? ldl_lookahead<true>(v, n, ls, k, rdk, rdn, lane)
                    : ldl_lookahead<false>(v, n, ls, k, rdk, rdn, lane)) &&
             ok;
#pragma unroll
        for (int c = 0; c < 6; c++) rdk[c] = rdn[c];
      }
    } else if (!(dbg & 1)) {
      ldl_trailing(v, n, ls, k, wid - 1, lane, st);
    }
    __syncthreads();
    lstamp(st, 3 + k);
  }
  if (wid == 0 && !ok && lane == 0) *v.fail = 1;
  ldl_prepare_chains(v, N, ls);
  __syncthreads();
  lstamp(st, 39);
  if (wid == 0) {
    if (n > kS1)
      ldl_chains<true>(v, N, ls, lane);
    else
      ldl_chains<false>(v, N, ls, lane);
    __builtin_amdgcn_s_setprio(0);
  }
  __syncthreads();
  lstamp(st, 40);
  const bool good = *v.fail == 0;
  for (int it = 0; good && it < refine; it++) {
    ldl_residual(v.S, v.y, v.x, v.rv, N);
    __syncthreads();
    lstamp(st, 41 + 2 * it);
    if (wid == 0) {
      if (n > kS1)
        ldl_refine_chain<true>(v, N, ls, lane);
      else
        ldl_refine_chain<false>(v, N, ls, lane);
    }
    __syncthreads();
    lstamp(st, 42 + 2 * it);
  }
  if (!good) {
    for (int t = tid; t < n; t += blockDim.x) v.x[t] = 0.0;
    __syncthreads();
  }
  return good;
}

}  // namespace bad
}  // namespace dpvo
