// ba_gj_mma.hpp -- EXPERIMENT (not in the product; DESIGN.md "F-BA solve",
// round 5): the window solve as a block Gauss-Jordan sweep on the matrix
// cores (the inverse in MFMA accumulators over the four waves, a solve = one
// mat-vec).  Correct (rel. err ~5e-13 vs the host fp64 Cholesky in
// wsolve_bench -DWSOLVE_MMA) but 7k cycles per block step at N = 11 against
// ~1.9k for ba_solve.hpp's Cholesky step: 68k vs 37k cycles per solve.
#pragma once

#include "ba_solve.hpp"

namespace dpvo {
namespace bad {

// ===========================================================================
// wsolve_mma: the inverse by a block Gauss-Jordan sweep on the matrix cores.
//
// The blocked Cholesky above is a chain of N block steps on wave 0 (~2k
// cycles each, mostly LDS round trips under the trailing waves' traffic)
// followed by two forward/backward sweep passes of 2N - 1 dependent steps each
// (~6k cycles per pass): 37k cycles at N = 11.  The sweep operator instead
// keeps the whole (padded, symmetric) matrix in MFMA accumulators spread over
// the four waves and turns it into -A^-1 in N block steps; a solve is then one
// parallel mat-vec.  Block step k (pivot block K = rows / columns 6k .. 6k+5):
//     Q = M_KK^-1,  M_ij -= M_iK Q M_Kj  (i, j not in K),
//     M_iK <- M_iK Q,  M_Kj <- Q M_Kj,  M_KK <- -Q
// (after every block: M = -A^-1).  With M_KK = L L^T and V_i = L^-1 M_iK^T the
// rank-6 update is M -= V V^T: two v_mfma_f32_16x16x4_f32 per 16 x 16 tile,
// applied to every tile; the strip K is then overwritten with M_iK Q = (L^-T
// V_i)^T and -Q.  Per step: the strip's owners publish it (LDS), one barrier,
// a thread per row forms V_i and the new strip value (6 x 6 Cholesky of the
// pivot redundantly per thread, one forward + one backward substitution),
// one barrier, the MFMAs and the strip fix-ups.  The pivots are the LDL^T
// pivots of A (positive for SPD A; no pivoting, as the Cholesky).  fp32
// inverse + fp64 refinement as wsolve: x = A^-1 y, then x += A^-1 (y - S x).
// ===========================================================================
typedef float gjf4 __attribute__((ext_vector_type(4)));

__host__ __device__ constexpr int gj_np(int N) { return 16 * ((6 * N + 15) / 16); }
// Mi [np][np], C / V / W [np][8], v [np] (fp32), x [6N] (fp64)
__host__ __device__ constexpr size_t gj_bytes(int N) {
  return sizeof(float) * ((size_t)gj_np(N) * gj_np(N) + 3 * 8 * (size_t)gj_np(N) + gj_np(N)) +
         sizeof(double) * 6 * (size_t)N;
}
constexpr int kGjMaxT = 6;                            // 96 / 16 (N <= 16)
constexpr int kGjMaxM = (kGjMaxT * kGjMaxT + 3) / 4;  // accumulator tiles per wave

struct GJSolve {
  const double* S;  // [NB][36] damped S, lower blocks (fp64)
  const double* y;  // [6N]
  float* Mi;        // [np][np] A^-1 after the sweep (row-major)
  float* C;         // [np][8] pivot strip of the current step
  float* V;         // [np][8] V_i (columns 6, 7 zero)
  float* W;         // [np][8] the strip's new values
  float* v;         // [np] fp32 right-hand side / residual
  double* x;        // [6N] solution (fp64)
};

__device__ __forceinline__ double gj_s_at(const double* S, int i, int j) {
  const int a = i / 6, x = i % 6, b = j / 6, z = j % 6;
  return a >= b ? S[36 * lblk(a, b) + 6 * x + z] : S[36 * lblk(b, a) + 6 * z + x];
}

// z = L^-T t (backward substitution), L strictly lower + ri
__device__ __forceinline__ void bwd6(const float L[6][6], const float ri[6], const float t[6],
                                     float z[6]) {
#pragma unroll
  for (int q = 5; q >= 0; q--) {
    float s = t[q];
#pragma unroll
    for (int p = q + 1; p < 6; p++) s -= L[p][q] * z[p];
    z[q] = s * ri[q];
  }
}

// x (+)= Mi v over rows < n, fixed summation order: lanes_per_row parts per
// row, each a contiguous run of whole float4s of the row (np is a multiple of
// 16; the padded columns of Mi and v are zero), all loads issued before the sums
__device__ __forceinline__ void gj_matvec(const float* Mi, int np, const float* v, double* x,
                                          int n, bool add) {
  const int tid = threadIdx.x, lpr = lanes_per_row(n), row = tid / lpr, part = tid % lpr;
  const int seg = np / lpr;  // columns per part: a multiple of 4, <= 48
  const int rr = min(row, n - 1), c0 = part * seg;
  const float4* mr = reinterpret_cast<const float4*>(Mi + rr * np + c0);
  const float4* vr = reinterpret_cast<const float4*>(v + c0);
  constexpr int kQ = 12;  // 48 / 4
  float4 a[kQ], b[kQ];
#pragma unroll
  for (int q = 0; q < kQ; q++) {
    const int qq = min(q, seg / 4 - 1);
    a[q] = mr[qq];
    b[q] = vr[qq];
  }
  float s = 0.0f;
#pragma unroll
  for (int q = 0; q < kQ; q++)
    if (4 * q < seg) s += (a[q].x * b[q].x + a[q].y * b[q].y) + (a[q].z * b[q].z + a[q].w * b[q].w);
  s = row_sum(s, lpr);
  if (row < n && part == 0) x[row] = (add ? x[row] : 0.0) + (double)s;
}

// The sweep for TT x TT tiles (np = 16 TT).  Loads from LDS are never inside
// lane-divergent branches (indices clamped, values selected): a load under a
// divergent branch is waited for at the join, one LDS round trip each.
template <int TT>
__device__ __forceinline__ void gj_sweep(const GJSolve& s, int N, int* fail, long long* st) {
  constexpr int np = 16 * TT, nt = TT * TT, kM = (nt + 3) / 4;
  const int tid = threadIdx.x, wid = wave_uniform(tid >> 6), lane = tid & 63;
  const int n = 6 * N;
  const int li = lane & 15, lq = lane >> 4;
  // tile t = wid + 4 m, (I, J) = (t / TT, t % TT) (wave-uniform); the lane
  // holds column 16 J + li, rows 16 I + 4 lq + r (the MFMA D layout);
  // padding: identity
  gjf4 acc[kM];
  int rb[kM], cj[kM], tI[kM], tJ[kM];
#pragma unroll
  for (int m = 0; m < kM; m++) {
    const int t = min(wid + 4 * m, nt - 1);
    tI[m] = t / TT;
    tJ[m] = t % TT;
    rb[m] = 16 * tI[m] + 4 * lq;
    cj[m] = 16 * tJ[m] + li;
    const int j = cj[m], jc = min(j, n - 1);
#pragma unroll
    for (int r = 0; r < 4; r++) {
      const int i = rb[m] + r, ic = min(i, n - 1);
      const float v = (float)gj_s_at(s.S, ic, jc);
      acc[m][r] = (i < n && j < n) ? v : (i == j ? 1.0f : 0.0f);
    }
  }
  for (int k = tid; k < np; k += blockDim.x) s.v[k] = k < n ? (float)s.y[k] : 0.0f;
  wstamp(st, 1);
  for (int k = 0; k < N; k++) {
    const int K0 = 6 * k;
    // ---- the strip's owners publish column block K ----
#pragma unroll
    for (int m = 0; m < kM; m++) {
      if (wid + 4 * m < nt && 16 * tJ[m] < K0 + 6 && 16 * tJ[m] + 16 > K0) {
        const int j = cj[m];
        if (j >= K0 && j < K0 + 6) {
#pragma unroll
          for (int r = 0; r < 4; r++) s.C[(rb[m] + r) * 8 + (j - K0)] = acc[m][r];
        }
      }
    }
    __syncthreads();
    if (st && k == 2 && tid == 0) st[50] = (long long)__builtin_amdgcn_s_memtime();
    // ---- a thread per row: V_i = L^-1 C_i^T and the strip's new value ----
    if (tid < np) {
      const int i = tid;
      float m6[6][6], L[6][6], ri[6];
#pragma unroll
      for (int a = 0; a < 6; a++) {
        const float4 p0 = *reinterpret_cast<const float4*>(s.C + (K0 + a) * 8);
        const float2 p1 = *reinterpret_cast<const float2*>(s.C + (K0 + a) * 8 + 4);
        const float pr[6] = {p0.x, p0.y, p0.z, p0.w, p1.x, p1.y};
#pragma unroll
        for (int b = 0; b <= a; b++) m6[a][b] = pr[b];
      }
      float ci[6];
      {
        const float4 c0 = *reinterpret_cast<const float4*>(s.C + i * 8);
        const float2 c1 = *reinterpret_cast<const float2*>(s.C + i * 8 + 4);
        ci[0] = c0.x; ci[1] = c0.y; ci[2] = c0.z; ci[3] = c0.w; ci[4] = c1.x; ci[5] = c1.y;
      }
      const bool ok = chol6_m(m6, L, ri);
      if (!ok && i == 0) *fail = 1;
      const bool inK = i >= K0 && i < K0 + 6;
      float tv[6], r2[6], t2[6], u[6];
      fwd6(L, ri, ci, tv);
#pragma unroll
      for (int q = 0; q < 6; q++) r2[q] = inK ? ((q == i - K0) ? 1.0f : 0.0f) : ci[q];
      fwd6(L, ri, r2, t2);
      bwd6(L, ri, t2, u);
      float* vo = s.V + i * 8;
      float* wo = s.W + i * 8;
      *reinterpret_cast<float4*>(vo) = make_float4(tv[0], tv[1], tv[2], tv[3]);
      *reinterpret_cast<float4*>(vo + 4) = make_float4(tv[4], tv[5], 0.0f, 0.0f);
      const float sg = inK ? -1.0f : 1.0f;
      *reinterpret_cast<float4*>(wo) = make_float4(sg * u[0], sg * u[1], sg * u[2], sg * u[3]);
      *reinterpret_cast<float2*>(wo + 4) = make_float2(sg * u[4], sg * u[5]);
    }
    if (st && k == 2 && tid == 0) st[51] = (long long)__builtin_amdgcn_s_memtime();
    __syncthreads();
    if (st && k == 2 && tid == 0) st[52] = (long long)__builtin_amdgcn_s_memtime();
    // ---- M -= V V^T on every tile (all operand loads first), then the strip ----
    float a0[kM], a1[kM], b0[kM], b1[kM];
#pragma unroll
    for (int m = 0; m < kM; m++) {
      const float* va = s.V + (rb[m] - 4 * lq + li) * 8 + lq;  // row 16 I + li
      const float* vb = s.V + cj[m] * 8 + lq;
      a0[m] = -va[0];
      a1[m] = -va[4];
      b0[m] = vb[0];
      b1[m] = vb[4];
    }
#pragma unroll
    for (int m = 0; m < kM; m++)
      if (wid + 4 * m < nt) acc[m] = __builtin_amdgcn_mfma_f32_16x16x4f32(a0[m], b0[m], acc[m], 0, 0, 0);
#pragma unroll
    for (int m = 0; m < kM; m++)
      if (wid + 4 * m < nt) acc[m] = __builtin_amdgcn_mfma_f32_16x16x4f32(a1[m], b1[m], acc[m], 0, 0, 0);
    if (st && k == 2 && tid == 0) st[53] = (long long)__builtin_amdgcn_s_memtime();
    // strip values: column K (W[i][j - K0]) or row K (W[j][i - K0]); every
    // tile's loads first (clamped indices), then the selects
    float wc[kM][4], wr[kM][4];
#pragma unroll
    for (int m = 0; m < kM; m++) {
      const int j = cj[m], jk = min(max(j - K0, 0), 5);
#pragma unroll
      for (int r = 0; r < 4; r++) {
        const int i = rb[m] + r, ik = min(max(i - K0, 0), 5);
        wc[m][r] = s.W[i * 8 + jk];
        wr[m][r] = s.W[j * 8 + ik];
      }
    }
#pragma unroll
    for (int m = 0; m < kM; m++) {
      const int j = cj[m];
      const bool colK = j >= K0 && j < K0 + 6;
#pragma unroll
      for (int r = 0; r < 4; r++) {
        const int i = rb[m] + r;
        const bool rowK = i >= K0 && i < K0 + 6;
        acc[m][r] = colK ? wc[m][r] : (rowK ? wr[m][r] : acc[m][r]);
      }
    }
    wstamp(st, 2 + k);
  }
  // ---- A^-1 = -M to LDS ----
#pragma unroll
  for (int m = 0; m < kM; m++) {
    if (wid + 4 * m < nt) {
#pragma unroll
      for (int r = 0; r < 4; r++) s.Mi[(rb[m] + r) * np + cj[m]] = -acc[m][r];
    }
  }
  __syncthreads();
}

// Whole workgroup (blockDim.x == 256, 1 <= N <= 16).  Solves S x = y into s.x
// (fp64); false (x = 0) if a pivot was not positive.  `fail` is an LDS int.
// st (instrumentation, may be null): [0] start, [1] loaded, [2 + k] block step
// k done, [40] inverse stored, [41] first solve, [42 + it] refinement it.
__device__ inline bool wsolve_mma(const GJSolve& s, int N, int refine, int* fail,
                                  long long* st = nullptr) {
  const int tid = threadIdx.x, n = 6 * N, np = gj_np(N);
  wstamp(st, 0);
  if (tid == 0) *fail = 0;
  switch (np / 16) {
    case 1: gj_sweep<1>(s, N, fail, st); break;
    case 2: gj_sweep<2>(s, N, fail, st); break;
    case 3: gj_sweep<3>(s, N, fail, st); break;
    case 4: gj_sweep<4>(s, N, fail, st); break;
    case 5: gj_sweep<5>(s, N, fail, st); break;
    default: gj_sweep<6>(s, N, fail, st); break;
  }
  wstamp(st, 40);
  const bool ok = *fail == 0;
  gj_matvec(s.Mi, np, s.v, s.x, n, false);
  __syncthreads();
  wstamp(st, 41);
  for (int it = 0; it < refine && ok; it++) {
    residual64(s.S, s.y, s.x, s.v, N);
    __syncthreads();
    gj_matvec(s.Mi, np, s.v, s.x, n, true);
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
