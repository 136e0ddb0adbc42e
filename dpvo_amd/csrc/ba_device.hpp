// ba_device.hpp -- device code shared by the F-BA window kernel (ba_window.hip,
// via ba_solve.hpp): the reference's fp32 edge linearisation, block scan, the
// 6x6 LDL^T pivot factorisation and small index helpers.
#pragma once

#include "common.hpp"

namespace dpvo {
namespace bad {

__device__ __forceinline__ int lblk(int a, int b) { return a * (a + 1) / 2 + b; }  // a >= b

__device__ __forceinline__ void tri_of(int bt, int& a, int& b) {  // bt -> (a, b), a >= b
  int r = (int)((sqrtf(8.0f * bt + 1.0f) - 1.0f) * 0.5f);
  while (r * (r + 1) / 2 > bt) r--;
  while ((r + 1) * (r + 2) / 2 <= bt) r++;
  a = r;
  b = bt - r * (r + 1) / 2;
}

// block-wide exclusive scan of LDS ints data[0..n), returns the total.  Each
// thread owns a contiguous run of at most kScanRun elements whose loads are
// all issued before the first add (one LDS latency, not one per element).
constexpr int kScanRun = 16;
// pack_shift > 0: each input c is first replaced by (c << pack_shift) | (c > 0),
// so one scan gives both the exclusive prefix of c (high bits) and the number
// of nonzero entries before (low bits) -- bucket starts and bucket indices.
__device__ inline int fscan(int* data, int n, int* scr, int pack_shift = 0) {
  const int tid = threadIdx.x, nt = blockDim.x;
  if (n <= 0) {
    // keep the barrier of every other path: callers rely on it to order their
    // LDS atomics before reading the results (plan_sharded's ctl[4..6] on a
    // shard with an empty kk range)
    __syncthreads();
    return 0;
  }
  if (n <= 64 * kScanRun) {
    // small scans (the plan's shard ranges, the BA setup's patch counts at
    // cfg2): wave 0 alone, one DPP scan, two barriers instead of three
    if (tid < 64) {
      const int per = (n + 63) / 64;
      const int lo = min(tid * per, n), hi = min(lo + per, n);
      int v[kScanRun];
#pragma unroll
      for (int k = 0; k < kScanRun; k++) {
        const int d = data[min(lo + k, max(n - 1, 0))];
        v[k] = (lo + k < hi) ? d : 0;
        if (pack_shift > 0) v[k] = (v[k] << pack_shift) | (v[k] > 0 ? 1 : 0);
      }
      int sum = 0;
#pragma unroll
      for (int k = 0; k < kScanRun; k++) sum += v[k];
      const int x = wave_incl_sum(sum);
      int run = x - sum;
#pragma unroll
      for (int k = 0; k < kScanRun; k++)
        if (lo + k < hi) {
          data[lo + k] = run;
          run += v[k];
        }
      if (tid == 63) scr[0] = x;
    }
    __syncthreads();
    const int total = scr[0];
    __syncthreads();  // scr[0] read everywhere before the next scan writes it
    return total;
  }
  const int per = (n + nt - 1) / nt;
  int total = 0;
  for (int base = 0; base < n; base += nt * kScanRun) {  // chunks of nt * kScanRun
    const int cn = min(n - base, nt * kScanRun);
    const int cper = min(per, kScanRun);
    const int lo = base + min(tid * cper, cn), hi = base + min(tid * cper + cper, cn);
    int v[kScanRun];
#pragma unroll
    for (int k = 0; k < kScanRun; k++) {  // unconditional read, then select (no branch per load)
      const int d = data[min(lo + k, n - 1)];
      v[k] = (lo + k < hi) ? d : 0;
    }
    if (pack_shift > 0) {
#pragma unroll
      for (int k = 0; k < kScanRun; k++) v[k] = (v[k] << pack_shift) | (v[k] > 0 ? 1 : 0);
    }
    int s = 0;
#pragma unroll
    for (int k = 0; k < kScanRun; k++) s += v[k];
    const int lane = tid & 63, wid = tid >> 6, nw = nt / 64;
    const int x = wave_incl_sum(s);  // DPP: no LDS round trip per step
    if (lane == 63) scr[wid] = x;
    __syncthreads();
    if (wid == 0) {  // exclusive prefix of the (<= 16) wave totals, one DPP scan
      const int y = lane < nw ? scr[lane] : 0;
      const int inc = wave_incl_sum(y);
      if (lane < nw) scr[lane] = inc - y;
      if (lane == nw - 1) scr[nw] = inc;
    }
    __syncthreads();
    int run = total + scr[wid] + x - s;
#pragma unroll
    for (int k = 0; k < kScanRun; k++)
      if (lo + k < hi) {
        data[lo + k] = run;
        run += v[k];
      }
    total += scr[nt / 64];
    __syncthreads();
  }
  return total;
}

// ---------------------------------------------------------------------------
// fp32 edge linearisation, ba_cuda.cu:265-333 (operation order of the C
// oracle; no contraction).
// ---------------------------------------------------------------------------
struct Lin {
  float w[2], r[2], Jz[2], Ji[2][6], Jj[2][6];
};

#pragma clang fp contract(off)
__device__ __forceinline__ void lin_edge(const float* Pi, const float* Pj, float nx, float ny,
                                         float depth, float tx, float ty, float wx, float wy,
                                         float fx, float fy, float cx, float cy, Lin& o) {
  float ti[3] = {Pi[0], Pi[1], Pi[2]}, qi[4] = {Pi[3], Pi[4], Pi[5], Pi[6]};
  float tj[3] = {Pj[0], Pj[1], Pj[2]}, qj[4] = {Pj[3], Pj[4], Pj[5], Pj[6]};
  float Xi[4], Xj[4];
  Xi[0] = nx;  // (x - cx) / fx, per patch
  Xi[1] = ny;
  Xi[2] = 1.0f;
  Xi[3] = depth;
  float tij[3], qij[4];
  relSE3(ti, qi, tj, qj, tij, qij);
  actSE3(tij, qij, Xi, Xj);
  const float X = Xj[0], Y = Xj[1], Z = Xj[2], W = Xj[3];
  const float d = ((double)Z >= 0.2) ? (float)(1.0 / (double)Z) : 0.0f;  // ba_cuda.cu:296
  const float d2 = d * d;
  const float x1 = fx * (X / Z) + cx;
  const float y1 = fy * (Y / Z) + cy;
  const float rx = tx - x1, ry = ty - y1;
  const bool in_bounds = (sqrtf(rx * rx + ry * ry) < 128.0f) && ((double)Z > 0.2) &&
                         (x1 > -64.0f) && (y1 > -64.0f) && (x1 < 2.0f * cx + 64.0f) &&
                         (y1 < 2.0f * cy + 64.0f);  // :305-306
  const float mask = in_bounds ? 1.0f : 0.0f;
  o.w[0] = mask * wx;
  o.w[1] = mask * wy;
  o.r[0] = rx;
  o.r[1] = ry;
  o.Jz[0] = fx * (tij[0] * d - tij[2] * (X * d2));
  o.Jz[1] = fy * (tij[1] * d - tij[2] * (Y * d2));
  o.Jj[0][0] = fx * W * d;
  o.Jj[0][1] = 0.0f;
  o.Jj[0][2] = fx * -X * W * d2;
  o.Jj[0][3] = fx * -X * Y * d2;
  o.Jj[0][4] = fx * (1 + X * X * d2);
  o.Jj[0][5] = fx * -Y * d;
  o.Jj[1][0] = 0.0f;
  o.Jj[1][1] = fy * W * d;
  o.Jj[1][2] = fy * -Y * W * d2;
  o.Jj[1][3] = fy * (-1 - Y * Y * d2);
  o.Jj[1][4] = fy * (X * Y * d2);
  o.Jj[1][5] = fy * X * d;
  adjSE3(tij, qij, o.Jj[0], o.Ji[0]);
  adjSE3(tij, qij, o.Jj[1], o.Ji[1]);
}
#pragma clang fp contract(fast)

// v_rcp_f64 (~2^-24 relative) + one Newton step (~2^-48): the pivot
// reciprocals sit on the solve's dependency chain, where each dependent fp64
// FMA costs ~36 cycles on gfx950
__device__ __forceinline__ double rcp64(double d) {
  const double r = __builtin_amdgcn_rcp(d);
  return __builtin_fma(r, __builtin_fma(-d, r, 1.0), r);
}

// one lane: LDL^T of the (lower triangle of the) 6x6 pivot block and
// w = L^-1 y.  piv: L strictly lower, 1/D on the diagonal.  false if a pivot
// is not positive (the Cholesky failure of ba_cuda.cu:561 / dpvo/ba.py:17-21).
__device__ inline bool ldl6(const double* Skk, const double* yk, double* piv, double* wk) {
  double a[6][6], w[6];
#pragma unroll
  for (int r = 0; r < 6; r++) {
#pragma unroll
    for (int c = 0; c <= r; c++) a[r][c] = Skk[6 * r + c];
    w[r] = yk[r];
  }
  bool ok = true;
#pragma unroll
  for (int c = 0; c < 6; c++) {
    const double d = a[c][c];
    ok = ok && (d > 0.0);
    const double r = rcp64(d);
    piv[7 * c] = r;
#pragma unroll
    for (int i = c + 1; i < 6; i++) {
      const double l = a[i][c] * r;
      piv[6 * i + c] = l;
#pragma unroll
      for (int j = c + 1; j <= i; j++) a[i][j] -= l * a[j][c];
      w[i] -= l * w[c];
    }
  }
#pragma unroll
  for (int r = 0; r < 6; r++) wk[r] = w[r];
  return ok;
}

// ---------------------------------------------------------------------------
// Dense solve of the damped pose Schur complement S dX = y for DPVO windows
// (ba_cuda.cu:560-562: S += I (1e-4 S + 1), L = chol(S), dX = chol_solve).
// The reference factors in fp32; the solve here is a blocked (6 x 6, one
// block per pose) right-looking fp32 Cholesky followed by one step of fp64
// iterative refinement (r = y - S x in fp64 from the fp64 S, x += S^-1 r with
// the fp32 factors).  Why fp32: on gfx950 a dependent v_fma_f64 costs ~36
// cycles against ~4 for v_fma_f32, and a 66 x 66 factorisation is a chain of
// N small dependent steps; the refinement brings the result back to fp64
// accuracy (||dX - dX_64|| / ||dX_64|| ~ 1e-9 on the cfg2 systems, whose
// condition numbers are ~2e5).
// Layout: lower 6x6 blocks, block (a, b) (a >= b) at lblk(a, b), row-major;
// diagonal blocks stored full.
// ---------------------------------------------------------------------------
struct Solver32 {
  const double* S;  // [NB][36] damped S (fp64)
  const double* y;  // [6N]
  double* x;        // [6N] solution (fp64)
  double* part;     // [4][6N] residual partial sums
  float* A;         // [NB][36] fp32 copy -> Cholesky factor blocks
  float* Li;        // [N][36] inverse of each diagonal factor block (lower)
  float* w;         // [6N] right-hand side -> forward -> solution (fp32)
  float* Nf;        // [NB][36] block (i, k), i > k: L_ik Li_k (forward, refinement only)
};

__host__ __device__ constexpr size_t solver32_bytes(int N) {
  return sizeof(double) * (36 * (size_t)(N * (N + 1) / 2) + 6 * (size_t)N * 6) +
         sizeof(float) * (2 * 36 * (size_t)(N * (N + 1) / 2) + 36 * (size_t)N + 6 * (size_t)N) + 64;
}

// one lane: Cholesky factor L of a 6x6 block (lower triangle of a,
// row-major), li = L^-1 (lower 21 entries written; the caller keeps the upper
// ones 0), wk <- li wk.  L itself is
// not stored: the panel, the substitutions and the refinement only use li.
// false if a pivot is not positive (ba_cuda.cu:547 leaves info unchecked;
// dpvo/ba.py:17-21 zeroes the step).  v_rsq_f32 (1 ulp) instead of a correctly
// rounded 1/sqrt: the refinement step absorbs it.
__device__ inline bool chol6_inv(const float* a, float* li, float* wk) {
  float m[6][6], L[6][6], R[6];
#pragma unroll
  for (int r = 0; r < 6; r++)
#pragma unroll
    for (int c = 0; c <= r; c++) m[r][c] = a[6 * r + c];
  bool ok = true;
#pragma unroll
  for (int c = 0; c < 6; c++) {
    const float d = m[c][c];
    ok = ok && (d > 0.0f);
    const float r = __builtin_amdgcn_rsqf(d);
    R[c] = r;
#pragma unroll
    for (int i = c + 1; i < 6; i++) L[i][c] = m[i][c] * r;
#pragma unroll
    for (int i = c + 1; i < 6; i++)
#pragma unroll
      for (int j = c + 1; j <= i; j++) m[i][j] -= L[i][c] * L[j][c];
  }
  float I[6][6];
#pragma unroll
  for (int i = 0; i < 6; i++) {
    I[i][i] = R[i];
#pragma unroll
    for (int j = 0; j < i; j++) {
      float s = L[i][j] * I[j][j];
#pragma unroll
      for (int k = j + 1; k < i; k++) s += L[i][k] * I[k][j];
      I[i][j] = -R[i] * s;
    }
  }
  float wv[6];
#pragma unroll
  for (int q = 0; q < 6; q++) wv[q] = wk[q];
#pragma unroll
  for (int q = 0; q < 6; q++) {
    float s = I[q][0] * wv[0];
#pragma unroll
    for (int p = 1; p <= q; p++) s += I[q][p] * wv[p];
    wk[q] = s;
  }
#pragma unroll
  for (int r = 0; r < 6; r++)
#pragma unroll
    for (int c = 0; c <= r; c++) li[6 * r + c] = I[r][c];
  return ok;
}

// whole wave (uniform control flow): the same factorisation with the six
// columns of L^-1 computed by lanes 0..5 in parallel (lane j solves
// L x = e_j; the Cholesky factor and wk are computed redundantly in every
// lane, so no cross-lane exchange).  Lanes 0..5 write column `lane` of li
// (zeros above the diagonal), lane 0 writes wk.  Returns the pivot check.
__device__ inline bool chol6_inv_wave(const float* a, float* li, float* wk, int lane) {
  float m[6][6], L[6][6], R[6];
#pragma unroll
  for (int r = 0; r < 6; r++)
#pragma unroll
    for (int c = 0; c <= r; c++) m[r][c] = a[6 * r + c];
  bool ok = true;
#pragma unroll
  for (int c = 0; c < 6; c++) {
    const float d = m[c][c];
    ok = ok && (d > 0.0f);
    const float r = __builtin_amdgcn_rsqf(d);
    R[c] = r;
#pragma unroll
    for (int i = c + 1; i < 6; i++) L[i][c] = m[i][c] * r;
#pragma unroll
    for (int i = c + 1; i < 6; i++)
#pragma unroll
      for (int j = c + 1; j <= i; j++) m[i][j] -= L[i][c] * L[j][c];
  }
  float x[6], v[6];
#pragma unroll
  for (int i = 0; i < 6; i++) {
    float e = (lane == i) ? 1.0f : 0.0f, t = wk[i];
#pragma unroll
    for (int k = 0; k < i; k++) {
      e -= L[i][k] * x[k];
      t -= L[i][k] * v[k];
    }
    x[i] = e * R[i];
    v[i] = t * R[i];
  }
  if (lane < 6) {
#pragma unroll
    for (int i = 0; i < 6; i++) li[6 * i + lane] = x[i];
  }
  if (lane == 0) {
#pragma unroll
    for (int i = 0; i < 6; i++) wk[i] = v[i];
  }
  return ok;
}

// lane-resident vector of wave 0: element t of w lives in lane t & 63, in
// register hi = t >> 6 (n <= 128)
__device__ __forceinline__ float wread(float w0, float w1, int t) {  // t wave-uniform
  const float v = (t < 64) ? w0 : w1;
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), t & 63));
}

// wave 0: w <- L^-1 w, register-resident: per block step k, the pivot rows
// take own = (Li_k w_k)[c] and rows i > k subtract (L_ik Li_k) w_k, with w_k
// broadcast by six readlanes -- the only dependency chain between steps
__device__ inline void chol32_forward(const Solver32& L, int N, int lane, float& w0, float& w1) {
  const int n = 6 * N;
  const int r0 = lane / 6, c0 = lane % 6, r1 = (lane + 64) / 6, c1 = (lane + 64) % 6;
  const bool v1 = lane + 64 < n;
  for (int k = 0; k < N; k++) {
    const float* li = L.Li + 36 * k;
    float wk[6];
#pragma unroll
    for (int p = 0; p < 6; p++) wk[p] = wread(w0, w1, 6 * k + p);
    {
      const int i = min(max(r0, k), N - 1);
      const float* b = L.Nf + 36 * lblk(i, k) + 6 * c0;
      const float* o = li + 6 * c0;
      float s = w0, own = 0.0f;
#pragma unroll
      for (int q = 0; q < 6; q++) {
        s -= b[q] * wk[q];
        own += o[q] * wk[q];  // upper entries of li are 0
      }
      w0 = (r0 > k && lane < n) ? s : ((r0 == k) ? own : w0);
    }
    if (n > 64) {
      const int i = min(max(r1, k), N - 1);
      const float* b = L.Nf + 36 * lblk(i, k) + 6 * c1;
      const float* o = li + 6 * c1;
      float s = w1, own = 0.0f;
#pragma unroll
      for (int q = 0; q < 6; q++) {
        s -= b[q] * wk[q];
        own += o[q] * wk[q];
      }
      w1 = (r1 > k && v1) ? s : ((r1 == k) ? own : w1);
    }
  }
}

// wave 0: w <- L^-T w, register-resident: v = Li_k^T w_k (uniform), pivot
// rows take v[c] (recomputed from per-lane loads: no indexed select), rows
// j < k subtract L_kj^T v
__device__ inline void chol32_backward(const Solver32& L, int N, int lane, float& w0, float& w1) {
  const int n = 6 * N;
  const int r0 = lane / 6, c0 = lane % 6, r1 = (lane + 64) / 6, c1 = (lane + 64) % 6;
  for (int k = N - 1; k >= 0; k--) {
    const float* li = L.Li + 36 * k;
    float wk[6], v[6];
#pragma unroll
    for (int p = 0; p < 6; p++) wk[p] = wread(w0, w1, 6 * k + p);
#pragma unroll
    for (int q = 0; q < 6; q++) {
      float s = li[6 * 5 + q] * wk[5];
#pragma unroll
      for (int p = 4; p >= q; p--) s += li[6 * p + q] * wk[p];
      v[q] = s;
    }
    {
      const float* b = L.A + 36 * lblk(k, min(r0, k)) + c0;
      float s = w0, own = 0.0f;
#pragma unroll
      for (int q = 0; q < 6; q++) {
        s -= b[6 * q] * v[q];
        own += li[6 * q + c0] * wk[q];  // upper entries of li are 0
      }
      w0 = (r0 < k) ? s : ((r0 == k) ? own : w0);
    }
    if (n > 64) {
      const float* b = L.A + 36 * lblk(k, min(r1, k)) + c1;
      float s = w1, own = 0.0f;
#pragma unroll
      for (int q = 0; q < 6; q++) {
        s -= b[6 * q] * v[q];
        own += li[6 * q + c1] * wk[q];
      }
      w1 = (r1 < k) ? s : ((r1 == k) ? own : w1);
    }
  }
}

__device__ __forceinline__ void dstamp(int64_t* st, int slot) {
  if (st && threadIdx.x == 0) st[slot] = (int64_t)__builtin_amdgcn_s_memtime();
}

// whole workgroup (>= 2 waves, blockDim a multiple of 64, 6N <= 128):
// dX = S^-1 y.  Returns with a workgroup barrier passed; *fail set on a failed
// pivot.  st (diagnostic builds only, may be null): shader-clock stamps by
// thread 0, [0] start, [1] converted, [2 + 2k] panel k done, [3 + 2k]
// trailing k done, [40] factored, [41] back-substituted, [42] residual,
// [43] refined, [44] end
__device__ inline void chol32_solve(const Solver32& L, int N, double* dX, int* fail, bool refine,
                                    int64_t* marks, int64_t* st = nullptr) {
  const int tid = threadIdx.x, T = blockDim.x, wid = tid >> 6, lane = tid & 63;
  const int NB = N * (N + 1) / 2, n = 6 * N;
  dstamp(st, 0);
  for (int k = tid; k < 36 * NB; k += T) L.A[k] = (float)L.S[k];
  for (int k = tid; k < n; k += T) L.w[k] = (float)L.y[k];
  for (int k = tid; k < 36 * N; k += T) L.Li[k] = 0.0f;  // chol6_inv writes the lower 21
  __syncthreads();
  if (wid == 0 && !chol6_inv_wave(L.A, L.Li, L.w, lane) && lane == 0) *fail = 1;
  __syncthreads();
  dstamp(st, 1);
  for (int k = 0; k + 1 < N; k++) {
    const int m = N - 1 - k;
    const float* li = L.Li + 36 * k;
    // panel: L_ik = S_ik L_kk^-T; forward step w_i -= L_ik w_k
    for (int t = tid; t < 6 * m; t += T) {
      const int i = k + 1 + t / 6, x = t % 6;
      float* a = L.A + 36 * lblk(i, k) + 6 * x;
      float av[6], lv[6];
#pragma unroll
      for (int q = 0; q < 6; q++) av[q] = a[q];
#pragma unroll
      for (int q = 0; q < 6; q++) {
        float s = av[0] * li[6 * q];
#pragma unroll
        for (int p = 1; p <= q; p++) s += av[p] * li[6 * q + p];
        lv[q] = s;
      }
      float wv = L.w[6 * i + x];
#pragma unroll
      for (int q = 0; q < 6; q++) {
        a[q] = lv[q];
        wv -= lv[q] * L.w[6 * k + q];
      }
      L.w[6 * i + x] = wv;
      if (refine) {  // Nf_ik = L_ik Li_k, row x
        float* no = L.Nf + 36 * lblk(i, k) + 6 * x;
#pragma unroll
        for (int p = 0; p < 6; p++) {
          float s = 0.0f;
#pragma unroll
          for (int q = p; q < 6; q++) s += lv[q] * li[6 * q + p];
          no[p] = s;
        }
      }
    }
    __syncthreads();
    dstamp(st, 2 + 2 * k);
    // trailing update S_ij -= L_ik L_jk^T; wave 0 takes the next pivot block
    // and factors it (look-ahead) while the other waves update the rest
    if (wid == 0) {
      if (lane < 36) {
        const int x = lane / 6, z = lane % 6, i = k + 1;
        if (z <= x) {
          const float* Lx = L.A + 36 * lblk(i, k) + 6 * x;
          const float* Lz = L.A + 36 * lblk(i, k) + 6 * z;
          float* d = L.A + 36 * lblk(i, i) + 6 * x + z;
          float s = *d;
#pragma unroll
          for (int q = 0; q < 6; q++) s -= Lx[q] * Lz[q];
          *d = s;
        }
      }
      wave_lds_sync();
      if (!chol6_inv_wave(L.A + 36 * lblk(k + 1, k + 1), L.Li + 36 * (k + 1), L.w + 6 * (k + 1),
                          lane) &&
          lane == 0)
        *fail = 1;
    } else {
      const int ntask = 6 * (m * (m + 1) / 2);
      for (int t = 6 + (tid - 64); t < ntask; t += T - 64) {
        const int x = t % 6;
        int a, b;
        tri_of(t / 6, a, b);
        const int i = k + 1 + a, j = k + 1 + b;
        const float* Li_ = L.A + 36 * lblk(i, k) + 6 * x;
        const float* Lj = L.A + 36 * lblk(j, k);
        float* Sij = L.A + 36 * lblk(i, j) + 6 * x;
        float v[6];
#pragma unroll
        for (int q = 0; q < 6; q++) v[q] = Li_[q];
        const int zmax = (i == j) ? x : 5;  // diagonal blocks: lower triangle only
#pragma unroll
        for (int z = 0; z < 6; z++) {
          if (z > zmax) break;
          float s = Sij[z];
#pragma unroll
          for (int q = 0; q < 6; q++) s -= v[q] * Lj[6 * z + q];
          Sij[z] = s;
        }
      }
    }
    __syncthreads();
    dstamp(st, 3 + 2 * k);
  }
  dstamp(st, 40);
  if (marks && tid == 0) marks[4] = (int64_t)wall_clock64();
  float w0 = 0.0f, w1 = 0.0f;
  if (wid == 0) {
    w0 = (lane < n) ? L.w[lane] : 0.0f;
    w1 = (lane + 64 < n) ? L.w[lane + 64] : 0.0f;
    chol32_backward(L, N, lane, w0, w1);
    if (lane < n) L.x[lane] = (double)w0;
    if (lane + 64 < n) L.x[lane + 64] = (double)w1;
  }
  __syncthreads();
  dstamp(st, 41);
  if (refine) {
    // r = y - S x in fp64: thread (row i, part) sums its block columns in order
    const int parts = min(T / n, 4);
    if (tid < parts * n) {
      const int i = tid % n, pt = tid / n, bi = i / 6, xi = i % 6;
      const int b0 = (N * pt) / parts, b1 = (N * (pt + 1)) / parts;
      double s[6] = {0.0, 0.0, 0.0, 0.0, 0.0, 0.0};
      for (int bj = b0; bj < b1; bj++) {
        const double* blk = (bi >= bj) ? L.S + 36 * lblk(bi, bj) + 6 * xi
                                       : L.S + 36 * lblk(bj, bi) + xi;
        const int stp = (bi >= bj) ? 1 : 6;
#pragma unroll
        for (int z = 0; z < 6; z++) s[z] += blk[stp * z] * L.x[6 * bj + z];
      }
      L.part[pt * n + i] = ((s[0] + s[1]) + (s[2] + s[3])) + (s[4] + s[5]);
    }
    __syncthreads();
    dstamp(st, 42);
    if (wid == 0) {
      float r[2];
#pragma unroll
      for (int h = 0; h < 2; h++) {
        const int i = lane + 64 * h;
        double sm = 0.0;
        if (i < n)
          for (int pt = 0; pt < parts; pt++) sm += L.part[pt * n + i];
        r[h] = (i < n) ? (float)(L.y[i] - sm) : 0.0f;
      }
      chol32_forward(L, N, lane, r[0], r[1]);
      chol32_backward(L, N, lane, r[0], r[1]);
      if (lane < n) L.x[lane] += (double)r[0];
      if (lane + 64 < n) L.x[lane + 64] += (double)r[1];
    }
    __syncthreads();
    dstamp(st, 43);
  }
  for (int k = tid; k < n; k += T) dX[k] = L.x[k];
  __syncthreads();
  dstamp(st, 44);
}

__device__ __forceinline__ void load6(const double* src, double* e) {
  const double2* q = reinterpret_cast<const double2*>(src);
#pragma unroll
  for (int k = 0; k < 3; k++) {
    const double2 v = q[k];
    e[2 * k] = v.x;
    e[2 * k + 1] = v.y;
  }
}

}  // namespace bad
}  // namespace dpvo
