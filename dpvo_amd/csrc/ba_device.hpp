// ba_device.hpp -- device code shared by the F-BA kernels (ba_fused.hip,
// ba_blocks.hip): the reference's fp32 edge linearisation, block scan, the
// 6x6 LDL^T pivot factorisation and small index helpers.
#pragma once

#include "common.hpp"

namespace dpvo {
namespace bad {

__device__ __forceinline__ int lblk(int a, int b) { return a * (a + 1) / 2 + b; }  // a >= b

// block-wide exclusive scan of LDS ints data[0..n), returns the total.  Each
// thread owns a contiguous run of at most kScanRun elements whose loads are
// all issued before the first add (one LDS latency, not one per element).
constexpr int kScanRun = 16;
__device__ inline int fscan(int* data, int n, int* scr) {
  const int tid = threadIdx.x, nt = blockDim.x;
  const int per = (n + nt - 1) / nt;
  int total = 0;
  for (int base = 0; base < n; base += nt * kScanRun) {  // chunks of nt * kScanRun
    const int cn = min(n - base, nt * kScanRun);
    const int cper = min(per, kScanRun);
    const int lo = base + min(tid * cper, cn), hi = base + min(tid * cper + cper, cn);
    int v[kScanRun];
#pragma unroll
    for (int k = 0; k < kScanRun; k++) v[k] = (lo + k < hi) ? data[lo + k] : 0;
    int s = 0;
#pragma unroll
    for (int k = 0; k < kScanRun; k++) s += v[k];
    const int lane = tid & 63, wid = tid >> 6;
    int x = s;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const int t = __shfl_up(x, o, 64);
      if (lane >= o) x += t;
    }
    if (lane == 63) scr[wid] = x;
    __syncthreads();
    if (tid == 0) {
      int acc = 0;
      for (int w = 0; w < nt / 64; w++) {
        const int y = scr[w];
        scr[w] = acc;
        acc += y;
      }
      scr[nt / 64] = acc;
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

__device__ __forceinline__ double rcp64(double d) {  // v_rcp_f64 (2^-24) + 2 Newton steps
  double r = __builtin_amdgcn_rcp(d);
  r = __builtin_fma(r, __builtin_fma(-d, r, 1.0), r);
  r = __builtin_fma(r, __builtin_fma(-d, r, 1.0), r);
  return r;
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

__device__ __forceinline__ void tri_of(int bt, int& a, int& b) {  // bt -> (a, b), a >= b
  int r = (int)((sqrtf(8.0f * bt + 1.0f) - 1.0f) * 0.5f);
  while (r * (r + 1) / 2 > bt) r--;
  while ((r + 1) * (r + 2) / 2 <= bt) r++;
  a = r;
  b = bt - r * (r + 1) / 2;
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
