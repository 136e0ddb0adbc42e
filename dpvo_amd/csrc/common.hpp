// common.hpp -- shared device/host helpers for the gfx950 DPVO hot path.
#pragma once

#include <hip/hip_fp16.h>
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "dpvo_hot.h"

#define DPVO_EXPORT extern "C" __attribute__((visibility("default")))

namespace dpvo {

constexpr int kWave = 64;  // CDNA wavefront width (never 32)
constexpr int kMaxDevices = 64;  // per-device one-time host state (function attributes)

inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }

inline int launch_status() {
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? DPVO_OK : DPVO_ERR_LAUNCH;
}

// --- element type helpers ---------------------------------------------------
template <typename T>
struct Acc { using type = float; };
template <>
struct Acc<double> { using type = double; };

__device__ __forceinline__ float to_acc(float v) { return v; }
__device__ __forceinline__ float to_acc(__half v) { return __half2float(v); }
__device__ __forceinline__ double to_acc(double v) { return v; }

template <typename T>
__device__ __forceinline__ T from_acc(float v);
template <>
__device__ __forceinline__ float from_acc<float>(float v) { return v; }
template <>
__device__ __forceinline__ __half from_acc<__half>(float v) { return __float2half(v); }
template <>
__device__ __forceinline__ double from_acc<double>(float v) { return (double)v; }
__device__ __forceinline__ double from_acc_d(double v) { return v; }

// static_cast<int>(floor(v)) with out-of-range values pushed far outside
// every map (the reference is undefined there; correlation_kernel.cu:156-157)
__device__ __forceinline__ int ifloor_safe(float v) {
  float f = floorf(v);
  f = fminf(fmaxf(f, -1.0e8f), 1.0e8f);  // NaN -> -1e8 (fmaxf drops NaN)
  return (int)f;
}

__device__ __forceinline__ int wave_uniform(int v) { return __builtin_amdgcn_readfirstlane(v); }

// Order LDS traffic between lanes of ONE wave (a wave's DS ops execute in
// order; this stops the compiler from moving them across the point).  The
// fence is restricted to the LDS address space ("local"): a plain fence also
// orders global memory and makes the compiler wait for every outstanding
// global load (vmcnt(0)) at the point, which drains the load rings of the
// streaming kernels (A-CORR's tile ring) at every use.
__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront", "local");
  __builtin_amdgcn_wave_barrier();
}

// wave64 inclusive scan of ints with DPP (row shifts 1/2/4/8 inside each row
// of 16 lanes, then row_bcast:15 / row_bcast:31 across rows): six VALU ops
// with a DPP source.  A __shfl_* is a ds_bpermute, an LDS round trip per
// step.  `id` is op's identity (what an out-of-row source contributes).
template <typename Op>
__device__ __forceinline__ int wave_scan_dpp(int x, int id, Op op) {
  x = op(x, __builtin_amdgcn_update_dpp(id, x, 0x111, 0xf, 0xf, false));  // row_shr:1
  x = op(x, __builtin_amdgcn_update_dpp(id, x, 0x112, 0xf, 0xf, false));  // row_shr:2
  x = op(x, __builtin_amdgcn_update_dpp(id, x, 0x114, 0xf, 0xf, false));  // row_shr:4
  x = op(x, __builtin_amdgcn_update_dpp(id, x, 0x118, 0xf, 0xf, false));  // row_shr:8
  x = op(x, __builtin_amdgcn_update_dpp(id, x, 0x142, 0xa, 0xf, false));  // row_bcast:15
  x = op(x, __builtin_amdgcn_update_dpp(id, x, 0x143, 0xc, 0xf, false));  // row_bcast:31
  return x;
}
__device__ __forceinline__ int wave_incl_sum(int x) {
  return wave_scan_dpp(x, 0, [](int a, int b) { return a + b; });
}
// wave-wide reductions (every lane gets the result)
__device__ __forceinline__ int wave_sum_i(int x) {
  return __builtin_amdgcn_readlane(wave_incl_sum(x), 63);
}
__device__ __forceinline__ int wave_min_i(int x) {
  return __builtin_amdgcn_readlane(
      wave_scan_dpp(x, 0x7fffffff, [](int a, int b) { return a < b ? a : b; }), 63);
}
__device__ __forceinline__ int wave_max_i(int x) {
  return __builtin_amdgcn_readlane(
      wave_scan_dpp(x, (int)0x80000000, [](int a, int b) { return a > b ? a : b; }), 63);
}

template <typename T>
__device__ __forceinline__ T wave_sum(T v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, kWave);
  return v;
}

// --- fp32 SE3 primitives of ba_cuda.cu:36-174 (restated, device) ---------------
// No FMA contraction here: the per-edge arithmetic then rounds exactly like the
// C oracle (x86, no FMA), which keeps the parity tests tight.
#pragma clang fp contract(off)
__device__ __forceinline__ void actSO3(const float* q, const float* X, float* Y) {
  float uv[3];
  uv[0] = 2.0f * (q[1] * X[2] - q[2] * X[1]);
  uv[1] = 2.0f * (q[2] * X[0] - q[0] * X[2]);
  uv[2] = 2.0f * (q[0] * X[1] - q[1] * X[0]);
  Y[0] = X[0] + q[3] * uv[0] + (q[1] * uv[2] - q[2] * uv[1]);
  Y[1] = X[1] + q[3] * uv[1] + (q[2] * uv[0] - q[0] * uv[2]);
  Y[2] = X[2] + q[3] * uv[2] + (q[0] * uv[1] - q[1] * uv[0]);
}

__device__ __forceinline__ void actSE3(const float* t, const float* q, const float* X, float* Y) {
  actSO3(q, X, Y);
  Y[3] = X[3];
  Y[0] += X[3] * t[0];
  Y[1] += X[3] * t[1];
  Y[2] += X[3] * t[2];
}

// Ji = Adj(Gij)^T Jj (ba_cuda.cu:57-72)
__device__ __forceinline__ void adjSE3(const float* t, const float* q, const float* X, float* Y) {
  float qinv[4] = {-q[0], -q[1], -q[2], q[3]};
  actSO3(qinv, &X[0], &Y[0]);
  actSO3(qinv, &X[3], &Y[3]);
  float u[3], v[3];
  u[0] = t[2] * X[1] - t[1] * X[2];
  u[1] = t[0] * X[2] - t[2] * X[0];
  u[2] = t[1] * X[0] - t[0] * X[1];
  actSO3(qinv, u, v);
  Y[3] += v[0];
  Y[4] += v[1];
  Y[5] += v[2];
}

// Gij = Pj * Pi^-1 (ba_cuda.cu:74-85)
__device__ __forceinline__ void relSE3(const float* ti, const float* qi, const float* tj,
                                       const float* qj, float* tij, float* qij) {
  qij[0] = -qj[3] * qi[0] + qj[0] * qi[3] - qj[1] * qi[2] + qj[2] * qi[1];
  qij[1] = -qj[3] * qi[1] + qj[1] * qi[3] - qj[2] * qi[0] + qj[0] * qi[2];
  qij[2] = -qj[3] * qi[2] + qj[2] * qi[3] - qj[0] * qi[1] + qj[1] * qi[0];
  qij[3] = qj[3] * qi[3] + qj[0] * qi[0] + qj[1] * qi[1] + qj[2] * qi[2];
  actSO3(qij, ti, tij);
  tij[0] = tj[0] - tij[0];
  tij[1] = tj[1] - tij[1];
  tij[2] = tj[2] - tij[2];
}

__device__ __forceinline__ void expSO3(const float* phi, float* q) {  // ba_cuda.cu:88-110
  float theta_sq = phi[0] * phi[0] + phi[1] * phi[1] + phi[2] * phi[2];
  float theta_p4 = theta_sq * theta_sq;
  float theta = sqrtf(theta_sq);
  float imag, real;
  if (theta_sq < 1e-8f) {
    imag = 0.5f - (1.0f / 48.0f) * theta_sq + (1.0f / 3840.0f) * theta_p4;
    real = 1.0f - (1.0f / 8.0f) * theta_sq + (1.0f / 384.0f) * theta_p4;
  } else {
    imag = sinf(0.5f * theta) / theta;
    real = cosf(0.5f * theta);
  }
  q[0] = imag * phi[0];
  q[1] = imag * phi[1];
  q[2] = imag * phi[2];
  q[3] = real;
}

__device__ __forceinline__ void crossInplace(const float* a, float* b) {
  float x0 = a[1] * b[2] - a[2] * b[1];
  float x1 = a[2] * b[0] - a[0] * b[2];
  float x2 = a[0] * b[1] - a[1] * b[0];
  b[0] = x0;
  b[1] = x1;
  b[2] = x2;
}

__device__ __forceinline__ void expSE3(const float* xi, float* t, float* q) {  // :125-153
  expSO3(xi + 3, q);
  float tau[3] = {xi[0], xi[1], xi[2]};
  float phi[3] = {xi[3], xi[4], xi[5]};
  float theta_sq = phi[0] * phi[0] + phi[1] * phi[1] + phi[2] * phi[2];
  float theta = sqrtf(theta_sq);
  t[0] = tau[0];
  t[1] = tau[1];
  t[2] = tau[2];
  if (theta > 1e-4f) {
    float a = (1.0f - cosf(theta)) / theta_sq;
    crossInplace(phi, tau);
    t[0] += a * tau[0];
    t[1] += a * tau[1];
    t[2] += a * tau[2];
    float b = (theta - sinf(theta)) / (theta * theta_sq);
    crossInplace(phi, tau);
    t[0] += b * tau[0];
    t[1] += b * tau[1];
    t[2] += b * tau[2];
  }
}

// pose <- Exp(xi) * pose, no renormalisation (ba_cuda.cu:156-174)
__device__ __forceinline__ void retrSE3(const float* xi, const float* t, const float* q, float* t1,
                                        float* q1) {
  float dt[3] = {0, 0, 0};
  float dq[4] = {0, 0, 0, 1};
  expSE3(xi, dt, dq);
  q1[0] = dq[3] * q[0] + dq[0] * q[3] + dq[1] * q[2] - dq[2] * q[1];
  q1[1] = dq[3] * q[1] + dq[1] * q[3] + dq[2] * q[0] - dq[0] * q[2];
  q1[2] = dq[3] * q[2] + dq[2] * q[3] + dq[0] * q[1] - dq[1] * q[0];
  q1[3] = dq[3] * q[3] - dq[0] * q[0] - dq[1] * q[1] - dq[2] * q[2];
  actSO3(dq, t, t1);
  t1[0] += dt[0];
  t1[1] += dt[1];
  t1[2] += dt[2];
}

// F-REPROJ of one (edge n, patch pixel pix) (ba_cuda.cu:379-429): shared by
// reproject_kernel (ba.hip) and the fused reproject + BA-plan launch
// (ba_window.hip), so both round identically.
// reprojected pixel (u, v) of patch pixel `pix` of edge n (ba_cuda.cu:379-429)
__device__ __forceinline__ void reproject_uv(const float* __restrict__ poses,
                                             const float* __restrict__ patches,
                                             const float* __restrict__ intrinsics,
                                             const int64_t* __restrict__ ii,
                                             const int64_t* __restrict__ jj,
                                             const int64_t* __restrict__ kk, int n, int pix, int P,
                                             int num_poses, int num_patches, float& u, float& v) {
  const int PP = P * P;
  const float fx = intrinsics[0], fy = intrinsics[1], cx = intrinsics[2], cy = intrinsics[3];
  const int ix = (int)min(max(ii[n], (int64_t)0), (int64_t)num_poses - 1);
  const int jx = (int)min(max(jj[n], (int64_t)0), (int64_t)num_poses - 1);
  const int64_t kx = min(max(kk[n], (int64_t)0), (int64_t)num_patches - 1);
  const float* pi = poses + 7 * (size_t)ix;
  const float* pj = poses + 7 * (size_t)jx;
  float ti[3] = {pi[0], pi[1], pi[2]}, qi[4] = {pi[3], pi[4], pi[5], pi[6]};
  float tj[3] = {pj[0], pj[1], pj[2]}, qj[4] = {pj[3], pj[4], pj[5], pj[6]};
  float tij[3], qij[4];
  relSE3(ti, qi, tj, qj, tij, qij);
  const float* pk = patches + (size_t)kx * 3 * PP;
  float Xi[4], Xj[4];
  Xi[0] = (pk[pix] - cx) / fx;
  Xi[1] = (pk[PP + pix] - cy) / fy;
  Xi[2] = 1.0f;
  Xi[3] = pk[2 * PP + pix];
  actSE3(tij, qij, Xi, Xj);
  u = fx * (Xj[0] / Xj[2]) + cx;
  v = fy * (Xj[1] / Xj[2]) + cy;
}

__device__ __forceinline__ void reproject_pixel(const float* __restrict__ poses,
                                                const float* __restrict__ patches,
                                                const float* __restrict__ intrinsics,
                                                const int64_t* __restrict__ ii,
                                                const int64_t* __restrict__ jj,
                                                const int64_t* __restrict__ kk, int n, int pix,
                                                int P, int num_poses, int num_patches,
                                                float* __restrict__ coords) {
  const int PP = P * P;
  float u, v;
  reproject_uv(poses, patches, intrinsics, ii, jj, kk, n, pix, P, num_poses, num_patches, u, v);
  coords[((size_t)n * 2 + 0) * PP + pix] = u;
  coords[((size_t)n * 2 + 1) * PP + pix] = v;
}

#pragma clang fp contract(fast)

// --- edge order for A-CORR (XCD-aware scheduling) -----------------------------
// One workgroup: order[p] = the edge at position p when edges are grouped by
// their target frame jj and, inside a frame, by the 16-pixel row band of the
// reprojected patch centre (counting sort; the order inside a (frame, band)
// bin is whatever the LDS atomics give -- A-CORR results do not depend on it,
// every edge is computed independently).  A-CORR gives each XCD an eighth of
// the positions: a frame's edges on one L2, and edges whose windows overlap
// near each other in the sequence, so the waves that share box lines run at
// the same time (cfg2 fp32: 41.3 -> 40.4 us, scripts/corr_order_probe.py).
// The centre is recomputed in both passes (no per-edge LDS: E is unbounded
// here).  bins: >= kOrderBins + 1 ints of LDS.  Frames outside
// [0, min(N2, kOrderBins / kOrderBands)) share the last frame's bins.
struct OrderIn {
  const float* poses;
  const float* patches;
  const float* intrinsics;
  const int64_t* ii;
  const int64_t* kk;
  int P, num_poses, num_patches;
};
constexpr int kOrderBins = 1024;
constexpr int kOrderBands = 16;  // row bands of 16 level-1 pixels (rows >= 240 share the last)
__device__ __forceinline__ int edge_order_key(const OrderIn& q, const int64_t* __restrict__ jj,
                                              int e, int nf) {
  const int64_t f = jj[e];
  float u, v;
  const int c = (q.P / 2) * q.P + q.P / 2;
  reproject_uv(q.poses, q.patches, q.intrinsics, q.ii, jj, q.kk, e, c, q.P, q.num_poses,
               q.num_patches, u, v);
  const int band = v >= 0.0f ? (int)fminf(v * (1.0f / 16.0f), (float)(kOrderBands - 1)) : 0;  // NaN: 0
  return ((f >= 0 && f < nf) ? (int)f : nf - 1) * kOrderBands + band;
}
__device__ inline void edge_order_block(const OrderIn& q, const int64_t* __restrict__ jj, int E,
                                        int N2, int* __restrict__ order, int* bins) {
  const int tid = threadIdx.x, T = blockDim.x;
  const int nf = min(max(N2, 1), kOrderBins / kOrderBands), nb = nf * kOrderBands;
  if (E <= 0) return;
  // keys of 4 edges (tid + 4 T k + r T) at a time, every load of the four
  // issued before the first use; the first group's keys stay in registers
  // for the scatter pass (E <= 4 T: no recomputation, cfg2)
  auto keys4 = [&](int e0, int (&k)[4]) __attribute__((always_inline)) {
#pragma unroll
    for (int r = 0; r < 4; r++) k[r] = edge_order_key(q, jj, min(e0 + r * T, E - 1), nf);
  };
  int k0[4];
  keys4(tid, k0);
  for (int b = tid; b <= nb; b += T) bins[b] = 0;
  __syncthreads();
  for (int e0 = tid; e0 < E; e0 += 4 * T) {
    int k[4];
    if (e0 == tid) {
#pragma unroll
      for (int r = 0; r < 4; r++) k[r] = k0[r];
    } else {
      keys4(e0, k);
    }
#pragma unroll
    for (int r = 0; r < 4; r++)
      if (e0 + r * T < E) atomicAdd(&bins[k[r]], 1);
  }
  __syncthreads();
  if (tid < 64) {  // exclusive scan of nb <= 1024 bins by one wave
    int carry = 0;
    for (int b0 = 0; b0 < nb; b0 += 64) {
      const int b = b0 + tid;
      const int c = (b < nb) ? bins[b] : 0;
      int x = c;
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        const int y = __shfl_up(x, o, 64);
        if (tid >= o) x += y;
      }
      if (b < nb) bins[b] = carry + x - c;
      carry += __shfl(x, 63, 64);
    }
  }
  __syncthreads();
  for (int e0 = tid; e0 < E; e0 += 4 * T) {
    int k[4];
    if (e0 == tid) {
#pragma unroll
      for (int r = 0; r < 4; r++) k[r] = k0[r];
    } else {
      keys4(e0, k);
    }
#pragma unroll
    for (int r = 0; r < 4; r++)
      if (e0 + r * T < E) order[atomicAdd(&bins[k[r]], 1)] = e0 + r * T;
  }
}

}  // namespace dpvo
