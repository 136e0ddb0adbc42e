// spd_solve.hip -- batched dense SPD factor + solve on gfx950 for the training
// surface's CholeskySolver (dpvo/ba.py:13-38: torch.linalg.cholesky_ex +
// cholesky_solve; block_solve 67-77 feeds it the damped pose system).
//
// One 256-thread workgroup per batch item.  The matrix and the right-hand
// sides live in LDS when n (n + k) elements fit 160 KB - 64 B (one rhs: fp64
// n <= 142, fp32 n <= 201; every DPVO training / python_ba system), else in
// the caller's factor buffer in HBM (same code, global addresses); the work
// is latency-bound either way (n column steps).
//   factor: right-looking Cholesky on the lower triangle (torch reads only
//           the lower triangle of H, cholesky_ex default upper=False):
//           column j: pivot d = a_jj (d <= 0 or NaN: info = j + 1, the
//           first failed column, as LAPACK potrf), l_jj = sqrt(d),
//           l_ij = a_ij / l_jj into a contiguous LDS column, then
//           a_ic -= l_ij l_cj (j < c <= i) by 8 row groups x 32 column lanes;
//   solve:  L Y = B (forward), L^T X = Y (backward), k right-hand sides;
//           with one rhs and the factor in LDS, the factor also mirrors L^T
//           into the upper triangle and wave 0 runs both sweeps alone as
//           contiguous row axpys (no workgroup barrier per step).
// Outputs: L (lower, zeros above, like cholesky_ex), X, info.  A failed
// factorisation leaves X = 0 (the caller's "don't crash training" branch
// returns zeros anyway).  Deterministic: every sum in a fixed order.
#include "common.hpp"

namespace dpvo {
namespace {

constexpr int kSpdThreads = 256;
constexpr size_t kSpdLds = 160 * 1024;

template <typename T>
__device__ __forceinline__ T spd_sqrt(T v);
template <>
__device__ __forceinline__ float spd_sqrt<float>(float v) { return sqrtf(v); }
template <>
__device__ __forceinline__ double spd_sqrt<double>(double v) { return sqrt(v); }

// M: the n x n working matrix (row-major, LDS or HBM), lv: n scratch entries
// of LDS (the current column), Y: n x k right-hand sides.  Per column: the
// scaled column goes to lv (contiguous, read as broadcasts and unit-stride
// runs), then the trailing triangle a_ic -= l_i l_c with 8 row groups x 32
// column lanes (consecutive c in consecutive lanes); two barriers a column.
template <typename T>
__device__ void spd_factor(T* M, T* lv, int n, int* fail_col, bool mirror) {
  const int tid = threadIdx.x, tr = tid >> 5, tc = tid & 31;
  for (int j = 0; j < n; j++) {
    const T d = M[(size_t)j * n + j];
    if (!(d > T(0))) {  // not positive definite (NaN included): block-uniform
      if (tid == 0) *fail_col = j + 1;
      __syncthreads();
      return;
    }
    const T s = spd_sqrt(d), rs = T(1) / s;
    for (int i = j + 1 + tid; i < n; i += kSpdThreads) {
      const T l = M[(size_t)i * n + j] * rs;
      M[(size_t)i * n + j] = l;
      lv[i] = l;
      if (mirror) M[(size_t)j * n + i] = l;  // L^T in the upper triangle (row j)
    }
    if (tid == 0) M[(size_t)j * n + j] = s;
    __syncthreads();
    for (int i = j + 1 + tr; i < n; i += kSpdThreads / 32) {
      const T li = lv[i];
      T* row = M + (size_t)i * n;
      for (int c = j + 1 + tc; c <= i; c += 32) row[c] -= li * lv[c];
    }
    __syncthreads();
  }
}

// One right-hand side, L in the lower AND L^T in the upper triangle of M
// (spd_factor with mirror): both sweeps as column axpys on wave 0 alone, each
// step reading one contiguous row of M (forward: row j of the upper part =
// column j of L; backward: row j of L), no workgroup barrier inside a sweep
// (a wave's LDS accesses complete in order; wave_lds_sync orders the steps).
template <typename T>
__device__ void spd_solve1_wave(const T* M, T* y, int n) {
  const int lane = threadIdx.x;
  for (int j = 0; j < n; j++) {  // L y = b
    const T yj = y[j] / M[(size_t)j * n + j];
    const T* row = M + (size_t)j * n;
    for (int i = j + 1 + lane; i < n; i += kWave) y[i] -= row[i] * yj;
    if (lane == 0) y[j] = yj;
    wave_lds_sync();
  }
  for (int j = n - 1; j >= 0; j--) {  // L^T x = y
    const T xj = y[j] / M[(size_t)j * n + j];
    const T* row = M + (size_t)j * n;
    for (int i = lane; i < j; i += kWave) y[i] -= row[i] * xj;
    if (lane == 0) y[j] = xj;
    wave_lds_sync();
  }
}

// L Y = B then L^T X = Y in place (Y: n x k), L lower in M
template <typename T>
__device__ void spd_solve(const T* M, T* Y, int n, int k) {
  const int tid = threadIdx.x;
  for (int j = 0; j < n; j++) {  // forward
    const T rl = T(1) / M[(size_t)j * n + j];
    for (int c = tid; c < k; c += kSpdThreads) Y[(size_t)j * k + c] *= rl;
    __syncthreads();
    for (int e = tid; e < (n - j - 1) * k; e += kSpdThreads) {
      const int i = j + 1 + e / k, c = e % k;
      Y[(size_t)i * k + c] -= M[(size_t)i * n + j] * Y[(size_t)j * k + c];
    }
    __syncthreads();
  }
  for (int j = n - 1; j >= 0; j--) {  // backward (L^T)
    const T rl = T(1) / M[(size_t)j * n + j];
    for (int c = tid; c < k; c += kSpdThreads) Y[(size_t)j * k + c] *= rl;
    __syncthreads();
    for (int e = tid; e < j * k; e += kSpdThreads) {
      const int i = e / k, c = e % k;
      Y[(size_t)i * k + c] -= M[(size_t)j * n + i] * Y[(size_t)j * k + c];
    }
    __syncthreads();
  }
}

// factor != 0: H (lower triangle read) -> L, X = H^-1 B, info.
// factor == 0: H is already the lower factor L (read-only): X = (L L^T)^-1 B.
template <typename T>
__global__ void __launch_bounds__(kSpdThreads)
    spd_kernel(const T* __restrict__ H, const T* __restrict__ B, T* __restrict__ L,
               T* __restrict__ X, int* __restrict__ info, int n, int k, int factor, int in_lds) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  __shared__ int fail_col;
  T* lv = reinterpret_cast<T*>(smem) + (in_lds ? (size_t)n * n + (size_t)n * k : 0);  // [n]
  const int tid = threadIdx.x;
  const size_t b = blockIdx.x, nn = (size_t)n * n, nk = (size_t)n * k;
  const T* Hb = H + b * nn;
  T* Lb = L ? L + b * nn : nullptr;
  T* Xb = X + b * nk;
  // working matrix: LDS, or the factor buffer in HBM; a solve-only call
  // that does not fit LDS reads the given factor where it lies
  T* M = in_lds ? reinterpret_cast<T*>(smem) : (factor ? Lb : const_cast<T*>(Hb));
  T* Y = in_lds ? reinterpret_cast<T*>(smem) + nn : Xb;
  if (tid == 0) fail_col = 0;
  // stage: lower triangle of H (upper zero), B
  if (in_lds || factor)
    for (size_t e = tid; e < nn; e += kSpdThreads) {
      const int i = (int)(e / n), c = (int)(e % n);
      M[e] = (c <= i || !factor) ? Hb[e] : T(0);
    }
  for (size_t e = tid; e < nk; e += kSpdThreads) Y[e] = B[b * nk + e];
  __syncthreads();
  // one rhs with the factor in LDS: single-wave sweeps over a mirrored factor
  const bool wave_solve = factor && in_lds && k == 1;
  if (factor) spd_factor(M, lv, n, &fail_col, wave_solve);
  const bool ok = fail_col == 0;
  if (ok) {
    if (wave_solve) {
      if (tid < kWave) spd_solve1_wave(M, Y, n);
    } else {
      spd_solve(M, Y, n, k);
    }
  }
  __syncthreads();
  if (factor && in_lds && Lb)  // (in HBM the factor is already in place, zeros above)
    for (size_t e = tid; e < nn; e += kSpdThreads) {
      const int i = (int)(e / n), c = (int)(e % n);
      Lb[e] = c <= i ? M[e] : T(0);  // the mirrored upper triangle is not part of L
    }
  for (size_t e = tid; e < nk; e += kSpdThreads) Xb[e] = ok ? Y[e] : T(0);
  if (tid == 0 && info) info[b] = fail_col;
}

template <typename T>
int spd_launch(const void* H, const void* B, void* L, void* X, int32_t* info, int batch, int n,
               int k, int factor, void* stream) {
  // LDS: matrix + right-hand sides (when they fit) + the column scratch lv[n]
  const size_t full = sizeof(T) * ((size_t)n * n + (size_t)n * k + (size_t)n);
  const int in_lds = full <= kSpdLds - 64;
  const size_t lds = in_lds ? full : sizeof(T) * (size_t)n;
  if (!in_lds && factor && !L) return DPVO_ERR_INVALID;  // the HBM working copy is the factor buffer
  if (!in_lds && lds > 64 * 1024) return DPVO_ERR_UNSUPPORTED;  // lv alone past 64 KB: n > 8192
  if (in_lds && lds > 64 * 1024) {
    // the dynamic LDS beyond the default 64 KB (the static fail flag sits on
    // top), set once per device and instantiation
    static bool attr_set[kMaxDevices] = {};
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= kMaxDevices) return DPVO_ERR_LAUNCH;
    if (!attr_set[dev]) {
      if (hipFuncSetAttribute((const void*)spd_kernel<T>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              (int)(kSpdLds - 64)) != hipSuccess) {
        (void)hipGetLastError();  // not sticky: the launch reports its own status
        return DPVO_ERR_LAUNCH;
      }
      attr_set[dev] = true;
    }
  }
  hipLaunchKernelGGL(spd_kernel<T>, dim3(batch), dim3(kSpdThreads), lds,
                     as_stream(stream), (const T*)H, (const T*)B, (T*)L, (T*)X, (int*)info, n, k,
                     factor, in_lds);
  return launch_status();
}

}  // namespace
}  // namespace dpvo

using namespace dpvo;

DPVO_EXPORT int dpvo_spd_solve(const void* H, const void* B, void* L, void* X, int32_t* info,
                               int batch, int n, int k, int factor, int dtype, void* stream) {
  if (batch < 0 || n < 0 || k < 0) return DPVO_ERR_INVALID;
  if (batch == 0 || n == 0) return DPVO_OK;
  if (!H || !X || (k > 0 && !B)) return DPVO_ERR_INVALID;
  if (!factor && L) return DPVO_ERR_INVALID;  // solve-only reads H as the factor; L unused
  if (dtype == DPVO_F64) return spd_launch<double>(H, B, L, X, info, batch, n, k, factor, stream);
  if (dtype == DPVO_F32) return spd_launch<float>(H, B, L, X, info, batch, n, k, factor, stream);
  return DPVO_ERR_UNSUPPORTED;
}
