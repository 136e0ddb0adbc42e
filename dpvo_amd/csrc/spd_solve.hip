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
//           l_ij = a_ij / l_jj, then a_ic -= l_ij l_cj (j < c <= i);
//   solve:  L Y = B (forward), L^T X = Y (backward), k right-hand sides.
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

// M: the n x n working matrix (row-major, LDS or HBM), Y: n x k right-hand sides
template <typename T>
__device__ void spd_factor(T* M, int n, int* fail_col) {
  const int tid = threadIdx.x;
  for (int j = 0; j < n; j++) {
    const T d = M[(size_t)j * n + j];
    if (!(d > T(0))) {  // not positive definite (NaN included): block-uniform
      if (tid == 0) *fail_col = j + 1;
      __syncthreads();
      return;
    }
    const T s = spd_sqrt(d), rs = T(1) / s;
    // column j below the pivot (each thread its own rows: no barrier needed
    // between the scale and the diagonal store)
    for (int i = j + 1 + tid; i < n; i += kSpdThreads) M[(size_t)i * n + j] *= rs;
    if (tid == 0) M[(size_t)j * n + j] = s;
    __syncthreads();
    // trailing lower triangle: pairs (i, c), j < c <= i < n
    const int m = n - j - 1;
    const int pairs = m * (m + 1) / 2;
    for (int p = tid; p < pairs; p += kSpdThreads) {
      int r = (int)((sqrtf(8.0f * p + 1.0f) - 1.0f) * 0.5f);
      while (r * (r + 1) / 2 > p) r--;
      while ((r + 1) * (r + 2) / 2 <= p) r++;
      const int i = j + 1 + r, c = j + 1 + (p - r * (r + 1) / 2);
      M[(size_t)i * n + c] -= M[(size_t)i * n + j] * M[(size_t)c * n + j];
    }
    __syncthreads();
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
  if (factor) spd_factor(M, n, &fail_col);
  const bool ok = fail_col == 0;
  if (ok) spd_solve(M, Y, n, k);
  __syncthreads();
  if (factor && in_lds && Lb)  // (in HBM the factor is already in place, zeros above)
    for (size_t e = tid; e < nn; e += kSpdThreads) Lb[e] = M[e];
  for (size_t e = tid; e < nk; e += kSpdThreads) Xb[e] = ok ? Y[e] : T(0);
  if (tid == 0 && info) info[b] = fail_col;
}

template <typename T>
int spd_launch(const void* H, const void* B, void* L, void* X, int32_t* info, int batch, int n,
               int k, int factor, void* stream) {
  const size_t lds = sizeof(T) * ((size_t)n * n + (size_t)n * k);
  const int in_lds = lds <= kSpdLds - 64;
  if (!in_lds && factor && !L) return DPVO_ERR_INVALID;  // the HBM working copy is the factor buffer
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
  hipLaunchKernelGGL(spd_kernel<T>, dim3(batch), dim3(kSpdThreads), in_lds ? lds : 0,
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
