// Calibration of single-workgroup costs on gfx950 (barrier, LDS round trip,
// dependent global load, bitonic stage).  hipcc --offload-arch=gfx950 -O3.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

__global__ void __launch_bounds__(1024) k_barriers(int n, int64_t* out) {
  __shared__ int x[1024];
  int64_t t0 = wall_clock64();
  for (int i = 0; i < n; i++) {
    x[threadIdx.x] = i;
    __syncthreads();
  }
  int64_t t1 = wall_clock64();
  if (threadIdx.x == 0) { out[0] = t1 - t0; out[1] = x[5]; }
}

__global__ void __launch_bounds__(1024) k_lds_chain(int n, int64_t* out) {
  __shared__ int x[1024];
  x[threadIdx.x] = (threadIdx.x + 1) & 1023;
  __syncthreads();
  int p = threadIdx.x;
  int64_t t0 = wall_clock64();
  for (int i = 0; i < n; i++) p = x[p];
  int64_t t1 = wall_clock64();
  if (threadIdx.x == 0) { out[0] = t1 - t0; out[1] = p; }
}

__global__ void __launch_bounds__(64) k_lds_chain_1wave(int n, int64_t* out) {
  __shared__ int x[1024];
  for (int i = threadIdx.x; i < 1024; i += 64) x[i] = (i + 1) & 1023;
  __syncthreads();
  int p = threadIdx.x;
  int64_t t0 = wall_clock64();
  for (int i = 0; i < n; i++) p = x[p];
  int64_t t1 = wall_clock64();
  if (threadIdx.x == 0) { out[0] = t1 - t0; out[1] = p; }
}

__global__ void __launch_bounds__(1024) k_global_chain(const int* g, int n, int64_t* out) {
  int p = threadIdx.x;
  int64_t t0 = wall_clock64();
  for (int i = 0; i < n; i++) p = g[p];
  int64_t t1 = wall_clock64();
  if (threadIdx.x == 0) { out[0] = t1 - t0; out[1] = p; }
}

__global__ void __launch_bounds__(64) k_global_chain_1wave(const int* g, int n, int64_t* out) {
  int p = threadIdx.x;
  int64_t t0 = wall_clock64();
  for (int i = 0; i < n; i++) p = g[p];
  int64_t t1 = wall_clock64();
  if (threadIdx.x == 0) { out[0] = t1 - t0; out[1] = p; }
}

__global__ void __launch_bounds__(1024) k_bitonic(int P2, int64_t* out) {
  extern __shared__ unsigned long long keys[];
  for (int i = threadIdx.x; i < P2; i += blockDim.x) keys[i] = (unsigned long long)((i * 2654435761u) & 0xffff);
  __syncthreads();
  int64_t t0 = wall_clock64();
  for (int size = 2; size <= P2; size <<= 1)
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      for (int i = threadIdx.x; i < P2 / 2; i += blockDim.x) {
        const int lo = 2 * i - (i & (stride - 1)), hi = lo + stride;
        const bool up = ((lo & size) == 0);
        const unsigned long long a = keys[lo], b = keys[hi];
        if ((a > b) == up) { keys[lo] = b; keys[hi] = a; }
      }
      __syncthreads();
    }
  int64_t t1 = wall_clock64();
  if (threadIdx.x == 0) { out[0] = t1 - t0; out[1] = keys[7]; }
}

__global__ void __launch_bounds__(64) k_dbl_chain(int n, double* io, int64_t* out) {
  double a = io[threadIdx.x], b = io[64 + threadIdx.x];
  int64_t c0 = clock64();
  for (int i = 0; i < n; i++) a = fma(a, b, 1e-3);
  int64_t c1 = clock64();
  io[threadIdx.x] = a;
  if (threadIdx.x == 0) out[0] = c1 - c0;
}

__global__ void __launch_bounds__(64) k_shfl_chain(int n, double* io, int64_t* out) {
  double a = io[threadIdx.x];
  int64_t c0 = clock64();
  for (int i = 0; i < n; i++) a = __shfl(a, (threadIdx.x + 1) & 63, 64) + 1e-3;
  int64_t c1 = clock64();
  io[threadIdx.x] = a;
  if (threadIdx.x == 0) out[0] = c1 - c0;
}

int main() {
  int64_t* d_out; int64_t h[2];
  hipMalloc(&d_out, 64);
  int* g; hipMalloc(&g, 1 << 20);
  int hg[1024]; for (int i = 0; i < 1024; i++) hg[i] = (i * 97 + 13) & 1023;
  hipMemcpy(g, hg, sizeof(hg), hipMemcpyHostToDevice);
  double* io; hipMalloc(&io, 1024 * 8); hipMemset(io, 0, 1024 * 8);
  const int n = 1000;
  for (int rep = 0; rep < 3; rep++) {
    hipLaunchKernelGGL(k_barriers, 1, 1024, 0, 0, n, d_out);
    hipMemcpy(h, d_out, 16, hipMemcpyDeviceToHost);
    if (rep == 2) printf("barrier (1024 thr, + 1 ds_write): %.1f ns\n", h[0] * 10.0 / n);
    hipLaunchKernelGGL(k_lds_chain, 1, 1024, 0, 0, n, d_out);
    hipMemcpy(h, d_out, 16, hipMemcpyDeviceToHost);
    if (rep == 2) printf("dependent LDS load (16 waves): %.1f ns\n", h[0] * 10.0 / n);
    hipLaunchKernelGGL(k_lds_chain_1wave, 1, 64, 0, 0, n, d_out);
    hipMemcpy(h, d_out, 16, hipMemcpyDeviceToHost);
    if (rep == 2) printf("dependent LDS load (1 wave): %.1f ns\n", h[0] * 10.0 / n);
    hipLaunchKernelGGL(k_global_chain, 1, 1024, 0, 0, g, n, d_out);
    hipMemcpy(h, d_out, 16, hipMemcpyDeviceToHost);
    if (rep == 2) printf("dependent global load, L2-resident (16 waves): %.1f ns\n", h[0] * 10.0 / n);
    hipLaunchKernelGGL(k_global_chain_1wave, 1, 64, 0, 0, g, n, d_out);
    hipMemcpy(h, d_out, 16, hipMemcpyDeviceToHost);
    if (rep == 2) printf("dependent global load (1 wave): %.1f ns\n", h[0] * 10.0 / n);
    hipFuncSetAttribute((const void*)k_bitonic, hipFuncAttributeMaxDynamicSharedMemorySize, 65536);
    hipLaunchKernelGGL(k_bitonic, 1, 1024, 2048 * 8, 0, 2048, d_out);
    hipMemcpy(h, d_out, 16, hipMemcpyDeviceToHost);
    if (rep == 2) printf("bitonic 2048 (66 stages): %.2f us = %.1f ns/stage\n", h[0] * 0.01, h[0] * 10.0 / 66);
    hipLaunchKernelGGL(k_dbl_chain, 1, 64, 0, 0, n, io, d_out);
    hipMemcpy(h, d_out, 16, hipMemcpyDeviceToHost);
    if (rep == 2) printf("dependent f64 fma: %.1f cycles\n", (double)h[0] / n);
    hipLaunchKernelGGL(k_shfl_chain, 1, 64, 0, 0, n, io, d_out);
    hipMemcpy(h, d_out, 16, hipMemcpyDeviceToHost);
    if (rep == 2) printf("dependent f64 shfl + add: %.1f cycles\n", (double)h[0] / n);
  }
  return 0;
}
