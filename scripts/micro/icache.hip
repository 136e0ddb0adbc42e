// Straight-line code vs looped code of the same instruction count, one
// workgroup of 16 waves: measures instruction-fetch cost of cold code.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

template <int U>
__device__ __forceinline__ float body(float a, float b) {
#pragma unroll
  for (int i = 0; i < U; i++) a = __builtin_fmaf(a, b, (float)(i & 7) * 1e-3f);
  return a;
}

__global__ void __launch_bounds__(1024) k_straight(float* io, int64_t* out) {
  float a = io[threadIdx.x], b = io[1024 + threadIdx.x];
  __syncthreads();
  const int64_t t0 = wall_clock64();
  a = body<4096>(a, b);
  __syncthreads();
  const int64_t t1 = wall_clock64();
  io[threadIdx.x] = a;
  if (threadIdx.x == 0) out[0] = t1 - t0;
}

__global__ void __launch_bounds__(1024) k_loop(float* io, int64_t* out) {
  float a = io[threadIdx.x], b = io[1024 + threadIdx.x];
  __syncthreads();
  const int64_t t0 = wall_clock64();
#pragma unroll 1
  for (int i = 0; i < 64; i++) a = body<64>(a, b);
  __syncthreads();
  const int64_t t1 = wall_clock64();
  io[threadIdx.x] = a;
  if (threadIdx.x == 0) out[0] = t1 - t0;
}

int main() {
  float* io; int64_t* out; int64_t h;
  hipMalloc(&io, 4 * 2048); hipMalloc(&out, 64); hipMemset(io, 0, 4 * 2048);
  for (int rep = 0; rep < 3; rep++) {
    hipLaunchKernelGGL(k_straight, 1, 1024, 0, 0, io, out);
    hipMemcpy(&h, out, 8, hipMemcpyDeviceToHost);
    if (rep == 2) printf("straight-line 4096 dependent fma (32 KiB code): %.2f us\n", h * 0.01);
    hipLaunchKernelGGL(k_loop, 1, 1024, 0, 0, io, out);
    hipMemcpy(&h, out, 8, hipMemcpyDeviceToHost);
    if (rep == 2) printf("looped 64 x 64 dependent fma: %.2f us\n", h * 0.01);
  }
  return 0;
}
