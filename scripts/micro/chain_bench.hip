// Isolated timing of the ba_ldl.hpp triangular chains (one wave, LDS
// pre-filled with finite data): cycles per chain and per 6-step block.
#include <hip/hip_runtime.h>
#include <stdio.h>

#include "ba_ldl_experiment.hpp"
using namespace dpvo::bad;

template <bool TWO, int WHICH>
__global__ void __launch_bounds__(256) tchain(float* out, long long* cyc, int N) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  __shared__ int f;
  LSolve v = ldl_view((const double*)lds, (const double*)lds, lds, N, &f);
  const int n = 6 * N, ls = ldl_stride(n);
  for (int t = threadIdx.x; t < (n + 1 + kLdlPad) * ls; t += blockDim.x) v.A[t] = 0.001f * (t % 97);
  for (int t = threadIdx.x; t < n + 64; t += blockDim.x) v.rd[t] = 1.0f;
  for (int t = threadIdx.x; t < 36 * N; t += blockDim.x) v.db[t] = 0.001f * (t % 13);
  __syncthreads();
  if (threadIdx.x < 64) {
    const int lane = threadIdx.x;
    float w0 = out[lane], w1 = out[lane + 64];
    const long long t0 = __builtin_amdgcn_s_memtime();
    if (WHICH == 0)
      ldl_back<TWO>(v, N, ls, w0, w1, lane);
    else
      ldl_fwd<TWO>(v, N, ls, w0, w1, lane);
    __builtin_amdgcn_s_waitcnt(0);
    const long long t1 = __builtin_amdgcn_s_memtime();
    out[lane] = w0 + w1;
    if (lane == 0) *cyc = t1 - t0;
  }
}

template <bool TWO, int WHICH>
void run(const char* name, int N, float* o, long long* c) {
  hipFuncSetAttribute((const void*)(tchain<TWO, WHICH>), hipFuncAttributeMaxDynamicSharedMemorySize,
                      120 * 1024);
  long long best = 1LL << 60;
  for (int r = 0; r < 20; r++) {
    hipLaunchKernelGGL((tchain<TWO, WHICH>), dim3(1), dim3(256), 120 * 1024, 0, o, c, N);
    long long h;
    hipMemcpy(&h, c, 8, hipMemcpyDeviceToHost);
    best = h < best ? h : best;
  }
  printf("%-10s N=%2d %6lld cyc  %.0f per block\n", name, N, best, best / (double)N);
}

int main() {
  float* o;
  long long* c;
  hipMalloc(&o, 4096);
  hipMemset(o, 0, 4096);
  hipMalloc(&c, 8);
  run<false, 0>("back", 10, o, c);
  run<false, 1>("fwd", 10, o, c);
  run<true, 0>("back2", 11, o, c);
  run<true, 1>("fwd2", 11, o, c);
  run<true, 0>("back2", 16, o, c);
  return 0;
}
