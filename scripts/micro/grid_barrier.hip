// Software grid barrier cost among workgroups of one XCD vs all XCDs, and a
// dependent load of data another XCD just wrote.  Cooperative launch
// guarantees co-residency.  hipcc --offload-arch=gfx950 -O3.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

__device__ __forceinline__ void sw_barrier(unsigned* ctr, unsigned target) {
  __syncthreads();
  if (threadIdx.x == 0) {
    __threadfence();
    atomicAdd(ctr, 1u);
    while (__hip_atomic_load(ctr, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) < target) {
      __builtin_amdgcn_s_sleep(1);
    }
  }
  __syncthreads();
}

// participants: blocks with (blockIdx % stride == 0)
__global__ void __launch_bounds__(256) k_bar(unsigned* ctr, int stride, int n, int64_t* out) {
  if (blockIdx.x % stride) return;
  const unsigned np = gridDim.x / stride;
  const int64_t t0 = wall_clock64();
  for (int i = 1; i <= n; i++) sw_barrier(ctr, np * i);
  const int64_t t1 = wall_clock64();
  if (blockIdx.x == 0 && threadIdx.x == 0) out[0] = t1 - t0;
}

// ping-pong: block 0 writes, block p reads after a flag; measures handoff latency
__global__ void __launch_bounds__(64) k_pingpong(volatile int* flag, int* data, int partner, int n,
                                                int64_t* out) {
  if (blockIdx.x != 0 && blockIdx.x != partner) return;
  if (threadIdx.x) return;
  const int64_t t0 = wall_clock64();
  for (int i = 0; i < n; i++) {
    if (blockIdx.x == 0) {
      while (__hip_atomic_load((int*)flag, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) != 2 * i) {}
      __hip_atomic_store((int*)flag, 2 * i + 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    } else {
      while (__hip_atomic_load((int*)flag, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) != 2 * i + 1) {}
      __hip_atomic_store((int*)flag, 2 * i + 2, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  const int64_t t1 = wall_clock64();
  if (blockIdx.x == 0) out[0] = t1 - t0;
}

int main() {
  unsigned* ctr; int64_t* out; int64_t h;
  hipMalloc(&ctr, 256); hipMalloc(&out, 64);
  int* flag; hipMalloc(&flag, 256);
  const int n = 200;
  for (int stride : {8, 1}) {
    for (int nb : {64, 256}) {
      hipMemset(ctr, 0, 4);
      void* args[] = {&ctr, &stride, (void*)&n, &out};
      int st = stride; int nn = n;
      void* a2[] = {&ctr, &st, &nn, &out};
      hipError_t e = hipLaunchCooperativeKernel((const void*)k_bar, dim3(nb), dim3(256), a2, 0, 0);
      hipDeviceSynchronize();
      hipMemcpy(&h, out, 8, hipMemcpyDeviceToHost);
      printf("grid barrier: %d blocks launched, %d participants (stride %d): %.0f ns/barrier (%s)\n",
             nb, nb / stride, stride, h * 10.0 / n, hipGetErrorString(e));
      (void)args;
    }
  }
  for (int partner : {8, 1, 3}) {
    hipMemset(flag, 0, 4);
    hipLaunchKernelGGL(k_pingpong, dim3(16), dim3(64), 0, 0, (volatile int*)flag, flag + 16, partner, n, out);
    hipDeviceSynchronize();
    hipMemcpy(&h, out, 8, hipMemcpyDeviceToHost);
    printf("flag ping-pong block0 <-> block%d (%s XCD): %.0f ns per one-way handoff\n", partner,
           partner % 8 == 0 ? "same" : "other", h * 10.0 / n / 2);
  }
  return 0;
}
