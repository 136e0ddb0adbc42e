// Cost of the reference's fp32 edge linearisation (ba_device.hpp lin_edge) on
// one CU: cycles per linearisation per thread with poses / patches / targets
// in LDS, for 1 and 2 waves per SIMD.  hipcc --offload-arch=gfx950 -O3
// -I include -I dpvo_amd/csrc scripts/micro/lin_cost.hip
#include <stdio.h>

#include "ba_device.hpp"

using namespace dpvo::bad;

template <int NT>
__global__ void __launch_bounds__(NT) k_lin(int n, float* out, long long* cyc) {
  __shared__ float pose[16 * 8];
  __shared__ float4 tw[NT];
  const int t = threadIdx.x;
  if (t < 16 * 8) pose[t] = (t % 8 == 6) ? 1.0f : 0.01f * (t % 8) + 0.05f * (t / 8);
  tw[t] = make_float4(40.f + t % 7, 30.f + t % 5, 0.5f, 0.7f);
  __syncthreads();
  float acc = 0.f;
  const long long t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < n; i++) {
    const int a = (t + i) & 15, b = (t + 3 * i + 1) & 15;
    const float4 w = tw[(t + i) % NT];
    Lin o;
    lin_edge(pose + 8 * a, pose + 8 * b, 0.1f + 1e-3f * i, -0.2f, 0.5f, w.x, w.y, w.z, w.w, 80.f,
             80.f, 80.f, 60.f, o);
    acc += o.Ji[0][3] + o.Jj[1][4] + o.w[0] + o.r[1] + o.Jz[0];
  }
  __syncthreads();
  const long long t1 = __builtin_amdgcn_s_memtime();
  out[t] = acc;
  if (t == 0) cyc[0] = t1 - t0;
}

int main() {
  float* out;
  long long* cyc;
  (void)hipMalloc(&out, 1024 * sizeof(float));
  (void)hipMalloc(&cyc, sizeof(long long));
  long long c;
  const int n = 64;
  for (int rep = 0; rep < 2; rep++) {
    hipLaunchKernelGGL(k_lin<256>, dim3(1), dim3(256), 0, 0, n, out, cyc);
    (void)hipDeviceSynchronize();
    (void)hipMemcpy(&c, cyc, sizeof(c), hipMemcpyDeviceToHost);
    if (rep) printf("lin_edge, 256 threads (1 wave/SIMD): %.0f cycles per lin per thread\n", (double)c / n);
    hipLaunchKernelGGL(k_lin<512>, dim3(1), dim3(512), 0, 0, n, out, cyc);
    (void)hipDeviceSynchronize();
    (void)hipMemcpy(&c, cyc, sizeof(c), hipMemcpyDeviceToHost);
    if (rep) printf("lin_edge, 512 threads (2 waves/SIMD): %.0f cycles per lin per thread\n", (double)c / n);
    hipLaunchKernelGGL(k_lin<1024>, dim3(1), dim3(1024), 0, 0, n, out, cyc);
    (void)hipDeviceSynchronize();
    (void)hipMemcpy(&c, cyc, sizeof(c), hipMemcpyDeviceToHost);
    if (rep) printf("lin_edge, 1024 threads (4 waves/SIMD): %.0f cycles per lin per thread\n", (double)c / n);
  }
  return 0;
}
