// Back-to-back dependent launch cost on one stream (plain and hipGraph), and
// fp64 / fp32 FMA throughput of one CU.  hipcc --offload-arch=gfx950 -O3.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#include <vector>
#include <algorithm>

__global__ void k_stamp(int64_t* t, int i) {
  if (threadIdx.x == 0 && blockIdx.x == 0) t[i] = wall_clock64();
}

template <typename T>
__global__ void __launch_bounds__(1024) k_fma(int n, T* io, int64_t* out) {
  T a0 = io[threadIdx.x], a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5,
    a6 = a0 + 6, a7 = a0 + 7;
  const T b = io[1024 + threadIdx.x];
  __syncthreads();
  int64_t c0 = clock64();
  for (int i = 0; i < n; i++) {
    a0 = a0 * b + (T)1e-3; a1 = a1 * b + (T)1e-3; a2 = a2 * b + (T)1e-3; a3 = a3 * b + (T)1e-3;
    a4 = a4 * b + (T)1e-3; a5 = a5 * b + (T)1e-3; a6 = a6 * b + (T)1e-3; a7 = a7 * b + (T)1e-3;
  }
  __syncthreads();
  int64_t c1 = clock64();
  io[threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7;
  if (threadIdx.x == 0) out[0] = c1 - c0;
}

int main() {
  int64_t* t; hipMalloc(&t, 8 * 4096);
  hipStream_t s; hipStreamCreate(&s);
  const int n = 200;
  for (int rep = 0; rep < 3; rep++) {
    for (int i = 0; i < n; i++) hipLaunchKernelGGL(k_stamp, 1, 64, 0, s, t, i);
    hipStreamSynchronize(s);
    std::vector<int64_t> h(n);
    hipMemcpy(h.data(), t, 8 * n, hipMemcpyDeviceToHost);
    std::vector<double> d;
    for (int i = 1; i < n; i++) d.push_back((h[i] - h[i - 1]) * 10.0);
    std::sort(d.begin(), d.end());
    if (rep == 2) printf("plain launches: start-to-start gap median %.0f ns, p10 %.0f ns\n", d[d.size() / 2], d[d.size() / 10]);
  }
  // graph of n stamps
  hipGraph_t g; hipGraphExec_t ge;
  hipStreamBeginCapture(s, hipStreamCaptureModeGlobal);
  for (int i = 0; i < n; i++) hipLaunchKernelGGL(k_stamp, 1, 64, 0, s, t, i);
  hipStreamEndCapture(s, &g);
  hipGraphInstantiate(&ge, g, nullptr, nullptr, 0);
  for (int rep = 0; rep < 3; rep++) {
    hipGraphLaunch(ge, s);
    hipStreamSynchronize(s);
    std::vector<int64_t> h(n);
    hipMemcpy(h.data(), t, 8 * n, hipMemcpyDeviceToHost);
    std::vector<double> d;
    for (int i = 1; i < n; i++) d.push_back((h[i] - h[i - 1]) * 10.0);
    std::sort(d.begin(), d.end());
    if (rep == 2) printf("graph launches: start-to-start gap median %.0f ns, p10 %.0f ns\n", d[d.size() / 2], d[d.size() / 10]);
  }
  double* iod; float* iof; int64_t* out; int64_t h;
  hipMalloc(&iod, 8 * 2048); hipMalloc(&iof, 4 * 2048); hipMalloc(&out, 64);
  hipMemset(iod, 0, 8 * 2048); hipMemset(iof, 0, 4 * 2048);
  for (int rep = 0; rep < 2; rep++) {
    hipLaunchKernelGGL(k_fma<double>, 1, 1024, 0, s, 1000, iod, out);
    hipMemcpy(&h, out, 8, hipMemcpyDeviceToHost);
    if (rep) printf("fp64 FMA, 1 CU 16 waves x 8 indep: %.2f cycles per wave-instr per SIMD\n", (double)h / (1000.0 * 8 * 4));
    hipLaunchKernelGGL(k_fma<float>, 1, 1024, 0, s, 1000, iof, out);
    hipMemcpy(&h, out, 8, hipMemcpyDeviceToHost);
    if (rep) printf("fp32 FMA, 1 CU 16 waves x 8 indep: %.2f cycles per wave-instr per SIMD\n", (double)h / (1000.0 * 8 * 4));
  }
  return 0;
}
