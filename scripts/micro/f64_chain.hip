// Calibration of the fp64 costs that bound the BA solve on gfx950: dependent
// v_fma_f64 latency, v_rcp_f64 / v_rsq_f64 latency and accuracy (vs the IEEE
// 1/x and 1/sqrt(x) sequences), independent fp64 FMA issue rate, readlane and
// ds_bpermute round trips.  hipcc --offload-arch=gfx950 -O3.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>
#include <stdio.h>

__global__ void __launch_bounds__(64) k_fma_chain(int n, double a, double b, double* out,
                                                  int64_t* cyc) {
  double x = threadIdx.x * 1e-3;
  __syncthreads();
  const int64_t t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < n; i += 16)
#pragma unroll
    for (int k = 0; k < 16; k++) x = __builtin_fma(x, a, b);
  const int64_t t1 = __builtin_amdgcn_s_memtime();
  out[threadIdx.x] = x;
  if (threadIdx.x == 0) cyc[0] = t1 - t0;
}

__global__ void __launch_bounds__(64) k_fma32_chain(int n, float a, float b, double* out,
                                                    int64_t* cyc) {
  float x = threadIdx.x * 1e-3f;
  __syncthreads();
  const int64_t t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < n; i += 16)
#pragma unroll
    for (int k = 0; k < 16; k++) x = __builtin_fmaf(x, a, b);
  const int64_t t1 = __builtin_amdgcn_s_memtime();
  out[threadIdx.x] = x;
  if (threadIdx.x == 0) cyc[0] = t1 - t0;
}

__global__ void __launch_bounds__(64) k_rcp_chain(int n, double c, double* out, int64_t* cyc) {
  double x = 1.5 + threadIdx.x * 1e-3;
  __syncthreads();
  const int64_t t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < n; i += 16)
#pragma unroll
    for (int k = 0; k < 16; k++) x = __builtin_amdgcn_rcp(x) + c;
  const int64_t t1 = __builtin_amdgcn_s_memtime();
  out[threadIdx.x] = x;
  if (threadIdx.x == 0) cyc[0] = t1 - t0;
}

__global__ void __launch_bounds__(64) k_rsq_chain(int n, double c, double* out, int64_t* cyc) {
  double x = 1.5 + threadIdx.x * 1e-3;
  __syncthreads();
  const int64_t t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < n; i += 16)
#pragma unroll
    for (int k = 0; k < 16; k++) x = __builtin_amdgcn_rsq(x) + c;
  const int64_t t1 = __builtin_amdgcn_s_memtime();
  out[threadIdx.x] = x;
  if (threadIdx.x == 0) cyc[0] = t1 - t0;
}

__global__ void __launch_bounds__(64) k_div_chain(int n, double c, double* out, int64_t* cyc) {
  double x = 1.5 + threadIdx.x * 1e-3;
  __syncthreads();
  const int64_t t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < n; i += 16)
#pragma unroll
    for (int k = 0; k < 16; k++) x = 1.0 / x + c;
  const int64_t t1 = __builtin_amdgcn_s_memtime();
  out[threadIdx.x] = x;
  if (threadIdx.x == 0) cyc[0] = t1 - t0;
}

__global__ void __launch_bounds__(64) k_readlane_chain(int n, double* out, int64_t* cyc) {
  double x = threadIdx.x * 1e-3;
  __syncthreads();
  const int64_t t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < n; i++) {
    const int lo = __builtin_amdgcn_readlane(__double2loint(x), i & 63);
    const int hi = __builtin_amdgcn_readlane(__double2hiint(x), i & 63);
    x = __builtin_fma(__hiloint2double(hi, lo), 0.5, x);
  }
  const int64_t t1 = __builtin_amdgcn_s_memtime();
  out[threadIdx.x] = x;
  if (threadIdx.x == 0) cyc[0] = t1 - t0;
}

// 8 independent chains per lane, 16 waves: fp64 FMA throughput per SIMD
__global__ void __launch_bounds__(1024) k_fma_tput(int n, double a, double b, double* out,
                                                   int64_t* cyc) {
  double x[8];
  for (int k = 0; k < 8; k++) x[k] = threadIdx.x * 1e-3 + k;
  __syncthreads();
  const int64_t t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < n; i++)
#pragma unroll
    for (int k = 0; k < 8; k++) x[k] = __builtin_fma(x[k], a, b);
  __syncthreads();
  const int64_t t1 = __builtin_amdgcn_s_memtime();
  double s = 0;
  for (int k = 0; k < 8; k++) s += x[k];
  out[threadIdx.x] = s;
  if (threadIdx.x == 0) cyc[0] = t1 - t0;
}

__global__ void k_accuracy(int n, uint64_t seed, double* err) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  double e_rcp = 0, e_rsq = 0, e_sqrt = 0;
  uint64_t s = seed ^ (0x9E3779B97F4A7C15ull * (t + 1));
  for (int i = 0; i < n; i++) {
    s = s * 6364136223846793005ull + 1442695040888963407ull;
    const double u = (double)(s >> 11) * (1.0 / 9007199254740992.0);
    const double x = exp2(-20.0 + 60.0 * u);
    const double r_ref = 1.0 / x, q_ref = 1.0 / sqrt(x), s_ref = sqrt(x);
    e_rcp = fmax(e_rcp, fabs(__builtin_amdgcn_rcp(x) - r_ref) / r_ref);
    e_rsq = fmax(e_rsq, fabs(__builtin_amdgcn_rsq(x) - q_ref) / q_ref);
    e_sqrt = fmax(e_sqrt, fabs(__builtin_amdgcn_sqrt(x) - s_ref) / s_ref);
  }
  atomicMax((unsigned long long*)&err[0], (unsigned long long)__double_as_longlong(e_rcp));
  atomicMax((unsigned long long*)&err[1], (unsigned long long)__double_as_longlong(e_rsq));
  atomicMax((unsigned long long*)&err[2], (unsigned long long)__double_as_longlong(e_sqrt));
}

int main() {
  double* out;
  int64_t* cyc;
  double* err;
  hipMalloc(&out, 1024 * sizeof(double));
  hipMalloc(&cyc, sizeof(int64_t));
  hipMalloc(&err, 3 * sizeof(double));
  const int n = 4096;
  int64_t c;
  auto run = [&](const char* name, int per) {
    hipDeviceSynchronize();
    hipMemcpy(&c, cyc, sizeof(c), hipMemcpyDeviceToHost);
    printf("%-34s %8.2f cycles per op\n", name, (double)c / per);
  };
  for (int rep = 0; rep < 2; rep++) {
    hipLaunchKernelGGL(k_fma_chain, dim3(1), dim3(64), 0, 0, n, 0.999, 1e-3, out, cyc);
    if (rep) run("dependent v_fma_f64 (1 wave)", n);
    hipLaunchKernelGGL(k_fma32_chain, dim3(1), dim3(64), 0, 0, n, 0.999f, 1e-3f, out, cyc);
    if (rep) run("dependent v_fma_f32 (1 wave)", n);
    hipLaunchKernelGGL(k_rcp_chain, dim3(1), dim3(64), 0, 0, n, 0.5, out, cyc);
    if (rep) run("dependent v_rcp_f64 + v_add_f64", n);
    hipLaunchKernelGGL(k_rsq_chain, dim3(1), dim3(64), 0, 0, n, 0.5, out, cyc);
    if (rep) run("dependent v_rsq_f64 + v_add_f64", n);
    hipLaunchKernelGGL(k_div_chain, dim3(1), dim3(64), 0, 0, n, 0.5, out, cyc);
    if (rep) run("dependent IEEE 1.0/x + add (f64)", n);
    hipLaunchKernelGGL(k_readlane_chain, dim3(1), dim3(64), 0, 0, n, out, cyc);
    if (rep) run("dependent 2x readlane + fma (f64)", n);
    hipLaunchKernelGGL(k_fma_tput, dim3(1), dim3(1024), 0, 0, n, 0.999, 1e-3, out, cyc);
    if (rep) run("fp64 FMA tput, 16 waves x 8 chains", n * 8 * 4);  // per wave-instr per SIMD
  }
  hipMemset(err, 0, 3 * sizeof(double));
  hipLaunchKernelGGL(k_accuracy, dim3(256), dim3(256), 0, 0, 4096, 12345ull, err);
  double e[3];
  hipMemcpy(e, err, sizeof(e), hipMemcpyDeviceToHost);
  printf("max rel err v_rcp_f64 %.3e  v_rsq_f64 %.3e  v_sqrt_f64 %.3e (2^-52 = 2.2e-16)\n", e[0],
         e[1], e[2]);
  return 0;
}
