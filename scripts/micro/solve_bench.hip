// Standalone timing of the dense pose solve (ba_device.hpp chol32_solve) in
// one 256-thread workgroup, with per-phase shader-clock stamps, against a host
// fp64 Cholesky on a random SPD system shaped like a DPVO window.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I include -I dpvo_amd/csrc \
//         scripts/micro/solve_bench.hip -o scripts/micro/solve_bench
//   ./scripts/micro/solve_bench [N=11] [refine=1]
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <vector>

#include "ba_device.hpp"

using namespace dpvo::bad;

__global__ void __launch_bounds__(256) k_solve(const double* S, const double* y, int N, int refine,
                                               double* dX, int64_t* st, int* fail) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  const int NB = N * (N + 1) / 2;
  double* Sd = (double*)lds;
  double* yd = Sd + 36 * NB;
  Solver32 sv;
  sv.S = Sd;
  sv.y = yd;
  sv.x = yd + 6 * N;
  sv.part = sv.x + 6 * N;
  sv.A = (float*)(sv.part + 24 * N);
  sv.Li = sv.A + 36 * NB;
  sv.w = sv.Li + 36 * N;
  sv.Nf = sv.w + 6 * N;
  for (int k = threadIdx.x; k < 36 * NB; k += blockDim.x) Sd[k] = S[k];
  for (int k = threadIdx.x; k < 6 * N; k += blockDim.x) yd[k] = y[k];
  __shared__ int f;
  if (threadIdx.x == 0) f = 0;
  __syncthreads();
  chol32_solve(sv, N, dX, &f, refine != 0, nullptr, st);
  if (threadIdx.x == 0) *fail = f;
}

static int lb(int a, int b) { return a * (a + 1) / 2 + b; }

int main(int argc, char** argv) {
  const int N = argc > 1 ? atoi(argv[1]) : 11;
  const int refine = argc > 2 ? atoi(argv[2]) : 1;
  const int n = 6 * N, NB = N * (N + 1) / 2;
  srand(1);
  std::vector<double> G(n * n), D(n * n, 0.0), y(n);
  for (auto& v : G) v = (rand() / (double)RAND_MAX - 0.5) * 300.0;
  for (int i = 0; i < n; i++)
    for (int j = 0; j < n; j++) {
      double s = 0;
      for (int k = 0; k < n; k++) s += G[i * n + k] * G[j * n + k];
      D[i * n + j] = s;
    }
  for (int i = 0; i < n; i++) D[i * n + i] += 1e-4 * D[i * n + i] + 1.0;
  for (auto& v : y) v = rand() / (double)RAND_MAX - 0.5;
  std::vector<double> Sb(36 * NB);
  for (int a = 0; a < N; a++)
    for (int b = 0; b <= a; b++)
      for (int x = 0; x < 6; x++)
        for (int z = 0; z < 6; z++) Sb[36 * lb(a, b) + 6 * x + z] = D[(6 * a + x) * n + 6 * b + z];
  // host fp64 Cholesky solve
  std::vector<double> L(n * n, 0.0), ref(n);
  for (int j = 0; j < n; j++) {
    double s = D[j * n + j];
    for (int k = 0; k < j; k++) s -= L[j * n + k] * L[j * n + k];
    L[j * n + j] = sqrt(s);
    for (int i = j + 1; i < n; i++) {
      double t = D[i * n + j];
      for (int k = 0; k < j; k++) t -= L[i * n + k] * L[j * n + k];
      L[i * n + j] = t / L[j * n + j];
    }
  }
  std::vector<double> z(n);
  for (int i = 0; i < n; i++) {
    double s = y[i];
    for (int k = 0; k < i; k++) s -= L[i * n + k] * z[k];
    z[i] = s / L[i * n + i];
  }
  for (int i = n - 1; i >= 0; i--) {
    double s = z[i];
    for (int k = i + 1; k < n; k++) s -= L[k * n + i] * ref[k];
    ref[i] = s / L[i * n + i];
  }
  double *dS, *dy, *dX;
  int64_t* dst;
  int* dfail;
  hipMalloc(&dS, sizeof(double) * Sb.size());
  hipMalloc(&dy, sizeof(double) * n);
  hipMalloc(&dX, sizeof(double) * n);
  hipMalloc(&dst, sizeof(int64_t) * 64);
  hipMalloc(&dfail, sizeof(int));
  hipMemcpy(dS, Sb.data(), sizeof(double) * Sb.size(), hipMemcpyHostToDevice);
  hipMemcpy(dy, y.data(), sizeof(double) * n, hipMemcpyHostToDevice);
  const size_t lds = solver32_bytes(N) + 256;
  hipFuncSetAttribute((const void*)k_solve, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  const int reps = 50;
  std::vector<std::vector<long long>> ph(64);
  for (int r = 0; r < reps; r++) {
    hipMemset(dst, 0, sizeof(int64_t) * 64);
    hipLaunchKernelGGL(k_solve, dim3(1), dim3(256), lds, 0, dS, dy, N, refine, dX, dst, dfail);
    hipDeviceSynchronize();
    int64_t h[64];
    hipMemcpy(h, dst, sizeof(h), hipMemcpyDeviceToHost);
    for (int k = 1; k < 64; k++)
      if (h[k] && h[k - 1]) ph[k].push_back(h[k] - h[k - 1]);
    if (r == reps - 1) {
      std::vector<double> got(n);
      int fail = 0;
      hipMemcpy(got.data(), dX, sizeof(double) * n, hipMemcpyDeviceToHost);
      hipMemcpy(&fail, dfail, sizeof(int), hipMemcpyDeviceToHost);
      double e = 0, nr = 0;
      for (int i = 0; i < n; i++) {
        e += (got[i] - ref[i]) * (got[i] - ref[i]);
        nr += ref[i] * ref[i];
      }
      printf("N=%d refine=%d fail=%d rel.err=%.3e total=%lld cyc\n", N, refine, fail,
             sqrt(e / nr), (long long)(h[44] - h[0]));
    }
  }
  auto med = [&](int k) {
    auto v = ph[k];
    if (v.empty()) return -1LL;
    std::sort(v.begin(), v.end());
    return v[v.size() / 2];
  };
  printf("convert+chol0 %lld\n", med(1));
  long long pan = 0, trl = 0;
  for (int k = 0; k + 1 < N; k++) {
    printf("step %2d panel %5lld trailing %5lld\n", k, med(2 + 2 * k), med(3 + 2 * k));
    pan += med(2 + 2 * k);
    trl += med(3 + 2 * k);
  }
  printf("panel total %lld trailing total %lld (shader cycles)\n", pan, trl);
  printf("backsub %lld residual %lld refine-subst %lld tail %lld\n", med(41), med(42), med(43),
         med(44));
  return 0;
}
