// Standalone check + timing of the window solver (dpvo_amd/csrc/ba_solve.hpp
// wsolve): one 256-thread workgroup, random SPD systems shaped like a DPVO
// window (Gram matrix + the reference's damping), against a host fp64
// Cholesky.  Prints rel. error and shader cycles (s_memtime) per solve.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I include -I dpvo_amd/csrc \
//         scripts/micro/wsolve_bench.hip -o scripts/micro/wsolve_bench
//   ./scripts/micro/wsolve_bench [N=11] [refine=1] [cond_scale=300]
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <vector>

#include "ba_solve.hpp"
#ifdef WSOLVE_MMA
#include "ba_gj_mma.hpp"
#endif

using namespace dpvo::bad;

__global__ void __launch_bounds__(256) k_wsolve(const double* S, const double* y, int N, int refine,
                                                double* dX, long long* cyc, int* fail, long long* stg) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  const int NB = N * (N + 1) / 2, n = 6 * N;
  double* Sd = (double*)lds;
  double* yd = Sd + 36 * NB;
  WSolve s;
  s.S = Sd;
  s.y = yd;
  s.x = yd + n;
  s.r = s.x + n;
  s.A = (float*)(s.r + n);
  s.Z = s.A + 36 * NB;
  s.v0 = s.Z + 36 * NB;
  s.v1 = s.v0 + n;
  __shared__ int f;
  __shared__ long long stl[64];
  for (int k = threadIdx.x; k < 36 * NB; k += blockDim.x) Sd[k] = S[k];
  for (int k = threadIdx.x; k < n; k += blockDim.x) yd[k] = y[k];
  __syncthreads();
#ifdef WSOLVE_MMA
  // the sweep solver's workspace after S, y, x (16-B aligned)
  GJSolve g;
  g.S = Sd;
  g.y = yd;
  g.x = s.x;
  const int np = gj_np(N);
  {  // 16-B aligned by pointer arithmetic (an integer round trip loses the LDS
     // address space: every access would become a flat load)
    char* p = reinterpret_cast<char*>(s.r + n);
    p += (16 - (int)(reinterpret_cast<uintptr_t>(p) & 15)) & 15;
    g.Mi = reinterpret_cast<float*>(p);
  }
  g.C = g.Mi + np * np;
  g.V = g.C + 8 * np;
  g.W = g.V + 8 * np;
  g.v = g.W + 8 * np;
  const long long t0 = __builtin_amdgcn_s_memtime();
  const bool ok = wsolve_mma(g, N, refine, &f, stl);
#else
  const long long t0 = __builtin_amdgcn_s_memtime();
  const bool ok = wsolve(s, N, refine, &f, stl);
#endif
  const long long t1 = __builtin_amdgcn_s_memtime();
  for (int k = threadIdx.x; k < n; k += blockDim.x) dX[k] = s.x[k];
  for (int k = threadIdx.x; k < 64; k += blockDim.x) stg[k] = stl[k];
  if (threadIdx.x == 0) {
    *cyc = t1 - t0;
    *fail = ok ? 0 : 1;
  }
}

static int lb(int a, int b) { return a * (a + 1) / 2 + b; }

int main(int argc, char** argv) {
  const int N = argc > 1 ? atoi(argv[1]) : 11;
  const int refine = argc > 2 ? atoi(argv[2]) : 1;
  const double scale = argc > 3 ? atof(argv[3]) : 300.0;
  const int n = 6 * N, NB = N * (N + 1) / 2;
  srand(1);
  std::vector<double> G(n * 2 * n), D(n * n, 0.0), y(n);
  for (auto& v : G) v = (rand() / (double)RAND_MAX - 0.5) * scale;
  for (int i = 0; i < n; i++)
    for (int j = 0; j < n; j++) {
      double s = 0;
      for (int k = 0; k < 2 * n; k++) s += G[i * 2 * n + k] * G[j * 2 * n + k] * (k % 7 == 0 ? 1e-3 : 1.0);
      D[i * n + j] = s;
    }
  for (int i = 0; i < n; i++) D[i * n + i] += 1e-4 * D[i * n + i] + 1.0;
  for (auto& v : y) v = rand() / (double)RAND_MAX - 0.5;
  std::vector<double> Sb(36 * NB);
  for (int a = 0; a < N; a++)
    for (int b = 0; b <= a; b++)
      for (int x = 0; x < 6; x++)
        for (int z = 0; z < 6; z++) Sb[36 * lb(a, b) + 6 * x + z] = D[(6 * a + x) * n + 6 * b + z];
  std::vector<double> L(n * n, 0.0), ref(n), z(n);
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
  double dmin = 1e300, dmax = 0;
  for (int i = 0; i < n; i++) {
    dmin = std::min(dmin, L[i * n + i]);
    dmax = std::max(dmax, L[i * n + i]);
  }
  double *dS, *dy, *dX;
  long long* dc;
  long long* dst;
  hipMalloc(&dst, sizeof(long long) * 64);
  int* dfail;
  hipMalloc(&dS, sizeof(double) * Sb.size());
  hipMalloc(&dy, sizeof(double) * n);
  hipMalloc(&dX, sizeof(double) * n);
  hipMalloc(&dc, sizeof(long long));
  hipMalloc(&dfail, sizeof(int));
  hipMemcpy(dS, Sb.data(), sizeof(double) * Sb.size(), hipMemcpyHostToDevice);
  hipMemcpy(dy, y.data(), sizeof(double) * n, hipMemcpyHostToDevice);
  const size_t lds = sizeof(double) * (36 * NB + 3 * n) + wsolve_bytes(N) + 64
#ifdef WSOLVE_MMA
                     + gj_bytes(N)
#endif
      ;
  hipFuncSetAttribute((const void*)k_wsolve, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  std::vector<long long> cs;
  for (int r = 0; r < 40; r++) {
    hipLaunchKernelGGL(k_wsolve, dim3(1), dim3(256), lds, 0, dS, dy, N, refine, dX, dc, dfail, dst);
    hipDeviceSynchronize();
    long long c;
    hipMemcpy(&c, dc, sizeof(c), hipMemcpyDeviceToHost);
    cs.push_back(c);
  }
  std::sort(cs.begin(), cs.end());
  long long h[64];
  hipMemcpy(h, dst, sizeof(h), hipMemcpyDeviceToHost);
#ifdef WSOLVE_MMA
  printf("load %lld |", h[1] - h[0]);
  for (int k = 0; k < N; k++) printf(" %lld", h[2 + k] - h[1 + k]);
  printf(" | store %lld | solve %lld", h[40] - h[1 + N], h[41] - h[40]);
  printf(" | k2: publish+bar %lld rows %lld bar %lld mfma %lld fix %lld", h[50] - h[3], h[51] - h[50],
         h[52] - h[51], h[53] - h[52], h[4] - h[53]);
  for (int it = 0; it < refine; it++) printf(" ref%d %lld", it, h[42 + it] - h[41 + it]);
  printf("\n");
#else
  printf("pre %lld piv0 %lld |", h[1] - h[0], 0LL);
  for (int k = 0; k < N; k++) printf(" %lld", h[2 + k] - (k ? h[1 + k] : h[1]));
  printf(" | post %lld | solve %lld", h[40] - h[1 + N], h[41] - h[40]);
  printf(" | k2 (from step start): w0 %lld w1 %lld w2 %lld w3 %lld w3+ldl %lld", h[50] - h[3],
         h[52] - h[3], h[53] - h[3], h[54] - h[3], h[55] - h[3]);
#ifdef WSOLVE_STEP_STAMPS
  printf(" | w0: update %lld readlane %lld chol %lld stores %lld panel %lld", h[56] - h[3],
         h[57] - h[56], h[58] - h[57], h[59] - h[58], h[50] - h[59]);
#endif
  for (int it = 0; it < refine; it++) printf(" ref%d %lld", it, h[42 + it] - (it ? h[41 + it] : h[41]));
  printf("\n");
#endif
  std::vector<double> got(n);
  int fail = 0;
  hipMemcpy(got.data(), dX, sizeof(double) * n, hipMemcpyDeviceToHost);
  hipMemcpy(&fail, dfail, sizeof(int), hipMemcpyDeviceToHost);
  double e = 0, nr = 0;
  for (int i = 0; i < n; i++) {
    e += (got[i] - ref[i]) * (got[i] - ref[i]);
    nr += ref[i] * ref[i];
  }
  printf("N=%d refine=%d cond~%.1e fail=%d rel.err=%.3e median=%lld cyc (%.2f us @2.4GHz)\n", N,
         refine, (dmax * dmax) / (dmin * dmin), fail, sqrt(e / nr), cs[cs.size() / 2],
         cs[cs.size() / 2] / 2400.0);
  return 0;
}
