// Window-solver A/B: ba_solve.hpp wsolve (blocked Cholesky + LDL^T sweeps)
// against ba_gjsolve.hpp gjsolve (block Gauss-Jordan inverse + matvecs), one
// 256-thread workgroup each, on the oracle's damped Schur systems
// (scripts/micro/make_solve_systems.py -> scripts/micro/data/*.bin) and on
// random SPD systems for every N = 1..16.  Prints rel. error against the
// host fp64 solution and shader cycles (s_memtime) per solve.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -fno-slp-vectorize -I include \
//         -I dpvo_amd/csrc -I scripts/micro scripts/micro/gj_bench.hip -o scripts/micro/gj_bench
// Result (profiles/r04_solver_gj/): the Gauss-Jordan inverse is 2.2-3.4x
// SLOWER than the blocked Cholesky at N = 10-16 (its per-step work is a
// full-matrix update, ~1000 VALU instructions per wave per block step at one
// wave per SIMD); not adopted.
//   ./scripts/micro/gj_bench
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <string>
#include <vector>

#include "ba_gjsolve.hpp"

using namespace dpvo::bad;

#define CK(x)                                                               \
  do {                                                                      \
    hipError_t e = (x);                                                     \
    if (e != hipSuccess) {                                                  \
      printf("HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__); \
      exit(1);                                                              \
    }                                                                       \
  } while (0)

__global__ void __launch_bounds__(256) k_solve(const double* S, const double* y, int N, int refine,
                                               int mode, double* dX, long long* cyc, int* fail) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  const int NB = N * (N + 1) / 2, n = 6 * N;
  double* Sd = (double*)lds;
  double* yd = Sd + 36 * NB;
  double* xd = yd + n;
  double* rd = xd + n;
  float* f = (float*)(rd + n);
  __shared__ int fl;
  for (int k = threadIdx.x; k < 36 * NB; k += blockDim.x) Sd[k] = S[k];
  for (int k = threadIdx.x; k < n; k += blockDim.x) yd[k] = y[k];
  __syncthreads();
  const long long t0 = __builtin_amdgcn_s_memtime();
  bool ok;
  if (mode == 0) {
    WSolve s;
    s.S = Sd;
    s.y = yd;
    s.x = xd;
    s.r = rd;
    s.A = f;
    s.Z = s.A + 36 * NB;
    s.v0 = s.Z + 36 * NB;
    s.v1 = s.v0 + n;
    ok = wsolve(s, N, refine, &fl);
  } else {
    GJSolve s;
    s.S = Sd;
    s.y = yd;
    s.x = xd;
    gj_carve(s, f, N);
    ok = gjsolve(s, N, refine, &fl);
  }
  const long long t1 = __builtin_amdgcn_s_memtime();
  for (int k = threadIdx.x; k < n; k += blockDim.x) dX[k] = xd[k];
  if (threadIdx.x == 0) {
    *cyc = t1 - t0;
    *fail = ok ? 0 : 1;
  }
}

struct Sys {
  std::string name;
  int N;
  std::vector<double> S, y, x;
};

static bool load(const char* path, Sys& s) {
  FILE* f = fopen(path, "rb");
  if (!f) return false;
  int N = 0;
  if (fread(&N, 4, 1, f) != 1) return false;
  const int NB = N * (N + 1) / 2, n = 6 * N;
  s.N = N;
  s.S.resize(36 * NB);
  s.y.resize(n);
  s.x.resize(n);
  bool ok = fread(s.S.data(), 8, s.S.size(), f) == s.S.size() &&
            fread(s.y.data(), 8, n, f) == (size_t)n && fread(s.x.data(), 8, n, f) == (size_t)n;
  fclose(f);
  return ok;
}

// random SPD: Gram + diagonal, solved on the host (dense Cholesky, fp64)
static Sys random_sys(int N, unsigned seed) {
  Sys s;
  s.name = "rand_N" + std::to_string(N);
  s.N = N;
  const int n = 6 * N, NB = N * (N + 1) / 2;
  srand(seed);
  std::vector<double> G((size_t)n * 2 * n), A((size_t)n * n);
  for (auto& v : G) v = rand() / (double)RAND_MAX - 0.5;
  for (int i = 0; i < n; i++)
    for (int j = 0; j < n; j++) {
      double t = 0;
      for (int k = 0; k < 2 * n; k++) t += G[i * 2 * n + k] * G[j * 2 * n + k];
      A[i * n + j] = t + (i == j ? 1.0 : 0.0);
    }
  s.y.resize(n);
  for (auto& v : s.y) v = rand() / (double)RAND_MAX - 0.5;
  s.S.assign(36 * NB, 0.0);
  for (int a = 0; a < N; a++)
    for (int b = 0; b <= a; b++)
      for (int r = 0; r < 6; r++)
        for (int c = 0; c < 6; c++)
          s.S[36 * (a * (a + 1) / 2 + b) + 6 * r + c] = A[(6 * a + r) * n + 6 * b + c];
  // Cholesky solve
  std::vector<double> L(A);
  for (int j = 0; j < n; j++) {
    for (int k = 0; k < j; k++) L[j * n + j] -= L[j * n + k] * L[j * n + k];
    L[j * n + j] = sqrt(L[j * n + j]);
    for (int i = j + 1; i < n; i++) {
      for (int k = 0; k < j; k++) L[i * n + j] -= L[i * n + k] * L[j * n + k];
      L[i * n + j] /= L[j * n + j];
    }
  }
  std::vector<double> z(n);
  for (int i = 0; i < n; i++) {
    double t = s.y[i];
    for (int k = 0; k < i; k++) t -= L[i * n + k] * z[k];
    z[i] = t / L[i * n + i];
  }
  s.x.resize(n);
  for (int i = n - 1; i >= 0; i--) {
    double t = z[i];
    for (int k = i + 1; k < n; k++) t -= L[k * n + i] * s.x[k];
    s.x[i] = t / L[i * n + i];
  }
  return s;
}

int main(int argc, char** argv) {
  const int refine = argc > 1 ? atoi(argv[1]) : 1;
  const int reps = 25;
  std::vector<Sys> systems;
  for (const char* nm : {"cfg2_s0", "cfg2_s4", "dpvo10", "dpvo25"}) {
    Sys s;
    s.name = nm;
    std::string p = std::string("scripts/micro/data/") + nm + ".bin";
    if (load(p.c_str(), s)) systems.push_back(s);
    else printf("missing %s\n", p.c_str());
  }
  for (int N = 1; N <= 16; N++) systems.push_back(random_sys(N, 100 + N));
  CK(hipFuncSetAttribute((const void*)k_solve, hipFuncAttributeMaxDynamicSharedMemorySize,
                         120 * 1024));
  double *dS, *dy, *dx;
  long long* dc;
  int* df;
  CK(hipMalloc(&dS, 8 * 36 * 136));
  CK(hipMalloc(&dy, 8 * 96));
  CK(hipMalloc(&dx, 8 * 96));
  CK(hipMalloc(&dc, 8));
  CK(hipMalloc(&df, 4));
  for (const Sys& s : systems) {
    const int N = s.N, n = 6 * N, NB = N * (N + 1) / 2;
    CK(hipMemcpy(dS, s.S.data(), 8 * s.S.size(), hipMemcpyHostToDevice));
    CK(hipMemcpy(dy, s.y.data(), 8 * n, hipMemcpyHostToDevice));
    const size_t lds = 8 * (36 * NB + 4 * n) + 4 * (2 * 36 * NB + 8 * n) + 4 * gjsolve_floats(N) + 256;
    printf("%-10s N=%2d", s.name.c_str(), N);
    for (int mode = 0; mode < 2; mode++) {
      std::vector<long long> cy;
      double err = 0;
      int fail = 0;
      for (int r = 0; r < reps; r++) {
        hipLaunchKernelGGL(k_solve, dim3(1), dim3(256), lds, 0, dS, dy, N, refine, mode, dx, dc, df);
        CK(hipDeviceSynchronize());
        long long c;
        CK(hipMemcpy(&c, dc, 8, hipMemcpyDeviceToHost));
        cy.push_back(c);
      }
      std::vector<double> x(n);
      CK(hipMemcpy(x.data(), dx, 8 * n, hipMemcpyDeviceToHost));
      CK(hipMemcpy(&fail, df, 4, hipMemcpyDeviceToHost));
      double num = 0, den = 0;
      for (int i = 0; i < n; i++) {
        num += (x[i] - s.x[i]) * (x[i] - s.x[i]);
        den += s.x[i] * s.x[i];
      }
      err = sqrt(num / den);
      std::sort(cy.begin(), cy.end());
      printf("  %s: rel %.2e fail %d cyc %lld", mode ? "gj" : "chol", err, fail, cy[reps / 2]);
    }
    printf("\n");
  }
  return 0;
}
