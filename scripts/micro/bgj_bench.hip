// Superblock inverse of the large-graph BA (ba_bgj.hpp wg_bgj_inverse, the
// 8 dependent k_cr_inv launches of a cfg4 solve, 36 us each in
// profiles/r03_cfg4_solve_launches.txt): one 1024-thread workgroup inverting a
// random SPD m x m matrix (m = 72 = cfg4's superblock, and 48 / 96), with
// the total cycles and the max |A A^-1 - I| (the per-phase stamps of round 4
// and the per-thread pivot-solve variant live in git history: the product
// header carries no diagnostic hooks since round 6).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I include -I dpvo_amd/csrc \
//         scripts/micro/bgj_bench.hip -o scripts/micro/bgj_bench
// (round-4 results: profiles/r04_cfg4_bgj_phases.txt)
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <vector>

__device__ long long* g_stamp;
#define BGJ_STAMP(k)                                                         \
  do {                                                                       \
    if (threadIdx.x == 0) g_stamp[(k)] = (long long)__builtin_amdgcn_s_memtime(); \
  } while (0)
#include "ba_bgj.hpp"

using namespace dpvo::gba;

#define CK(x)                                                                     \
  do {                                                                            \
    hipError_t e_ = (x);                                                          \
    if (e_ != hipSuccess) {                                                       \
      printf("HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
      exit(1);                                                                    \
    }                                                                             \
  } while (0)

__global__ void __launch_bounds__(1024) k_inv(double* A, int m, long long* stamps, int* ok) {
  extern __shared__ __attribute__((aligned(16))) double lds[];
  if (threadIdx.x == 0) g_stamp = stamps;
  __syncthreads();
  const bool good = wg_bgj_inverse(A, m, m, A, lds);
  if (threadIdx.x == 0) *ok = good ? 1 : 0;
}

int main() {
  for (int m : {48, 72, 96}) {
    std::vector<double> G((size_t)m * 2 * m), A((size_t)m * m);
    srand(7 + m);
    for (auto& v : G) v = rand() / (double)RAND_MAX - 0.5;
    for (int i = 0; i < m; i++)
      for (int j = 0; j < m; j++) {
        double t = 0;
        for (int k = 0; k < 2 * m; k++) t += G[i * 2 * m + k] * G[j * 2 * m + k];
        A[i * m + j] = t + (i == j ? 1.0 : 0.0);
      }
    double* dA;
    long long* dst;
    int* dok;
    const int nst = 4 * (m / 6) + 8;
    CK(hipMalloc(&dA, 8 * A.size()));
    CK(hipMalloc(&dst, 8 * nst));
    CK(hipMalloc(&dok, 4));
    const size_t lds = sizeof(double) * kBgjDoubles;
    std::vector<long long> best(nst, 1LL << 60);
    std::vector<double> inv(A.size());
    for (int rep = 0; rep < 20; rep++) {
      CK(hipMemcpy(dA, A.data(), 8 * A.size(), hipMemcpyHostToDevice));
      CK(hipMemset(dst, 0, 8 * nst));
      hipLaunchKernelGGL(k_inv, dim3(1), dim3(1024), lds, 0, dA, m, dst, dok);
      CK(hipDeviceSynchronize());
      std::vector<long long> st(nst);
      CK(hipMemcpy(st.data(), dst, 8 * nst, hipMemcpyDeviceToHost));
      const long long total = st[4 * (m / 6)] - st[0];
      if (total < best[nst - 1]) {
        best = st;
        best[nst - 1] = total;
      }
    }
    CK(hipMemcpy(inv.data(), dA, 8 * A.size(), hipMemcpyDeviceToHost));
    int ok = 0;
    CK(hipMemcpy(&ok, dok, 4, hipMemcpyDeviceToHost));
    double err = 0;
    for (int i = 0; i < m; i++)
      for (int j = 0; j < m; j++) {
        double t = 0;
        for (int k = 0; k < m; k++) t += A[i * m + k] * inv[k * m + j];
        err = std::max(err, fabs(t - (i == j ? 1.0 : 0.0)));
      }
    const int nb = m / 6;
    long long ph[4] = {0, 0, 0, 0};
    for (int K = 0; K < nb; K++) {
      long long prev = (K == 0) ? best[0] : best[4 * K];
      for (int q = 0; q < 4; q++) {
        ph[q] += best[1 + 4 * K + q] - prev;
        prev = best[1 + 4 * K + q];
      }
    }
    printf("m=%2d ok=%d err=%.2e total=%lld cycles (s_memtime) per step: publish %lld pivot %lld "
           "W/V %lld update %lld\n",
           m, ok, err, best[nst - 1], ph[0] / nb, ph[1] / nb, ph[2] / nb, ph[3] / nb);
    CK(hipFree(dA));
    CK(hipFree(dst));
    CK(hipFree(dok));
  }
  return 0;
}
