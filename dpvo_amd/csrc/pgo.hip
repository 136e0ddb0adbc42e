// Sim3 pose-graph normal equations for cuda_ba.solve_system (loop-closure
// backend, dpvo/fastba/ba.cpp:120-180; caller dpvo/loop_closure/optim_utils.py:229).
//
// The reference builds a sparse J [7r, 7n] from the per-edge 7x7 blocks
// J_Ginv_i / J_Ginv_j (ba.cpp:141-158), forms A = J^T J and b = -J^T res in
// fp64 on the host (ba.cpp:160-163), damps the diagonal (164-165) and solves
// with Eigen's SimplicialCholesky (103-118).  Here each edge is one wave that
// computes its four 7x7 blocks of J^T J and its two 7-vectors of J^T res in
// fp64 (the fp32 inputs widened, as Eigen's cast) and adds them into a dense
// fp64 [7n, 7n] system in HBM; a second launch applies the damping.  The
// dense layout costs 392 n^2 bytes (n = 4096 poses: 6.6 GB, comfortably
// resident in 288 GB) and hands a plain SPD matrix to the device Cholesky.
#include "common.hpp"

namespace dpvo {
namespace {

constexpr int kDof = 7;

__global__ void __launch_bounds__(64) pgo_assemble_kernel(
    const float* __restrict__ Ji, const float* __restrict__ Jj,
    const int64_t* __restrict__ ii, const int64_t* __restrict__ jj,
    const float* __restrict__ res, int r, int n, double* __restrict__ A,
    double* __restrict__ b) {
  const int x = blockIdx.x;
  if (x >= r) return;
  __shared__ double si[kDof * kDof], sj[kDof * kDof], sv[kDof];
  const int t = threadIdx.x;
  if (t < kDof * kDof) {
    si[t] = (double)Ji[(size_t)x * 49 + t];
    sj[t] = (double)Jj[(size_t)x * 49 + t];
  }
  if (t < kDof) sv[t] = (double)res[(size_t)x * 7 + t];
  __syncthreads();
  const int64_t i = ii[x], j = jj[x];
  const size_t N7 = (size_t)n * kDof;
  if (t < kDof * kDof) {
    const int l = t / kDof, m = t % kDof;
    double aii = 0.0, ajj = 0.0, aij = 0.0, aji = 0.0;
    for (int k = 0; k < kDof; k++) {  // (J^T J)[l][m] = sum_k J[k][l] J[k][m]
      aii += si[k * kDof + l] * si[k * kDof + m];
      ajj += sj[k * kDof + l] * sj[k * kDof + m];
      aij += si[k * kDof + l] * sj[k * kDof + m];
      aji += sj[k * kDof + l] * si[k * kDof + m];
    }
    atomicAdd(&A[(i * kDof + l) * N7 + i * kDof + m], aii);
    atomicAdd(&A[(j * kDof + l) * N7 + j * kDof + m], ajj);
    atomicAdd(&A[(i * kDof + l) * N7 + j * kDof + m], aij);
    atomicAdd(&A[(j * kDof + l) * N7 + i * kDof + m], aji);
  } else if (t < kDof * kDof + 2 * kDof) {
    const int s = t - kDof * kDof;  // 0..6: pose i, 7..13: pose j
    const double* J = s < kDof ? si : sj;
    const int l = s % kDof;
    double acc = 0.0;
    for (int k = 0; k < kDof; k++) acc += J[k * kDof + l] * sv[k];
    atomicAdd(&b[(s < kDof ? i : j) * kDof + l], -acc);
  }
}

// A.diagonal() += A.diagonal() * lm; A.diagonal() += ep  (ba.cpp:164-165)
__global__ void pgo_damp_kernel(double* __restrict__ A, int n7, double ep, double lm) {
  const int d = blockIdx.x * blockDim.x + threadIdx.x;
  if (d >= n7) return;
  double* a = &A[(size_t)d * n7 + d];
  const double v = *a;
  *a = (v + v * lm) + ep;
}

}  // namespace
}  // namespace dpvo

DPVO_EXPORT int dpvo_pgo_assemble(const float* J_Ginv_i, const float* J_Ginv_j,
                                  const int64_t* ii, const int64_t* jj, const float* res,
                                  int r, int n, float ep, float lm, double* A, double* b,
                                  void* stream_) {
  hipStream_t stream = (hipStream_t)stream_;
  if (r < 0 || n < 0 || (r > 0 && (!J_Ginv_i || !J_Ginv_j || !ii || !jj || !res)) ||
      (n > 0 && (!A || !b)))
    return DPVO_ERR_INVALID;
  const size_t n7 = (size_t)n * 7;
  if (n7 > (size_t)INT32_MAX) return DPVO_ERR_INVALID;
  if (n == 0) return DPVO_OK;
  if (hipMemsetAsync(A, 0, n7 * n7 * sizeof(double), stream) != hipSuccess ||
      hipMemsetAsync(b, 0, n7 * sizeof(double), stream) != hipSuccess)
    return DPVO_ERR_LAUNCH;
  if (r > 0)
    hipLaunchKernelGGL(dpvo::pgo_assemble_kernel, dim3(r), dim3(64), 0, stream, J_Ginv_i,
                       J_Ginv_j, ii, jj, res, r, n, A, b);
  hipLaunchKernelGGL(dpvo::pgo_damp_kernel, dim3((unsigned)((n7 + 255) / 256)), dim3(256), 0,
                     stream, A, (int)n7, (double)ep, (double)lm);
  return hipGetLastError() == hipSuccess ? DPVO_OK : DPVO_ERR_LAUNCH;
}
