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

// ===========================================================================
// Structured sparse solve (the default path of cuda_ba.solve_system).
//
// A loop-closure pose graph is an odometry chain plus a few long edges, so
// A = J^T J (7x7 blocks) is block-tridiagonal except for the rows / columns
// of the poses a long edge (|i - j| > 1) touches.  Those "border" poses are
// ordered last; the remaining "interior" poses form runs ("segments") of
// consecutive poses whose only couplings are the chain blocks (p, p - 1) and,
// at the two ends of a run, the chain blocks to the neighbouring border pose.
//   1. assemble (one wave per 7x7 block, contributing edges summed in
//      ascending edge order: deterministic, no atomics) into per-pose diagonal
//      / sub-diagonal blocks, the segment-end coupling blocks and the dense
//      border matrix S;
//   2. per segment (one wave), a block Cholesky sweep T = L L^T along the
//      run with 15 right-hand sides [b | C_left | C_right] forward-substituted
//      (Z = L^-1 rhs) and the Schur terms C^T T^-1 C = W^T W, C^T T^-1 b =
//      W^T z accumulated in a fixed order;
//   3. S -= sum of the segments' terms (one writer per block), the dense SPD
//      border solve runs in the caller (small: 7 x #border poses);
//   4. per segment, the backward sweep x = L^-T (z - W x_border).
// Fill-in is zero inside a segment, so the work is O(n) 7x7 block operations
// plus a dense solve of the border only (reference: Eigen
// SimplicialCholesky with its fill-reducing ordering, ba.cpp:103-118).
// ===========================================================================
#include <algorithm>
#include <utility>
#include <vector>

namespace dpvo {
namespace {

// plan header (int64): counts, table offsets (in int64 units) and workspace
// offsets (in doubles)
enum PgoHdr {
  hNf = 0, hNtask, hNseg, hM, hTasks, hContrib, hSegs, hBorder,
  hD, hE, hB, hL, hMM, hZ, hCL, hCR, hWR, hGLL, hGLR, hGRR, hgL, hgR, hS, hBB, hDelta, hWs,
  hCount = 32
};
constexpr int kTaskW = 8;  // a, b, c0, c1, dst, ld, mirror (or -1), bdst (or -1)
constexpr int kSegW = 4;   // p0, p1, uL, uR (border index or -1)
constexpr int kBordW = 3;  // pose, left segment, right segment (or -1)

__global__ void __launch_bounds__(64) pgo_block_kernel(
    const float* __restrict__ Ji, const float* __restrict__ Jj, const int64_t* __restrict__ ii,
    const float* __restrict__ res, const int64_t* __restrict__ plan, double ep, double lm,
    double* __restrict__ ws) {
  const int64_t* T = plan + plan[hTasks] + (int64_t)blockIdx.x * kTaskW;
  const int64_t* contrib = plan + plan[hContrib];
  const int64_t a = T[0], b = T[1], c0 = T[2], c1 = T[3];
  const int t = threadIdx.x;
  __shared__ double ja[49], jb[49], rv[7];
  double acc = 0.0;
  const int l = t / 7, m = t % 7;
  for (int64_t c = c0; c < c1; c++) {
    const int64_t e = contrib[c];
    const bool ai = ii[e] == a, bi = ii[e] == b;
    const float* Pa = (ai ? Ji : Jj) + e * 49;
    const float* Pb = (bi ? Ji : Jj) + e * 49;
    __syncthreads();
    if (t < 49) {
      ja[t] = (double)Pa[t];
      jb[t] = (double)Pb[t];
    } else if (t < 56) {
      rv[t - 49] = (double)res[e * 7 + (t - 49)];
    }
    __syncthreads();
    if (t < 49) {  // (J_a^T J_b)[l][m] = sum_k J_a[k][l] J_b[k][m]
#pragma unroll
      for (int k = 0; k < 7; k++) acc += ja[k * 7 + l] * jb[k * 7 + m];
    } else if (t < 56 && T[7] >= 0) {  // b_a = -J_a^T res
      const int q = t - 49;
#pragma unroll
      for (int k = 0; k < 7; k++) acc -= ja[k * 7 + q] * rv[k];
    }
  }
  if (t < 49) {
    if (a == b && l == m) acc = (acc + acc * lm) + ep;  // ba.cpp:164-165
    ws[T[4] + l * T[5] + m] = acc;
    if (T[6] >= 0) ws[T[6] + m * T[5] + l] = acc;  // mirrored block of the dense border
  } else if (t < 56 && T[7] >= 0) {
    ws[T[7] + (t - 49)] = acc;
  }
}

// 7x7 blocks row-major; one wave per segment
__global__ void __launch_bounds__(64) pgo_segment_forward_kernel(const int64_t* __restrict__ plan,
                                                                 double* __restrict__ ws,
                                                                 int* __restrict__ fail) {
  const int s = blockIdx.x, t = threadIdx.x;
  const int64_t* sg = plan + plan[hSegs] + (int64_t)s * kSegW;
  const int64_t p0 = sg[0], p1 = sg[1];
  const bool hasL = sg[2] >= 0, hasR = sg[3] >= 0;
  double* D = ws + plan[hD];
  double* Eb = ws + plan[hE];
  double* bv = ws + plan[hB];
  double* Lg = ws + plan[hL];
  double* Mg = ws + plan[hMM];
  double* Zg = ws + plan[hZ];
  __shared__ double Dm[49], Em[49], Mm[49], Lc[49], Lp[49], rhs[7 * 15], zc[7 * 15], zp[7 * 15];
  __shared__ double invc[7], invp[7];
  __shared__ int bad;
  if (t == 0) bad = 0;
  double gll = 0.0, gl = 0.0;  // lane t < 49: G_LL[t]; 49 <= t < 56: g_L[t - 49]
  for (int64_t p = p0; p <= p1; p++) {
    const bool first = p == p0;
    if (t < 49) {
      Dm[t] = D[p * 49 + t];
      if (!first) Em[t] = Eb[p * 49 + t];
    }
    for (int u = t; u < 105; u += 64) {
      const int r = u / 15, c = u % 15;
      double v = 0.0;
      if (c == 0) v = bv[p * 7 + r];
      else if (c < 8) v = (first && hasL) ? ws[plan[hCL] + s * 49 + r * 7 + (c - 1)] : 0.0;
      else v = (p == p1 && hasR) ? ws[plan[hCR] + s * 49 + r * 7 + (c - 8)] : 0.0;
      rhs[u] = v;
    }
    __syncthreads();
    if (!first) {
      if (t < 7) {  // M = E L_{p-1}^-T: row t, M L^T = E
        double mr[7];
#pragma unroll
        for (int j = 0; j < 7; j++) {
          double v = Em[t * 7 + j];
#pragma unroll
          for (int k = 0; k < j; k++) v -= mr[k] * Lp[j * 7 + k];
          mr[j] = v * invp[j];
        }
#pragma unroll
        for (int j = 0; j < 7; j++) Mm[t * 7 + j] = mr[j];
      }
      __syncthreads();
      if (t < 49) {  // D -= M M^T
        const int r = t / 7, c = t % 7;
        double v = Dm[t];
#pragma unroll
        for (int k = 0; k < 7; k++) v -= Mm[r * 7 + k] * Mm[c * 7 + k];
        Dm[t] = v;
        Mg[p * 49 + t] = Mm[t];
      }
      for (int u = t; u < 105; u += 64) {  // rhs -= M z_{p-1}
        const int r = u / 15, c = u % 15;
        double v = rhs[u];
#pragma unroll
        for (int k = 0; k < 7; k++) v -= Mm[r * 7 + k] * zp[k * 15 + c];
        rhs[u] = v;
      }
      __syncthreads();
    }
    // Cholesky of the updated diagonal block (right-looking, column j)
    for (int j = 0; j < 7; j++) {
      const double d = Dm[j * 7 + j];
      const bool ok = d > 0.0;  // NaN fails too
      const double Ljj = ok ? sqrt(d) : 1.0, inv = 1.0 / Ljj;
      if (t == 0 && !ok) bad = 1;
      if (t > j && t < 7) Lc[t * 7 + j] = Dm[t * 7 + j] * inv;
      if (t == j) {
        Lc[j * 7 + j] = Ljj;
        invc[j] = inv;
      }
      if (t < 7 && t < j) Lc[t * 7 + j] = 0.0;
      __syncthreads();
      if (t < 49) {
        const int r = t / 7, c = t % 7;
        if (r > j && c > j && c <= r) Dm[t] -= Lc[r * 7 + j] * Lc[c * 7 + j];
      }
      __syncthreads();
    }
    if (t < 15) {  // z = L^-1 rhs, column t
      double z[7];
#pragma unroll
      for (int r = 0; r < 7; r++) {
        double v = rhs[r * 15 + t];
#pragma unroll
        for (int k = 0; k < r; k++) v -= Lc[r * 7 + k] * z[k];
        z[r] = v * invc[r];
        zc[r * 15 + t] = z[r];
      }
    }
    __syncthreads();
    if (t < 49) {  // G_LL += W_L^T W_L, W_L = z columns 1..7
      const int r = t / 7, c = t % 7;
#pragma unroll
      for (int k = 0; k < 7; k++) gll += zc[k * 15 + 1 + r] * zc[k * 15 + 1 + c];
      Lg[p * 49 + t] = Lc[t];
    } else if (t < 56) {  // g_L += W_L^T z_b
      const int r = t - 49;
#pragma unroll
      for (int k = 0; k < 7; k++) gl += zc[k * 15 + 1 + r] * zc[k * 15];
    }
    for (int u = t; u < 56; u += 64) {  // Z_p = [z_b | W_L]  (7 x 8)
      const int r = u / 8, c = u % 8;
      Zg[p * 56 + u] = zc[r * 15 + c];
    }
    if (t < 49) Lp[t] = Lc[t];
    if (t < 7) invp[t] = invc[t];
    for (int u = t; u < 105; u += 64) zp[u] = zc[u];
    __syncthreads();
  }
  // terms of the right border pose: W_R = z_{p1} columns 8..14 (zero above p1)
  if (t < 49) {
    const int r = t / 7, c = t % 7;
    double rr = 0.0, rl = 0.0;
#pragma unroll
    for (int k = 0; k < 7; k++) {
      rr += zp[k * 15 + 8 + r] * zp[k * 15 + 8 + c];
      rl += zp[k * 15 + 8 + r] * zp[k * 15 + 1 + c];
    }
    ws[plan[hGLL] + s * 49 + t] = gll;
    ws[plan[hGRR] + s * 49 + t] = rr;
    ws[plan[hGLR] + s * 49 + t] = rl;        // W_R^T W_L: block (qR, qL)
    ws[plan[hWR] + s * 49 + t] = zp[r * 15 + 8 + c];
  } else if (t < 56) {
    const int r = t - 49;
    double g = 0.0;
#pragma unroll
    for (int k = 0; k < 7; k++) g += zp[k * 15 + 8 + r] * zp[k * 15];
    ws[plan[hgL] + s * 7 + r] = gl;
    ws[plan[hgR] + s * 7 + r] = g;
  }
  if (t == 0 && bad) atomicOr(fail, 1);
}

// S -= segment Schur terms; grid = m (diagonal blocks, left segment first)
// + nseg (the off-diagonal block between a segment's two border poses)
__global__ void __launch_bounds__(64) pgo_border_kernel(const int64_t* __restrict__ plan,
                                                        double* __restrict__ ws) {
  const int64_t m = plan[hM], nseg = plan[hNseg];
  const int t = threadIdx.x;
  const int64_t ld = 7 * m;
  double* S = ws + plan[hS];
  double* bB = ws + plan[hBB];
  const int64_t g = blockIdx.x;
  if (g < m) {
    const int64_t* bd = plan + plan[hBorder] + g * kBordW;
    const int64_t sl = bd[1], sr = bd[2];
    if (t < 49) {
      const int r = t / 7, c = t % 7;
      double v = S[(7 * g + r) * ld + 7 * g + c];
      if (sl >= 0) v -= ws[plan[hGRR] + sl * 49 + t];
      if (sr >= 0) v -= ws[plan[hGLL] + sr * 49 + t];
      S[(7 * g + r) * ld + 7 * g + c] = v;
    } else if (t < 56) {
      const int r = t - 49;
      double v = bB[7 * g + r];
      if (sl >= 0) v -= ws[plan[hgR] + sl * 7 + r];
      if (sr >= 0) v -= ws[plan[hgL] + sr * 7 + r];
      bB[7 * g + r] = v;
    }
  } else if (g - m < nseg) {
    const int64_t s = g - m;
    const int64_t* sg = plan + plan[hSegs] + s * kSegW;
    const int64_t uL = sg[2], uR = sg[3];
    if (uL < 0 || uR < 0 || t >= 49) return;
    const int r = t / 7, c = t % 7;
    const double v = ws[plan[hGLR] + s * 49 + t];
    S[(7 * uR + r) * ld + 7 * uL + c] -= v;
    S[(7 * uL + c) * ld + 7 * uR + r] -= v;
  }
}

// x = L^-T (z - W x_border), p = p1 .. p0; xB = solved border unknowns [m][7]
__global__ void __launch_bounds__(64) pgo_segment_backward_kernel(const int64_t* __restrict__ plan,
                                                                  const double* __restrict__ xB,
                                                                  double* __restrict__ ws) {
  const int s = blockIdx.x, t = threadIdx.x;
  const int64_t* sg = plan + plan[hSegs] + (int64_t)s * kSegW;
  const int64_t p0 = sg[0], p1 = sg[1], uL = sg[2], uR = sg[3];
  const double* Lg = ws + plan[hL];
  const double* Mg = ws + plan[hMM];
  const double* Zg = ws + plan[hZ];
  double* delta = ws + plan[hDelta];
  __shared__ double xl[7], xr[7], xn[7], rhs[7];
  if (t < 7) {
    xl[t] = uL >= 0 ? xB[7 * uL + t] : 0.0;
    xr[t] = uR >= 0 ? xB[7 * uR + t] : 0.0;
    xn[t] = 0.0;
  }
  __syncthreads();
  for (int64_t p = p1; p >= p0; p--) {
    if (t < 7) {
      const double* Z = Zg + p * 56 + t * 8;
      double v = Z[0];
#pragma unroll
      for (int c = 0; c < 7; c++) v -= Z[1 + c] * xl[c];
      if (p == p1) {
        const double* W = ws + plan[hWR] + (int64_t)s * 49 + t * 7;
#pragma unroll
        for (int c = 0; c < 7; c++) v -= W[c] * xr[c];
      } else {  // - M_{p+1}^T x_{p+1}
        const double* M = Mg + (p + 1) * 49;
#pragma unroll
        for (int k = 0; k < 7; k++) v -= M[k * 7 + t] * xn[k];
      }
      rhs[t] = v;
    }
    __syncthreads();
    if (t == 0) {  // L^T x = rhs, backward
      const double* L = Lg + p * 49;
      double x[7];
#pragma unroll
      for (int r = 6; r >= 0; r--) {
        double v = rhs[r];
#pragma unroll
        for (int k = r + 1; k < 7; k++) v -= L[k * 7 + r] * x[k];
        x[r] = v / L[r * 7 + r];
      }
#pragma unroll
      for (int r = 0; r < 7; r++) {
        xn[r] = x[r];
        delta[p * 7 + r] = x[r];
      }
    }
    __syncthreads();
  }
}

}  // namespace
}  // namespace dpvo

using namespace dpvo;

// Host-side plan.  ii / jj are HOST arrays.  First call with plan == nullptr
// returns the plan length (int64 words) in *plan_len; the second fills it.
DPVO_EXPORT int dpvo_pgo_plan(const int64_t* ii, const int64_t* jj, int r, int nf, int64_t* plan,
                              int64_t plan_cap, int64_t* plan_len) {
  if (r < 0 || nf < 0 || !plan_len || (r > 0 && (!ii || !jj))) return DPVO_ERR_INVALID;
  // border poses: endpoints of long edges inside the free range
  std::vector<char> border(nf, 0);
  for (int e = 0; e < r; e++) {
    const int64_t i = ii[e], j = jj[e];
    if (i < 0 || j < 0 || i == j) return DPVO_ERR_INVALID;
    if (i < nf && j < nf && (i - j > 1 || j - i > 1)) border[i] = border[j] = 1;
  }
  std::vector<int64_t> bidx(nf, -1), B;
  for (int p = 0; p < nf; p++)
    if (border[p]) {
      bidx[p] = (int64_t)B.size();
      B.push_back(p);
    }
  const int64_t m = (int64_t)B.size();
  // segments: maximal runs of interior poses
  std::vector<int64_t> segs, seg_of(nf, -1);
  for (int p = 0; p < nf;) {
    if (border[p]) {
      p++;
      continue;
    }
    int q = p;
    while (q + 1 < nf && !border[q + 1]) q++;
    const int64_t s = (int64_t)segs.size() / kSegW;
    segs.push_back(p);
    segs.push_back(q);
    segs.push_back(p > 0 ? bidx[p - 1] : -1);
    segs.push_back(q + 1 < nf ? bidx[q + 1] : -1);
    for (int x = p; x <= q; x++) seg_of[x] = s;
    p = q + 1;
  }
  const int64_t nseg = (int64_t)segs.size() / kSegW;
  std::vector<int64_t> bord;
  for (int64_t u = 0; u < m; u++) {
    const int64_t p = B[u];
    bord.push_back(p);
    bord.push_back(p > 0 && !border[p - 1] ? seg_of[p - 1] : -1);
    bord.push_back(p + 1 < nf && !border[p + 1] ? seg_of[p + 1] : -1);
  }
  // workspace offsets (doubles)
  int64_t hdr[hCount] = {0};
  int64_t w = 0;
  auto take = [&](int slot, int64_t n) {
    hdr[slot] = w;
    w += (n + 1) & ~(int64_t)1;
  };
  take(hD, 49LL * nf);
  take(hE, 49LL * nf);
  take(hB, 7LL * nf);
  take(hL, 49LL * nf);
  take(hMM, 49LL * nf);
  take(hZ, 56LL * nf);
  take(hCL, 49 * nseg);
  take(hCR, 49 * nseg);
  take(hWR, 49 * nseg);
  take(hGLL, 49 * nseg);
  take(hGLR, 49 * nseg);
  take(hGRR, 49 * nseg);
  take(hgL, 7 * nseg);
  take(hgR, 7 * nseg);
  take(hS, 49 * m * m);
  take(hBB, 7 * m);
  take(hDelta, 7LL * nf);
  hdr[hWs] = w;
  // block tasks: diagonal of every free pose (edges touching it, ascending),
  // then the distinct off-diagonal pairs inside the free range
  std::vector<std::pair<int64_t, int64_t>> dk;   // (pose, edge)
  std::vector<std::pair<std::pair<int64_t, int64_t>, int64_t>> ok;  // ((hi, lo), edge)
  for (int e = 0; e < r; e++) {
    const int64_t i = ii[e], j = jj[e];
    if (i < nf) dk.push_back({i, e});
    if (j < nf) dk.push_back({j, e});
    if (i < nf && j < nf) ok.push_back({{std::max(i, j), std::min(i, j)}, e});
  }
  std::sort(dk.begin(), dk.end());
  std::sort(ok.begin(), ok.end());
  std::vector<int64_t> tasks, contrib;
  const int64_t ld = 7 * m;
  auto sblk = [&](int64_t u, int64_t v) { return hdr[hS] + (7 * u) * ld + 7 * v; };
  size_t x = 0;
  for (int64_t p = 0; p < nf; p++) {
    const int64_t c0 = (int64_t)contrib.size();
    while (x < dk.size() && dk[x].first == p) contrib.push_back(dk[x++].second);
    const int64_t c1 = (int64_t)contrib.size();
    if (border[p]) {
      const int64_t u = bidx[p];
      tasks.insert(tasks.end(), {p, p, c0, c1, sblk(u, u), ld, -1, hdr[hBB] + 7 * u});
    } else {
      tasks.insert(tasks.end(), {p, p, c0, c1, hdr[hD] + 49 * p, 7, -1, hdr[hB] + 7 * p});
    }
  }
  for (size_t y = 0; y < ok.size();) {
    const int64_t hi = ok[y].first.first, lo = ok[y].first.second;
    const int64_t c0 = (int64_t)contrib.size();
    while (y < ok.size() && ok[y].first.first == hi && ok[y].first.second == lo)
      contrib.push_back(ok[y++].second);
    const int64_t c1 = (int64_t)contrib.size();
    if (!border[hi] && !border[lo]) {  // chain block inside a segment: E_hi = A(hi, lo)
      tasks.insert(tasks.end(), {hi, lo, c0, c1, hdr[hE] + 49 * hi, 7, -1, -1});
    } else if (!border[hi]) {  // hi = p0 of its segment, lo = its left border pose
      tasks.insert(tasks.end(), {hi, lo, c0, c1, hdr[hCL] + 49 * seg_of[hi], 7, -1, -1});
    } else if (!border[lo]) {  // lo = p1 of its segment, hi = its right border pose
      tasks.insert(tasks.end(), {lo, hi, c0, c1, hdr[hCR] + 49 * seg_of[lo], 7, -1, -1});
    } else {
      tasks.insert(tasks.end(),
                   {hi, lo, c0, c1, sblk(bidx[hi], bidx[lo]), ld, sblk(bidx[lo], bidx[hi]), -1});
    }
  }
  const int64_t ntask = (int64_t)tasks.size() / kTaskW;
  hdr[hNf] = nf;
  hdr[hNtask] = ntask;
  hdr[hNseg] = nseg;
  hdr[hM] = m;
  hdr[hTasks] = hCount;
  hdr[hContrib] = hdr[hTasks] + (int64_t)tasks.size();
  hdr[hSegs] = hdr[hContrib] + (int64_t)contrib.size();
  hdr[hBorder] = hdr[hSegs] + (int64_t)segs.size();
  const int64_t len = hdr[hBorder] + (int64_t)bord.size();
  *plan_len = len;
  if (!plan) return DPVO_OK;
  if (plan_cap < len) return DPVO_ERR_INVALID;
  int64_t* o = plan;
  for (int k = 0; k < hCount; k++) *o++ = hdr[k];
  for (int64_t v : tasks) *o++ = v;
  for (int64_t v : contrib) *o++ = v;
  for (int64_t v : segs) *o++ = v;
  for (int64_t v : bord) *o++ = v;
  return DPVO_OK;
}

// Phases 1-2 (after the plan is on the device): zero the workspace, assemble
// every block, factor the segments and scatter their Schur terms into the
// border system.  hdr = the plan's header, read on the host.
DPVO_EXPORT int dpvo_pgo_factor(const float* J_Ginv_i, const float* J_Ginv_j, const int64_t* ii,
                                const float* res, const int64_t* plan, const int64_t* hdr,
                                float ep, float lm, double* ws, int* fail, void* stream_) {
  hipStream_t stream = (hipStream_t)stream_;
  if (!plan || !hdr || !ws || !fail) return DPVO_ERR_INVALID;
  if (hipMemsetAsync(ws, 0, sizeof(double) * hdr[hWs], stream) != hipSuccess ||
      hipMemsetAsync(fail, 0, sizeof(int), stream) != hipSuccess)
    return DPVO_ERR_LAUNCH;
  if (hdr[hNtask] > 0)
    hipLaunchKernelGGL(pgo_block_kernel, dim3((unsigned)hdr[hNtask]), dim3(64), 0, stream,
                       J_Ginv_i, J_Ginv_j, ii, res, plan, (double)ep, (double)lm, ws);
  if (hdr[hNseg] > 0)
    hipLaunchKernelGGL(pgo_segment_forward_kernel, dim3((unsigned)hdr[hNseg]), dim3(64), 0,
                       stream, plan, ws, fail);
  if (hdr[hM] > 0)
    hipLaunchKernelGGL(pgo_border_kernel, dim3((unsigned)(hdr[hM] + hdr[hNseg])), dim3(64), 0,
                       stream, plan, ws);
  return launch_status();
}

// Phase 4: back-substitution of the segments given the border solution
// xB [m][7] (ignored when m == 0); the step of pose p < nf lands in
// ws[hdr[hDelta] + 7 p ..] (border poses are written by the caller).
DPVO_EXPORT int dpvo_pgo_back(const int64_t* plan, const int64_t* hdr, const double* xB,
                              double* ws, void* stream_) {
  if (!plan || !hdr || !ws) return DPVO_ERR_INVALID;
  if (hdr[hNseg] > 0)
    hipLaunchKernelGGL(pgo_segment_backward_kernel, dim3((unsigned)hdr[hNseg]), dim3(64), 0,
                       (hipStream_t)stream_, plan, xB, ws);
  return launch_status();
}
