// ba_blocks.hip -- F-BA with one persistent workgroup per lower 6x6 block of
// the pose Schur complement S (the default path for DPVO-sized windows).
//
// Reference semantics: dpvo/fastba/ba_cuda.cu:433-582 with the block-sparse
// Schur complement of block_e.cu:188-300 (see ba.hip / ba_fused.hip):
//   per edge: residual + Jacobians in fp32 (ba_cuda.cu:265-333)
//   B, E, C, v, u (:339-373); Q = 1/(C + lmbda) (:519)
//   S = B - E Q E^T, y = v - E Q u (:554-558), S += I (1e-4 S + 1) (:560)
//   dX = chol_solve(S, y) (:561-562), dZ = Q (u - E^T dX) (:563)
//   pose_retr_kernel (:178-206), patch_retr_kernel (:209-229).
//
// MI355X design (DESIGN.md "F-BA").  A DPVO window is latency-bound: ~2 k
// edges, N <= 16 free poses, a 6N x 6N dense solve.  One CU cannot issue the
// ~2.5 M lane-ops of linearisation + fp64 assembly per iteration in less than
// ~12 us, and summing per-CU partial S matrices costs a cross-XCD transfer per
// partial.  So:
//   * workgroup g owns lower block (a, b) of S (g = a(a+1)/2 + b).  At setup it
//     sorts the edge list itself (counting sort in LDS, redundantly in every
//     workgroup -- no cross-CU handoff) and keeps the patches whose E column
//     touches both a and b ("relevant"), with their edges, targets and
//     weights, in LDS.
//   * per iteration it re-linearises only those edges (thread per patch) and
//     accumulates its block -- B terms of its pose pair and -Q E_u[a] E_u[b]^T
//     -- in 42 fp64 registers per thread (no atomics), reduces them in a fixed
//     order and stores 288 bytes.  No partial sums exist, so the gather is one
//     19 KB read.
//   * workgroup 0 waits for every block (one release/acquire handoff), runs
//     the block LDL^T solve and publishes dX; every workgroup then applies the
//     same pose retraction and the inverse-depth update of its own relevant
//     patches (identical inputs -> identical bits: no depth exchange), and the
//     next iteration starts.  The owner of a patch (the diagonal workgroup of
//     its lowest free pose) writes its final inverse depth.
//   All spin-waits carry a wall-clock timeout so the grid always drains.
// The grid (<= 136 workgroups of 512 threads) is far below one workgroup per
// CU, so all workgroups are co-resident.
#include <map>
#include <mutex>
#include <utility>

#include "ba_device.hpp"

namespace dpvo {
namespace {
using namespace bad;

constexpr int kBT = 256;  // 1 wave per SIMD: 512 registers, no spills
constexpr int kBMaxN = 16;
constexpr int kBMaxE = 2048;
constexpr int kBRE = kBMaxE / kBT;  // edges per thread in the setup
constexpr int kSlots = 64;          // LDS pose table
constexpr int kBLds = 160 * 1024;
constexpr unsigned kFixed = 0xFF;   // free code of a fixed pose
constexpr unsigned kGlb = 0xFE;     // pose slot: read from HBM
constexpr int kV = 42;              // per-thread block accumulators: 36 S + 6 y
constexpr int kRedCols = 128;
constexpr long long kSpinTicks = 2000000;  // 20 ms of the 100 MHz wall clock
constexpr int kEpochWord = 2 * (kBMaxN * (kBMaxN + 1) / 2) + 4;  // in the flag buffer

struct BArgs {
  float* poses;
  float* patches;
  const float* intrinsics;
  const float* target;
  const float* weight;
  const float* lmbda;
  const int64_t* ii;
  const int64_t* jj;
  const int64_t* kk;
  int E, P, num_poses, num_patches, t0, N, iters, NB;
  double* Sg;      // [NB][2][36] the two halves of every block of S
  double* yg;      // [2][6N]
  double* dXg;     // [2][6N] dX of iteration it in slot it & 1
  long long* flags;  // persistent [G + 1]: arrival of workgroup g, [G] dX published
  long long epoch;   // unused on the host side (read on the device from flags[kEpochWord])
  double* EW;      // [2 NB][E][12] entries e_j, e_i of each relevant edge (per workgroup)
  double* QU;      // [NB][E][2]  Q, u of each relevant patch
  int* gidx;       // [NB][E][2]  pose indices of relevant edges (slot kGlb)
  int* kxw;        // [NB][E]     patch id of each relevant patch, -1 if not owned
  float* dbw;      // [NB][E]     first-iteration retraction base [2][0][0]
  int* meta;       // [8] [0] nuniq, [1] status
  int refine;      // solve mode: 0 fp32 Cholesky, 1 + fp64 refinement, 2 fp64 block LDL^T
  int64_t* marks;  // [64] wall-clock stamps of workgroup 0 (may be null)
};

struct BL {
  int* ctl;                // [64]
  float* pose;             // [kSlots][8]
  double* dX;              // [6N]
  unsigned short* roff;    // [nrel + 1] first relevant edge of each relevant patch
  float2* nxy;             // [nrel] normalised patch centre
  float* dep;              // [nrel] inverse depth
  unsigned short* pc;      // [nrp] pose slot of ii | slot of jj << 8
  float4* tw;              // [nrp] target, weight
  unsigned short* rpat;    // [nrp] relevant patch of each relevant edge
  char* scratch;           // reduction table / solver (workgroup 0)
  double* pe;              // [nrp][14] per edge: c, u, e_j[6], e_i[6] (null: HBM fallback)
  double2* pq;             // [nrel] Q, u per patch
};

enum { kCNrel = 0, kCNrp = 1, kCNuniq = 2, kCKmin = 3, kCKmax = 4, kCFmin = 5, kCBad = 6,
       kCFail = 7, kCGo = 8, kCTimeout = 9, kCScan = 16 };

__device__ __forceinline__ size_t al16(size_t v) { return (v + 15) & ~(size_t)15; }
__device__ __forceinline__ unsigned code_of(unsigned slot, int N) {
  return slot < (unsigned)N ? slot : kFixed;
}

// spin until *p >= target; returns false on timeout
__device__ bool wait_geq(long long* p, long long target) {
  const long long t0 = (long long)wall_clock64();
  while (__hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
    __builtin_amdgcn_s_sleep(1);
    if ((long long)wall_clock64() - t0 > kSpinTicks) return false;
  }
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  return true;
}

__device__ __forceinline__ void bstamp(const BArgs& A, int slot) {
  if (A.marks && blockIdx.x == 0 && threadIdx.x == 0) A.marks[slot] = (int64_t)wall_clock64();
}

// ---------------------------------------------------------------------------
// fp64 block LDL^T solve of the damped S (workgroup 0; solve mode 2).  S: lower blocks in LDS.
// ---------------------------------------------------------------------------
struct Solver {
  double* S;    // [NB][36]
  double* y;    // [6N]
  double* piv;  // [N][36]
  double* wv;   // [6N]
  double* tt;   // [6N]
  double* PV;   // [N][36]
};

__device__ void block_ldl_solve(const Solver& L, int N, double* dX, int* fail, int64_t* marks) {
  const int tid = threadIdx.x, T = blockDim.x, wid = tid >> 6, lane = tid & 63;
  if (tid == 0 && !ldl6(L.S, L.y, L.piv, L.wv)) *fail = 1;
  __syncthreads();
  // step k: P1  W_i = S_ik L_k^-T (into S_ik), V_i = W_i D_k^-1, y_i -= V_i w_k  (i > k)
  //         P2  S_ij -= V_i W_j^T (k < j <= i).  Wave 0 updates the next pivot block
  //         (k+1, k+1) and factors it while waves 1.. update the rest (look-ahead).
  for (int k = 0; k < N; k++) {
    const int m = N - 1 - k;
    const double* pk = L.piv + 36 * k;
    for (int t = tid; t < 6 * m; t += T) {
      const int i = k + 1 + t / 6, x = t % 6;
      double* Sik = L.S + 36 * lblk(i, k) + 6 * x;
      double W[6], V[6];
#pragma unroll
      for (int q = 0; q < 6; q++) {
        double s = Sik[q];
#pragma unroll
        for (int pq = 0; pq < q; pq++) s -= W[pq] * pk[6 * q + pq];
        W[q] = s;
        V[q] = s * pk[7 * q];
      }
      double yv = L.y[6 * i + x];
#pragma unroll
      for (int q = 0; q < 6; q++) {
        Sik[q] = W[q];
        L.PV[36 * i + 6 * x + q] = V[q];
        yv -= V[q] * L.wv[6 * k + q];
      }
      L.y[6 * i + x] = yv;
    }
    __syncthreads();
    if (m == 0) break;
    const int ntask = 6 * (m * (m + 1) / 2);
    if (wid == 0) {
      // look-ahead: pivot block (k+1, k+1), one entry per lane (36 lanes)
      if (lane < 36) {
        const int x = lane / 6, z = lane % 6, i = k + 1;
        const double* Vi = L.PV + 36 * i + 6 * x;
        const double* Wz = L.S + 36 * lblk(i, k) + 6 * z;
        double* Sxz = L.S + 36 * lblk(i, i) + 6 * x + z;
        double s = *Sxz;
#pragma unroll
        for (int q = 0; q < 6; q++) s -= Vi[q] * Wz[q];
        *Sxz = s;
      }
    } else {
      // tasks 6.. (rows of the other trailing blocks) on waves 1..
      for (int t = 6 + (tid - 64); t < ntask; t += T - 64) {
        const int x = t % 6;
        int a, b;
        tri_of(t / 6, a, b);
        const int i = k + 1 + a, j = k + 1 + b;
        const double* Vi = L.PV + 36 * i + 6 * x;
        const double* Wj = L.S + 36 * lblk(j, k);
        double* Sij = L.S + 36 * lblk(i, j) + 6 * x;
        double v[6], w[36];
#pragma unroll
        for (int q = 0; q < 6; q++) v[q] = Vi[q];
#pragma unroll
        for (int q = 0; q < 36; q += 2) {
          const double2 p2 = *reinterpret_cast<const double2*>(Wj + q);
          w[q] = p2.x;
          w[q + 1] = p2.y;
        }
#pragma unroll
        for (int z = 0; z < 6; z++) {  // diagonal blocks stay full (symmetric)
          double s = Sij[z];
#pragma unroll
          for (int q = 0; q < 6; q++) s -= v[q] * w[6 * z + q];
          Sij[z] = s;
        }
      }
    }
    if (wid == 0) {
      wave_lds_sync();
      if (tid == 0 && !ldl6(L.S + 36 * lblk(k + 1, k + 1), L.y + 6 * (k + 1), L.piv + 36 * (k + 1),
                            L.wv + 6 * (k + 1)))
        *fail = 1;
    }
    __syncthreads();
  }
  if (marks && threadIdx.x == 0) marks[4] = (int64_t)wall_clock64();
  // back substitution by wave 0 alone (no workgroup barriers):
  //   x_i = L_i^-T D_i^-1 t_i,  t_k -= W_ik^T x_i (k < i),  t = w initially
  if (wid == 0) {
    for (int k = lane; k < 6 * N; k += 64) L.tt[k] = L.wv[k];
    wave_lds_sync();
    for (int i = N - 1; i >= 0; i--) {
      const double* pi_ = L.piv + 36 * i;
      double xi[6];
#pragma unroll
      for (int q = 5; q >= 0; q--) {
        double s = L.tt[6 * i + q] * pi_[7 * q];
#pragma unroll
        for (int pq = q + 1; pq < 6; pq++) s -= pi_[6 * pq + q] * xi[pq];
        xi[q] = s;
      }
#pragma unroll
      for (int q = 0; q < 6; q++)
        if (lane == q) dX[6 * i + q] = xi[q];
      for (int t = lane; t < 6 * i; t += 64) {
        const int k = t / 6, x = t % 6;
        const double* Wik = L.S + 36 * lblk(i, k);
        double s = L.tt[6 * k + x];
#pragma unroll
        for (int q = 0; q < 6; q++) s -= Wik[6 * q + x] * xi[q];
        L.tt[6 * k + x] = s;
      }
      wave_lds_sync();
    }
  }
  __syncthreads();
}

// ---------------------------------------------------------------------------
// per-iteration assembly of block (ba, bb): thread per relevant patch,
// re-linearise its edges, accumulate in registers, reduce in a fixed order,
// store the block (+ y_ba) and arrive.  MODE 0: no free pose (N == 0: only
// Q, u for the inverse depths); 1: diagonal block (lower triangle + y);
// 2: off-diagonal block.
// ---------------------------------------------------------------------------
struct Ctx {
  const BArgs& A;
  const BL& L;
  double* EW;
  double* QU;
  const int* gidx;
  double* red;
  int nrel, ba, bb, g, it;
  double lam;
  float fx, fy, cx, cy;
};

// linearise relevant edge q: entries (e_j at jj, e_i at ii), c = sum w Jz^2,
// u = sum w r Jz (ba_cuda.cu:352-373) and this block's B terms into acc
template <int MODE, int NA>
__device__ __forceinline__ void edge_terms(const Ctx& c, int q, float2 nxy, float dp, double* acc,
                                           double& cq, double& uq, double* ej, double* ei) {
  const BArgs& A = c.A;
  const BL& L = c.L;
  const int N = A.N;
  const unsigned ba = (unsigned)c.ba, bb = (unsigned)c.bb;
  const unsigned b = L.pc[q];
  const unsigned si = b & 0xff, sj = b >> 8;
  const unsigned ci = code_of(si, N), cj = code_of(sj, N);
  const float4 tw = L.tw[q];
  float Pi[7], Pj[7];
  if (si != kGlb) {
    const float4 a0 = *reinterpret_cast<const float4*>(L.pose + 8 * si);
    const float4 a1 = *reinterpret_cast<const float4*>(L.pose + 8 * si + 4);
    Pi[0] = a0.x; Pi[1] = a0.y; Pi[2] = a0.z; Pi[3] = a0.w; Pi[4] = a1.x; Pi[5] = a1.y; Pi[6] = a1.z;
  } else {
    const float* g = A.poses + 7 * (size_t)c.gidx[2 * q];
#pragma unroll
    for (int k = 0; k < 7; k++) Pi[k] = g[k];
  }
  if (sj != kGlb) {
    const float4 a0 = *reinterpret_cast<const float4*>(L.pose + 8 * sj);
    const float4 a1 = *reinterpret_cast<const float4*>(L.pose + 8 * sj + 4);
    Pj[0] = a0.x; Pj[1] = a0.y; Pj[2] = a0.z; Pj[3] = a0.w; Pj[4] = a1.x; Pj[5] = a1.y; Pj[6] = a1.z;
  } else {
    const float* g = A.poses + 7 * (size_t)c.gidx[2 * q + 1];
#pragma unroll
    for (int k = 0; k < 7; k++) Pj[k] = g[k];
  }
  Lin o;
  lin_edge(Pi, Pj, nxy.x, nxy.y, dp, tw.x, tw.y, tw.z, tw.w, c.fx, c.fy, c.cx, c.cy, o);
  cq = 0.0;
  uq = 0.0;
#pragma unroll
  for (int k = 0; k < 6; k++) ej[k] = ei[k] = 0.0;
#pragma unroll
  for (int row = 0; row < 2; row++) {
    const double wr = o.w[row];
    const double wz = wr * (double)o.Jz[row];
#pragma unroll
    for (int k = 0; k < 6; k++) {
      ej[k] += wz * (double)o.Jj[row][k];
      ei[k] -= wz * (double)o.Ji[row][k];
    }
    cq += wz * (double)o.Jz[row];
    uq += (wr * (double)o.r[row]) * (double)o.Jz[row];
  }
  if (MODE == 0) return;
  // B terms of this block as one rank-1 update per residual row
  // (ba_cuda.cu:339-350; v :352-370).  Diagonal (ba, ba): u = [ii==ba] Ji -
  // [jj==ba] Jj gives Ji Ji^T, Jj Jj^T and -(Ji Jj^T + Jj Ji^T) of a self
  // edge in one product; v_ba -= w r u.  Off-diagonal (ba > bb): rows follow
  // ba, -w Ji Jj^T (ii == ba, jj == bb) or -w Jj Ji^T (jj == ba, ii == bb).
  const bool ia = ci == ba, ja = cj == ba, ib = ci == bb, jb = cj == bb;
  const bool hit = (MODE == 1) ? (ia || ja) : ((ia && jb) || (ja && ib));
  if (!hit) return;
#pragma unroll
  for (int row = 0; row < 2; row++) {
    double Rv[6], Cv[6];
#pragma unroll
    for (int k = 0; k < 6; k++) {
      const double ji = o.Ji[row][k], jv = o.Jj[row][k];
      if (MODE == 1) {
        Rv[k] = (ia ? ji : 0.0) - (ja ? jv : 0.0);
        Cv[k] = Rv[k];
      } else {
        Rv[k] = ia ? ji : jv;
        Cv[k] = ia ? jv : ji;
      }
    }
    const double wr = o.w[row];
    const double coef = (MODE == 1) ? wr : -wr;
    int k = 0;
#pragma unroll
    for (int x = 0; x < 6; x++) {
      const double t = coef * Rv[x];
      if (MODE == 1) {
#pragma unroll
        for (int z = 0; z <= x; z++) acc[k++] += t * Cv[z];
      } else {
#pragma unroll
        for (int z = 0; z < 6; z++) acc[6 * x + z] += t * Cv[z];
      }
    }
    if (MODE == 1) {
      const double wrr = wr * (double)o.r[row];
#pragma unroll
      for (int x = 0; x < 6; x++) acc[21 + x] -= wrr * Rv[x];
    }
  }
}

// Schur terms of patch ri from its Q, u and E entries at ba / bb (:554-558)
template <int MODE, int NA>
__device__ __forceinline__ void patch_terms(double Q, double U, const double* Ea, const double* Eb,
                                            double* acc) {
  if (MODE == 1) {
    int k = 0;
#pragma unroll
    for (int x = 0; x < 6; x++) {
      const double qa = Q * Ea[x];
#pragma unroll
      for (int z = 0; z <= x; z++) acc[k++] -= qa * Ea[z];
      acc[21 + x] -= (Q * U) * Ea[x];
    }
  } else if (MODE == 2) {
#pragma unroll
    for (int x = 0; x < 6; x++) {
      const double qa = Q * Ea[x];
#pragma unroll
      for (int z = 0; z < 6; z++) acc[6 * x + z] -= qa * Eb[z];
    }
  }
}

template <int MODE>
__device__ void assemble(const Ctx& c) {
  constexpr int NA = (MODE == 1) ? 27 : (MODE == 2 ? 36 : 1);  // accumulators
  const BArgs& A = c.A;
  const BL& L = c.L;
  const int tid = threadIdx.x, T = kBT, N = A.N;
  const unsigned ba = (unsigned)c.ba, bb = (unsigned)c.bb;
  const int nrp = L.roff[c.nrel];
  double acc[NA];
#pragma unroll
  for (int k = 0; k < NA; k++) acc[k] = 0.0;
  if (L.pe) {
    // pass 1: thread per relevant edge (balanced), entries kept in LDS
    for (int q = tid; q < nrp; q += T) {
      const int ri = L.rpat[q];
      double cq, uq, ej[6], ei[6];
      edge_terms<MODE, NA>(c, q, L.nxy[ri], L.dep[ri], acc, cq, uq, ej, ei);
      double2* pe = reinterpret_cast<double2*>(L.pe + 14 * (size_t)q);
      pe[0] = make_double2(cq, uq);
#pragma unroll
      for (int k = 0; k < 3; k++) {
        pe[1 + k] = make_double2(ej[2 * k], ej[2 * k + 1]);
        pe[4 + k] = make_double2(ei[2 * k], ei[2 * k + 1]);
      }
    }
    __syncthreads();
    // pass 2: thread per relevant patch: C, u, E_u[ba], E_u[bb] in edge order
    for (int ri = tid; ri < c.nrel; ri += T) {
      double C = 0.0, U = 0.0, Ea[6] = {0, 0, 0, 0, 0, 0}, Eb[6] = {0, 0, 0, 0, 0, 0};
      for (int q = L.roff[ri]; q < L.roff[ri + 1]; q++) {
        const double* pe = L.pe + 14 * (size_t)q;
        const unsigned b = L.pc[q];
        const unsigned ci = code_of(b & 0xff, N), cj = code_of(b >> 8, N);
        C += pe[0];
        U += pe[1];
        if (MODE != 0) {
#pragma unroll
          for (int k = 0; k < 6; k++) {
            Ea[k] += ((cj == ba) ? pe[2 + k] : 0.0) + ((ci == ba) ? pe[8 + k] : 0.0);
            if (MODE == 2) Eb[k] += ((cj == bb) ? pe[2 + k] : 0.0) + ((ci == bb) ? pe[8 + k] : 0.0);
          }
        }
      }
      const double Q = 1.0 / (C + c.lam);  // (:519)
      L.pq[ri] = make_double2(Q, U);
      patch_terms<MODE, NA>(Q, U, Ea, Eb, acc);
    }
  } else {
    // HBM fallback: thread per patch, entries to the per-workgroup scratch
    for (int ri = tid; ri < c.nrel; ri += T) {
      const float2 nxy = L.nxy[ri];
      const float dp = L.dep[ri];
      double C = 0.0, U = 0.0, Ea[6] = {0, 0, 0, 0, 0, 0}, Eb[6] = {0, 0, 0, 0, 0, 0};
      for (int q = L.roff[ri]; q < L.roff[ri + 1]; q++) {
        double cq, uq, ej[6], ei[6];
        edge_terms<MODE, NA>(c, q, nxy, dp, acc, cq, uq, ej, ei);
        const unsigned b = L.pc[q];
        const unsigned ci = code_of(b & 0xff, N), cj = code_of(b >> 8, N);
        C += cq;
        U += uq;
        double2* out = reinterpret_cast<double2*>(c.EW + 12 * (size_t)q);
#pragma unroll
        for (int k = 0; k < 3; k++) {
          out[k] = make_double2(ej[2 * k], ej[2 * k + 1]);
          out[3 + k] = make_double2(ei[2 * k], ei[2 * k + 1]);
        }
        if (MODE != 0) {
#pragma unroll
          for (int k = 0; k < 6; k++) {
            Ea[k] += ((cj == ba) ? ej[k] : 0.0) + ((ci == ba) ? ei[k] : 0.0);
            if (MODE == 2) Eb[k] += ((cj == bb) ? ej[k] : 0.0) + ((ci == bb) ? ei[k] : 0.0);
          }
        }
      }
      const double Q = 1.0 / (C + c.lam);  // (:519)
      reinterpret_cast<double2*>(c.QU)[ri] = make_double2(Q, U);
      patch_terms<MODE, NA>(Q, U, Ea, Eb, acc);
    }
  }
  if (c.g == 0) bstamp(A, 2 + 8 * c.it + 0);
  if (MODE == 0) return;
  // ---- fixed-order reduction: rows of kRedCols threads, then 8 segments ----
  double* red = c.red;
  const int nact = min(max(c.nrel, L.pe ? nrp : 0), T);
  const int rounds = (nact + kRedCols - 1) / kRedCols;
  for (int rd = 0; rd < rounds; rd++) {
    if (tid >= rd * kRedCols && tid < (rd + 1) * kRedCols) {
      const int col = tid - rd * kRedCols;
#pragma unroll
      for (int v = 0; v < NA; v++) {
        const double x = (tid < nact) ? acc[v] : 0.0;
        red[v * kRedCols + col] = (rd == 0) ? x : red[v * kRedCols + col] + x;
      }
    }
    __syncthreads();
  }
  double* part = red + kV * kRedCols;
  const int cols = rounds > 0 ? kRedCols : 0;
  for (int t = tid; t < NA * 8; t += T) {
    const int v = t >> 3, sg = t & 7;
    double s = 0.0;
    for (int cc = sg * (kRedCols / 8); cc < (sg + 1) * (kRedCols / 8) && cc < cols; cc++)
      s += red[v * kRedCols + cc];
    part[t] = s;
  }
  __syncthreads();
  if (tid < NA) {
    double s = 0.0;
#pragma unroll
    for (int sg = 0; sg < 8; sg++) s += part[tid * 8 + sg];
    if (MODE == 2) {
      A.Sg[36 * c.g + tid] = s;  // partial block of this half: Sg[2 blk + sub]
    } else if (tid < 21) {  // lower triangle -> full symmetric block
      int x = 0;
      while ((x + 1) * (x + 2) / 2 <= tid) x++;
      const int z = tid - x * (x + 1) / 2;
      A.Sg[36 * c.g + 6 * x + z] = s;
      A.Sg[36 * c.g + 6 * z + x] = s;
    } else {
      A.yg[6 * (A.N * (c.g & 1) + c.ba) + tid - 21] = s;
    }
  }
  __syncthreads();
  if (tid == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    __hip_atomic_store(&A.flags[c.g], A.epoch * 64 + c.it + 1, __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
  }
}

// ---------------------------------------------------------------------------
// the kernel
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(kBT) ba_blocks_kernel(BArgs A) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  const int tid = threadIdx.x, T = kBT, lane = tid & 63;
  const int g = blockIdx.x;  // workgroup g: half (g & 1) of the patches of block g >> 1
  const int blk = g >> 1, sub = g & 1;
  const int E = A.E, N = A.N, t0 = A.t0, P = A.P, PP = P * P;
  const int NB = A.NB;
  int ba = 0, bb = 0;
  if (NB > 0) tri_of(blk, ba, bb);
  const bool diag = (ba == bb);
  const float fx = A.intrinsics[0], fy = A.intrinsics[1], cx = A.intrinsics[2],
              cy = A.intrinsics[3];
  const int kmaxc = A.num_patches - 1;
  // this call's tag: read by every workgroup at start, advanced by workgroup 0
  // at its very end (after every workgroup has read it: they all arrive in
  // iteration 0 first), so graph replays get fresh tags too
  BArgs& Am = const_cast<BArgs&>(A);
  Am.epoch = __hip_atomic_load(&A.flags[kEpochWord], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1;
  double* EW = A.EW + (size_t)g * E * 12;
  double* QU = A.QU + (size_t)g * E * 2;
  int* gidx = A.gidx + (size_t)g * E * 2;
  int* kxw = A.kxw + (size_t)g * E;
  float* dbw = A.dbw + (size_t)g * E;

  BL L;
  L.ctl = (int*)lds;
  int* ctl = L.ctl;
  int* scr = ctl + kCScan;
  L.pose = (float*)(lds + 256);
  L.dX = (double*)(lds + 256 + sizeof(float) * 8 * kSlots);
  const size_t head_end = al16(256 + sizeof(float) * 8 * kSlots + sizeof(double) * 6 * kBMaxN);
  bstamp(A, 0);

  // ============================ setup ============================
  int ekv[kBRE], egi[kBRE], egj[kBRE];
  float4 etw[kBRE];
  {
    int lmin = 0x7fffffff, lmax = -1, bad = 0, fmin = 0x7fffffff;
#pragma unroll
    for (int r = 0; r < kBRE; r++) {
      const int e = tid + r * T;
      ekv[r] = 0;
      egi[r] = egj[r] = 0;
      etw[r] = make_float4(0.f, 0.f, 0.f, 0.f);
      if (e < E) {
        int64_t v = A.kk[e];
        if (v < 0 || v > kmaxc) {
          bad = 1;
          v = v < 0 ? 0 : kmaxc;
        }
        ekv[r] = (int)v;
        const int64_t gi = A.ii[e], gj = A.jj[e];
        const bool fi = gi >= t0 && gi < t0 + N, fj = gj >= t0 && gj < t0 + N;
        egi[r] = fi ? (int)gi : (int)min(max(gi, (int64_t)0), (int64_t)A.num_poses - 1);
        egj[r] = fj ? (int)gj : (int)min(max(gj, (int64_t)0), (int64_t)A.num_poses - 1);
        if (!fi) fmin = min(fmin, egi[r]);
        if (!fj) fmin = min(fmin, egj[r]);
        const float2 tg = reinterpret_cast<const float2*>(A.target)[e];
        const float2 wt = reinterpret_cast<const float2*>(A.weight)[e];
        etw[r] = make_float4(tg.x, tg.y, wt.x, wt.y);
        lmin = min(lmin, ekv[r]);
        lmax = max(lmax, ekv[r]);
      }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      lmin = min(lmin, __shfl_xor(lmin, o, 64));
      lmax = max(lmax, __shfl_xor(lmax, o, 64));
      fmin = min(fmin, __shfl_xor(fmin, o, 64));
      bad |= __shfl_xor(bad, o, 64);
    }
    if (tid == 0) {
      ctl[kCKmin] = 0x7fffffff;
      ctl[kCKmax] = -1;
      ctl[kCFmin] = 0x7fffffff;
      ctl[kCBad] = 0;
      ctl[kCFail] = 0;
      ctl[kCTimeout] = 0;
    }
    __syncthreads();
    if (lane == 0) {
      atomicMin(&ctl[kCKmin], lmin);
      atomicMax(&ctl[kCKmax], lmax);
      atomicMin(&ctl[kCFmin], fmin);
      atomicOr(&ctl[kCBad], bad);
    }
    __syncthreads();
  }
  const int kmin = ctl[kCKmin], R = ctl[kCKmax] - kmin + 1, fmin = ctl[kCFmin];
  bstamp(A, 40);
  auto slot_of = [&](int gp) -> unsigned {
    if (gp >= t0 && gp < t0 + N) return (unsigned)(gp - t0);
    const int k = gp - fmin;
    return (k >= 0 && k < kSlots - N) ? (unsigned)(N + k) : kGlb;
  };
  // setup temporaries from the top of LDS down
  char* top = lds + kBLds;
  int* spos = (int*)(top - sizeof(int) * kBMaxE);          // key (jj << 16 | edge) per position
  int* ehead = spos - kBMaxE;                               // head flags -> scan
  int* epos = ehead - kBMaxE;                               // position of each edge
  unsigned* pmask = (unsigned*)(epos - kBMaxE);             // free-pose mask per patch
  int* ridx = (int*)pmask - kBMaxE;                         // relevant index per patch (-1)
  int* poff = ridx - (kBMaxE + 1);                          // first position of each patch
  int* ppat = poff - kBMaxE;                                // patch of each position
  char* tmp_low = (char*)ppat;
  // S2: sort edges by (kk, jj, edge)
  {
    const size_t hist_room = (size_t)(tmp_low - (lds + head_end)) / sizeof(int);
    if ((size_t)R + (size_t)(kBMaxE * 32 / 4) <= hist_room && R <= 16384) {
      int* hist = (int*)tmp_low - R;
      for (int v = tid; v < R; v += T) hist[v] = 0;
      __syncthreads();
#pragma unroll
      for (int r = 0; r < kBRE; r++)
        if (tid + r * T < E) atomicAdd(&hist[ekv[r] - kmin], 1);
      __syncthreads();
      fscan(hist, R, scr);
#pragma unroll
      for (int r = 0; r < kBRE; r++) {
        const int e = tid + r * T;
        if (e < E) spos[atomicAdd(&hist[ekv[r] - kmin], 1)] = (min(max(egj[r], 0), 32767) << 16) | e;
      }
      __syncthreads();
      for (int v = tid; v < R; v += T) {  // hist[v] = end of bucket v
        const int b = hist[v], a = (v == 0) ? 0 : hist[v - 1];
        for (int t = a + 1; t < b; t++) {
          const int x = spos[t];
          int s2 = t - 1;
          while (s2 >= a && spos[s2] > x) {
            spos[s2 + 1] = spos[s2];
            s2--;
          }
          spos[s2 + 1] = x;
        }
      }
      for (int p = tid; p < E; p += T) ehead[p] = 0;
      __syncthreads();
      for (int v = tid; v < R; v += T) {
        const int b = hist[v], a = (v == 0) ? 0 : hist[v - 1];
        if (b > a) ehead[a] = 1;
      }
    } else {
      int P2 = 1;
      while (P2 < E) P2 <<= 1;
      unsigned long long* keys = (unsigned long long*)tmp_low - P2;
      for (int i = tid; i < P2; i += T) keys[i] = ~0ull;
      __syncthreads();
#pragma unroll
      for (int r = 0; r < kBRE; r++) {
        const int e = tid + r * T;
        if (e < E)
          keys[e] = ((unsigned long long)ekv[r] << 32) |
                    ((unsigned)min(max(egj[r], 0), 32767) << 16) | (unsigned)e;
      }
      __syncthreads();
      for (int size = 2; size <= P2; size <<= 1)
        for (int stride = size >> 1; stride > 0; stride >>= 1) {
          for (int i = tid; i < P2 / 2; i += T) {
            const int lo = 2 * i - (i & (stride - 1));
            const int hi = lo + stride;
            const bool up = ((lo & size) == 0);
            const unsigned long long a = keys[lo], b = keys[hi];
            if ((a > b) == up) {
              keys[lo] = b;
              keys[hi] = a;
            }
          }
          __syncthreads();
        }
      for (int p = tid; p < E; p += T) {
        spos[p] = (int)(keys[p] & 0xffffffffull);
        ehead[p] = (p == 0 || (keys[p] >> 32) != (keys[p - 1] >> 32)) ? 1 : 0;
      }
    }
    __syncthreads();
    for (int p = tid; p < E; p += T) epos[spos[p] & 0xffff] = p;
  }
  bstamp(A, 41);
  // S3: patch of each position (scan of heads), first positions, free-pose masks
  int heads[kBRE];
#pragma unroll
  for (int r = 0; r < kBRE; r++) heads[r] = (tid + r * T < E) ? ehead[tid + r * T] : 0;
  const int nuniq = fscan(ehead, E, scr);  // ehead[p] = #heads before p
  for (int u = tid; u < nuniq; u += T) pmask[u] = 0;
#pragma unroll
  for (int r = 0; r < kBRE; r++) {
    const int p = tid + r * T;
    if (p < E && heads[r]) poff[ehead[p]] = p;
  }
  if (tid == 0) poff[nuniq] = E;
  for (int p = tid; p < E; p += T) ppat[p] = (p + 1 < E) ? ehead[p + 1] - 1 : nuniq - 1;
  __syncthreads();
  auto patch_of = [&](int p) -> int { return ppat[p]; };
#pragma unroll
  for (int r = 0; r < kBRE; r++) {
    const int e = tid + r * T;
    if (e < E) {
      const unsigned ci = code_of(slot_of(egi[r]), N), cj = code_of(slot_of(egj[r]), N);
      const unsigned m = (ci != kFixed ? 1u << ci : 0u) | (cj != kFixed ? 1u << cj : 0u);
      if (m) atomicOr(&pmask[patch_of(epos[e])], m);
    }
  }
  __syncthreads();
  // S4: relevant patches of block (ba, bb): mask holds both; workgroup 0 also
  // takes the patches without a free pose (their dZ = Q u)
  const unsigned need = (NB > 0) ? ((1u << ba) | (1u << bb)) : 0u;
  for (int u = tid; u < nuniq; u += T) {
    const unsigned m = pmask[u];
    const bool rel = (NB == 0) ? (m == 0)
                               : ((u & 1) == sub) && ((m & need) == need || (blk == 0 && m == 0));
    ehead[u] = rel ? 1 : 0;
  }
  __syncthreads();
  const int nrel = fscan(ehead, nuniq, scr);  // ehead[u] = relevant index (exclusive)
  for (int u = tid; u < nuniq; u += T) {
    const int nx = (u + 1 < nuniq) ? ehead[u + 1] : nrel;
    ridx[u] = (nx != ehead[u]) ? ehead[u] : -1;
  }
  __syncthreads();
  // relevant-edge offsets: sizes of relevant patches, scanned (reuse spos)
  for (int u = tid; u < nuniq; u += T)
    if (ridx[u] >= 0) spos[ridx[u]] = poff[u + 1] - poff[u];
  __syncthreads();
  const int nrp = fscan(spos, nrel, scr);
  // carve persistent arrays
  {
    size_t o = head_end;
    auto take = [&](size_t b) {
      char* p = lds + o;
      o = al16(o + b);
      return p;
    };
    L.roff = (unsigned short*)take(sizeof(unsigned short) * (nrel + 1));
    L.nxy = (float2*)take(sizeof(float2) * (nrel > 0 ? nrel : 1));
    L.dep = (float*)take(sizeof(float) * (nrel > 0 ? nrel : 1));
    L.pc = (unsigned short*)take(sizeof(unsigned short) * (nrp > 0 ? nrp : 1));
    L.tw = (float4*)take(sizeof(float4) * (nrp > 0 ? nrp : 1));
    L.rpat = (unsigned short*)take(sizeof(unsigned short) * (nrp > 0 ? nrp : 1));
    L.scratch = lds + o;
    // scratch = [reduction table | solver (workgroup 0)] then, if they fit,
    // the per-edge entries and per-patch (Q, u) of the iteration in flight
    const size_t red_bytes = sizeof(double) * (kV * kRedCols + kV * 8);
    const size_t NN = (size_t)(N > 0 ? N : 1);
    const size_t s32 = solver32_bytes((int)NN), s64 = sizeof(double) * (36 * NN * (NN + 1) / 2 + 90 * NN);
    const size_t solve_bytes = s32 > s64 ? s32 : s64;
    size_t o2 = al16(o + (red_bytes > solve_bytes ? red_bytes : solve_bytes));
    const size_t pe_bytes = al16(sizeof(double) * 14 * (size_t)(nrp > 0 ? nrp : 1));
    const size_t pq_bytes = al16(sizeof(double2) * (size_t)(nrel > 0 ? nrel : 1));
    if (o2 + pe_bytes + pq_bytes <= (size_t)kBLds) {
      L.pe = (double*)(lds + o2);
      L.pq = (double2*)(lds + o2 + pe_bytes);
    } else {
      L.pe = nullptr;
      L.pq = nullptr;
    }
    if (tid == 0) {
      ctl[kCNrel] = nrel;
      ctl[kCNrp] = nrp;
      ctl[kCNuniq] = nuniq;
      ctl[kCGo] = (o <= (size_t)(tmp_low - lds)) ? 1 : 0;  // never overlaps the temporaries
    }
  }
  __syncthreads();
  bstamp(A, 42);
  // S5: relevant edges (edge owners scatter); patch heads -> poff[] slot reuse
#pragma unroll
  for (int r = 0; r < kBRE; r++) {
    const int e = tid + r * T;
    if (e >= E) continue;
    const int p = epos[e], u = patch_of(p);
    const int ri = ridx[u];
    if (ri < 0) continue;
    const int q = spos[ri] + (p - poff[u]);
    L.pc[q] = (unsigned short)(slot_of(egi[r]) | (slot_of(egj[r]) << 8));
    L.tw[q] = etw[r];
    L.rpat[q] = (unsigned short)ri;
    gidx[2 * q] = egi[r];
    gidx[2 * q + 1] = egj[r];
    if (p == poff[u]) ehead[ri] = ekv[r];  // patch id of relevant patch ri
  }
  __syncthreads();
  // patch records: all loads of a thread's patches issued together
  for (int u = tid; u < nuniq; u += T) {
    const int ri = ridx[u];
    if (ri < 0) continue;
    L.roff[ri] = (unsigned short)spos[ri];
    const int kx = ehead[ri];
    const float* pk = A.patches + (size_t)kx * 3 * PP;
    const int c11 = P + 1;  // [*][1][1] (ba_cuda.cu:282-285)
    const float px = pk[c11], py = pk[PP + c11], d11 = pk[2 * PP + c11], d00 = pk[2 * PP];
    L.nxy[ri] = make_float2((px - cx) / fx, (py - cy) / fy);
    L.dep[ri] = d11;
    dbw[ri] = d00;  // patch_retr_kernel reads [2][0][0] (:225)
    // owner: diagonal workgroup of the lowest free pose; workgroup 0 for none
    const unsigned m = pmask[u];
    const bool own = (m == 0) ? (blk == 0) : (diag && (int)__builtin_ctz(m) == ba);
    kxw[ri] = own ? kx : -1;
  }
  if (tid == 0) L.roff[nrel] = (unsigned short)nrp;
  // pose table: free poses t0.., then fixed ones from fmin
  for (int k = tid; k < kSlots * 8; k += T) {
    const int sl = k >> 3, c = k & 7;
    const int gp = (sl < N) ? t0 + sl : fmin + (sl - N);
    float v = (c == 6) ? 1.0f : 0.0f;
    if (c < 7 && gp >= 0 && gp < A.num_poses && (sl < N || fmin != 0x7fffffff))
      v = A.poses[7 * (size_t)gp + c];
    L.pose[k] = v;
  }
  __syncthreads();
  bstamp(A, 1);

  // ============================ iterations ============================
  const double lam = (double)A.lmbda[0];
  double* red = (double*)L.scratch;  // [kV][kRedCols] (+ [kV][8] partials)
  int timeout = 0;
  auto pose_ptr = [&](unsigned slot, int q, int which) -> const float* {
    return slot == kGlb ? A.poses + 7 * (size_t)gidx[2 * q + which] : L.pose + 8 * slot;
  };
  // apply dX of iteration `it`: poses (every workgroup, same bits) and the
  // inverse depths of the relevant patches (entries / Q, u of iteration it)
  auto apply_step = [&](int it) {
    if (tid == 0) {
      if (!wait_geq(&A.flags[gridDim.x], A.epoch * 64 + it + 1)) ctl[kCTimeout] = 1;
    }
    __syncthreads();
    const double* dXi = A.dXg + (size_t)(it & 1) * 6 * N;
    for (int k = tid; k < 6 * N; k += T) L.dX[k] = dXi[k];
    __syncthreads();
    for (int i = tid; i < N; i += T) {  // pose_retr_kernel (:178-206)
      float xi[6], tt[3], qq[4], t1[3], q1[4];
#pragma unroll
      for (int k = 0; k < 6; k++) xi[k] = (float)L.dX[6 * i + k];
      float* pl = L.pose + 8 * i;
      tt[0] = pl[0]; tt[1] = pl[1]; tt[2] = pl[2];
      qq[0] = pl[3]; qq[1] = pl[4]; qq[2] = pl[5]; qq[3] = pl[6];
      retrSE3(xi, tt, qq, t1, q1);
      pl[0] = t1[0]; pl[1] = t1[1]; pl[2] = t1[2];
      pl[3] = q1[0]; pl[4] = q1[1]; pl[5] = q1[2]; pl[6] = q1[3];
    }
    __syncthreads();  // pose table / dX before the depth update
    if (L.pe) {
      // E^T dX per edge (thread per edge), then per patch in edge order
      for (int q = tid; q < nrp; q += T) {
        double* pe = L.pe + 14 * (size_t)q;
        const unsigned b = L.pc[q];
        const unsigned ci = code_of(b & 0xff, N), cj = code_of(b >> 8, N);
        double ex = 0.0;
        if (cj != kFixed)
#pragma unroll
          for (int k = 0; k < 6; k++) ex += pe[2 + k] * L.dX[6 * cj + k];
        if (ci != kFixed)
#pragma unroll
          for (int k = 0; k < 6; k++) ex += pe[8 + k] * L.dX[6 * ci + k];
        pe[0] = ex;  // c is no longer needed
      }
      __syncthreads();
    }
    for (int ri = tid; ri < nrel; ri += T) {  // dZ = Q (u - E^T dX) (:563), patch_retr (:209-229)
      const double2 qu = L.pe ? L.pq[ri] : reinterpret_cast<const double2*>(QU)[ri];
      double ex = 0.0;
      for (int q = L.roff[ri]; q < L.roff[ri + 1]; q++) {
        if (L.pe) {
          ex += L.pe[14 * (size_t)q];
          continue;
        }
        const unsigned b = L.pc[q];
        const unsigned ci = code_of(b & 0xff, N), cj = code_of(b >> 8, N);
        double e6[6];
        if (cj != kFixed) {
          load6(EW + 12 * (size_t)q, e6);
#pragma unroll
          for (int k = 0; k < 6; k++) ex += e6[k] * L.dX[6 * cj + k];
        }
        if (ci != kFixed) {
          load6(EW + 12 * (size_t)q + 6, e6);
#pragma unroll
          for (int k = 0; k < 6; k++) ex += e6[k] * L.dX[6 * ci + k];
        }
      }
      const float dz = (float)(qu.x * (qu.y - ex));
      const float base = (it == 0) ? dbw[ri] : L.dep[ri];
      float d = base + dz;
      d = (d > 20.0f) ? 1.0f : d;
      L.dep[ri] = (float)fmax((double)d, 1e-4);
    }
    __syncthreads();
  };

  for (int it = 0; it < A.iters; it++) {
    if (it > 0) apply_step(it - 1);
    const int mb = 2 + 8 * it;
    // ---- linearise the relevant patches; accumulate and store block (ba, bb) ----
    {
      const Ctx cx_{A, L, EW, QU, gidx, red, nrel, ba, bb, g, it, lam, fx, fy, cx, cy};
      if (NB == 0)
        assemble<0>(cx_);
      else if (diag)
        assemble<1>(cx_);
      else
        assemble<2>(cx_);
    }
    if (g == 0) bstamp(A, mb + 1);
    // ---- workgroup 0: gather S, solve, publish dX ----
    if (g == 0) {
      const int NN = N > 0 ? N : 1;
      Solver32 sv;
      double* Sd = (double*)L.scratch;  // gathered + damped S, then y
      double* yd = Sd + 36 * (NB > 0 ? NB : 1);
      sv.S = Sd;
      sv.y = yd;
      sv.x = yd + 6 * NN;
      sv.part = sv.x + 6 * NN;
      sv.A = (float*)(sv.part + 24 * NN);
      sv.Li = sv.A + 36 * (NB > 0 ? NB : 1);
      sv.w = sv.Li + 36 * NN;
      sv.Nf = sv.w + 6 * NN;
      double* dXo = A.dXg + (size_t)(it & 1) * 6 * N;
      if (NB > 0) {
        for (int w = tid; w < 2 * NB; w += T)  // one lane per arrival flag
          if (!wait_geq(&A.flags[w], A.epoch * 64 + it + 1)) ctl[kCTimeout] = 1;
        __syncthreads();
        bstamp(A, mb + 2);
        {  // sum the two halves of every block (fixed order); 8 loads in flight
          const int tot = 36 * NB;
          for (int k0 = tid; k0 < tot; k0 += 8 * T) {
            double v0[8], v1[8];
#pragma unroll
            for (int r = 0; r < 8; r++) {
              const int k = k0 + r * T, b = k / 36, e = k % 36;
              v0[r] = (k < tot) ? A.Sg[72 * b + e] : 0.0;
              v1[r] = (k < tot) ? A.Sg[72 * b + 36 + e] : 0.0;
            }
#pragma unroll
            for (int r = 0; r < 8; r++)
              if (k0 + r * T < tot) Sd[k0 + r * T] = v0[r] + v1[r];
          }
          for (int k = tid; k < 6 * N; k += T) yd[k] = A.yg[k] + A.yg[6 * N + k];
        }
        __syncthreads();
        for (int k = tid; k < 6 * N; k += T) {  // S += I (1e-4 S + 1) (ba_cuda.cu:560)
          double* d = Sd + 36 * lblk(k / 6, k / 6) + 7 * (k % 6);
          *d += 1e-4 * *d + 1.0;
        }
        if (tid == 0) ctl[kCFail] = 0;
        __syncthreads();
        bstamp(A, mb + 3);
        if (A.refine == 2) {
          Solver sd;  // fp64 LDL^T in the same scratch (S, y in place)
          sd.S = Sd;
          sd.y = yd;
          sd.piv = yd + 6 * NN;
          sd.wv = sd.piv + 36 * NN;
          sd.tt = sd.wv + 6 * NN;
          sd.PV = sd.tt + 6 * NN;
          block_ldl_solve(sd, N, L.dX, &ctl[kCFail], A.marks ? A.marks + mb : nullptr);
        } else {
          chol32_solve(sv, N, L.dX, &ctl[kCFail], A.refine == 1, A.marks ? A.marks + mb : nullptr);
        }
        bstamp(A, mb + 5);
        const bool fail = ctl[kCFail] != 0 || ctl[kCTimeout] != 0;
        if (tid < 64)  // wave 0 writes: its own release fence below covers the stores
          for (int k = tid; k < 6 * N; k += 64) dXo[k] = fail ? 0.0 : L.dX[k];  // (dpvo/ba.py:17-21)
        __syncthreads();
      }
      bstamp(A, mb + 6);
      if (tid == 0) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        __hip_atomic_store(&A.flags[gridDim.x], A.epoch * 64 + it + 1, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
      }
    }
  }
  // ============================ final update + write-back ============================
  if (A.iters > 0) apply_step(A.iters - 1);
  for (int k = tid; k < nrel * PP; k += T) {
    const int ri = k / PP, c = k % PP;
    const int kx = kxw[ri];
    if (kx >= 0) A.patches[(size_t)kx * 3 * PP + 2 * PP + c] = L.dep[ri];
  }
  if (g == 0) {
    for (int i = tid; i < N; i += T) {
      const int gp = t0 + i;
      if (gp >= 0 && gp < A.num_poses)
        for (int c = 0; c < 7; c++) A.poses[7 * (size_t)gp + c] = L.pose[8 * i + c];
    }
    if (tid == 0) {
      __hip_atomic_store(&A.flags[kEpochWord], A.epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      A.meta[0] = nuniq;
      A.meta[1] = (ctl[kCFail] ? 1 : 0) | (ctl[kCBad] ? 2 : 0) | (ctl[kCTimeout] ? 16 : 0);
    }
    bstamp(A, 63);
  }
  (void)timeout;
}

}  // namespace

// host side ------------------------------------------------------------------
static size_t al256(size_t v) { return (v + 255) / 256 * 256; }

size_t ba_blocks_scratch_bytes(int E, int N) {
  const int NB = N * (N + 1) / 2, G = NB > 0 ? 2 * NB : 1, N1 = N > 0 ? N : 1;
  return al256(sizeof(double) * 36 * G) + al256(sizeof(double) * 12 * N1) +
         al256(sizeof(double) * 12 * N1) + al256(sizeof(double) * 12 * (size_t)G * E) +
         al256(sizeof(double) * 2 * (size_t)G * E) + al256(sizeof(int) * 2 * (size_t)G * E) +
         al256(sizeof(int) * (size_t)G * E) + al256(sizeof(float) * (size_t)G * E);
}

bool ba_blocks_supported(int E, int N, int P) {
  return E > 0 && E <= kBMaxE && N >= 0 && N <= kBMaxN && P >= 2 && P * P <= 64;
}

// Arrival / publish flags live in library-owned device memory, one set per
// device, zeroed once (so a hipGraph capture on a side stream finds them
// allocated; BA calls on one device must therefore not overlap in time).  Every call tags its flags with a new epoch
// kept in the same buffer (advanced on the device), so no per-call reset
// (memset launch) is needed, a call that timed out cannot confuse the next
// one, and hipGraph replays stay correct.
namespace {
constexpr int kFlagWords = 2 * (kBMaxN * (kBMaxN + 1) / 2) + 8;
std::mutex g_flag_mu;
std::map<int, long long*> g_flags;  // per device (streams share it: see below)
}  // namespace

static int g_blocks_refine = 2;  // fp64 block LDL^T (dpvo_ba_set_refine: fastest measured)
void ba_blocks_set_refine(int mode) { g_blocks_refine = mode; }

static long long* flag_slot(hipStream_t st) {
  int dev = 0;
  (void)hipGetDevice(&dev);
  std::lock_guard<std::mutex> lk(g_flag_mu);
  auto it = g_flags.find(dev);
  if (it != g_flags.end()) return it->second;
  long long* p = nullptr;
  if (hipMalloc(&p, sizeof(long long) * kFlagWords) != hipSuccess) return nullptr;
  if (hipMemsetAsync(p, 0, sizeof(long long) * kFlagWords, st) != hipSuccess) return nullptr;
  g_flags[dev] = p;
  return p;
}

int ba_blocks_launch(float* poses, float* patches, const float* intrinsics, const float* target,
                     const float* weight, const float* lmbda, const int64_t* ii, const int64_t* jj,
                     const int64_t* kk, int E, int P, int num_poses, int num_patches, int t0, int t1,
                     int iterations, char* scratch, int* meta, int64_t* marks, void* stream) {
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)ba_blocks_kernel,
                              hipFuncAttributeMaxDynamicSharedMemorySize, kBLds);
    attr = true;
  }
  if (iterations > 63) return DPVO_ERR_UNSUPPORTED;  // 6-bit iteration tag per epoch
  const int N = t1 - t0, NB = N * (N + 1) / 2, G = NB > 0 ? 2 * NB : 1, N1 = N > 0 ? N : 1;
  hipStream_t st = as_stream(stream);
  BArgs a;
  a.flags = flag_slot(st);
  a.epoch = 0;
  if (!a.flags) return DPVO_ERR_LAUNCH;
  a.poses = poses;
  a.patches = patches;
  a.intrinsics = intrinsics;
  a.target = target;
  a.weight = weight;
  a.lmbda = lmbda;
  a.ii = ii;
  a.jj = jj;
  a.kk = kk;
  a.E = E;
  a.P = P;
  a.num_poses = num_poses;
  a.num_patches = num_patches;
  a.t0 = t0;
  a.N = N;
  a.iters = iterations;
  a.NB = NB;
  char* s = scratch;
  a.Sg = (double*)s;
  s += al256(sizeof(double) * 36 * G);
  a.yg = (double*)s;
  s += al256(sizeof(double) * 12 * N1);
  a.dXg = (double*)s;
  s += al256(sizeof(double) * 12 * N1);
  a.EW = (double*)s;
  s += al256(sizeof(double) * 12 * (size_t)G * E);
  a.QU = (double*)s;
  s += al256(sizeof(double) * 2 * (size_t)G * E);
  a.gidx = (int*)s;
  s += al256(sizeof(int) * 2 * (size_t)G * E);
  a.kxw = (int*)s;
  s += al256(sizeof(int) * (size_t)G * E);
  a.dbw = (float*)s;
  a.meta = meta;
  a.marks = marks;
  a.refine = g_blocks_refine;
  hipLaunchKernelGGL(ba_blocks_kernel, dim3(G), dim3(kBT), kBLds, st, a);
  return launch_status();
}

}  // namespace dpvo
