// ba_large.hip -- F-BA for large patch graphs: DPVO's global BA
// (dpvo.py:695-715 -> fastba.BA(..., eff_impl=True)) and BASELINE cfg4
// (1024 frames x 96 patches, ~131k edges, N = 1023 free poses), on one GPU
// or edge-sharded across ranks.
//
// Reference semantics: dpvo/fastba/ba_cuda.cu:433-582 with the block-sparse
// E of block_e.cu:43-300 (EfficentE):
//   per edge: residual + Jacobians in fp32 (ba_cuda.cu:265-333)
//   B, E, C, v, u (:339-373); Q = 1/(C + lmbda) (:519)
//   S = B - E Q E^T, y = v - E Q u (block_e.cu:188-300), S += I (1e-4 S + 1)
//   dX = chol_solve(S, y) (ba_cuda.cu:561-562), dZ = Q (u - E^T dX) (:563)
//   pose_retr_kernel (:178-206), patch_retr_kernel (:209-229).
// The reference factorises the dense 6N x 6N S (150 MB fp32 at N = 1023,
// ~7.7e10 flop) after ~320 fp32 atomics per edge.  Here (DESIGN.md "F-BA,
// large graphs"):
//
//   setup (once per call, no host round trip)
//     positions = edges radix-sorted by patch (stable: edge order inside a
//     patch), unique patches, each patch's set of free poses (<= kMaxSet);
//     "items" (lower block (a, b), patch u) for every pose pair of every
//     patch, radix-sorted by block -> the block-sparse pattern of S and, per
//     block, the patches that feed it.  Band analysis: a pose with a
//     coupling more than kGCap poses back goes to the "border"; the rest is
//     block-tridiagonal in superblocks of g <= kGCap poses (m = 6g rows).
//   per iteration
//     lin     thread per patch: fp32 edge linearisation (J records), C, u, Q
//             and the E column blocks of the patch in fp64, in edge order.
//     block   wave per nonzero lower 6x6 block of S: B terms of the block's
//             pose pair + -Q E_a E_b^T over its patches, fixed lane order +
//             butterfly reduction (deterministic, no atomics); the diagonal
//             block also produces y_a.
//     -- edge-sharded: all_reduce(SUM) of the packed [y | S blocks] here --
//     assemble  damped S into superblocks D_k, couplings L_k = A[k+1, k],
//             border columns, border-border block.
//     solve   block cyclic reduction over the superblocks (each level: one
//             workgroup per eliminated superblock inverts D_o in LDS
//             (Gauss-Jordan, SPD, fp64) and forms D_o^-1 [L, L^T, rhs]; one
//             per kept superblock applies the Schur updates), then the
//             border Schur complement (dense, small), back substitution.
//     update  pose retraction (fp32, reference order), dZ, inverse depths.
// Everything is fp64 with a fixed summation order; the per-edge math is the
// reference's fp32 (no contraction), identical to the C oracle.
#include <cstring>
#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/device/device_scan.hpp>

#include "ba_bgj.hpp"
#include "ba_device.hpp"

namespace dpvo {
namespace gba {
using namespace bad;

constexpr int kMaxSet = 24;     // free poses one patch may touch
constexpr int kMaxBorder = 64;  // poses coupled further back than kGCap
constexpr int kMaxNB6 = 6 * kMaxBorder;
constexpr int kMaxN = 8192;
constexpr int kItemsPerEdge = 25;  // max over k of min(k (2k+1), kMaxSet (kMaxSet+1) / 2) / k
constexpr int kT = 256;
constexpr int kMetaInts = 16;
constexpr int kBP = 32;        // border Schur partial groups

// status bits (Meta::status)
constexpr int kStChol = 1;      // a pivot was not positive: dX = 0 this iteration
constexpr int kStClamp = 2;     // kk outside [0, num_patches) (clamped)
constexpr int kStSet = 4;       // a patch touches more than kMaxSet free poses
constexpr int kStBorder = 8;    // more than kMaxBorder border poses

struct Meta {
  int nuniq, nitems, nblk, nI, nB, g, m, nsb, status, kbits, pad[kMetaInts - 10];
};

struct Ws {
  Meta* meta;
  // setup
  uint32_t *pkey, *pkey2, *pval, *pval2;  // [E] patch sort
  int *flag, *scan;                       // [E] scratch
  int* poff;                              // [E+1] patch -> position range
  int* pkk;                               // [E] patch id (kk) of each unique patch
  uint8_t* own;                           // [E] patch owned by this rank
  int* psetf;                             // [E][kMaxSet] pose set (relative pose ids, ascending)
  int *pscnt, *psoff, *itcnt, *itoff;     // [E]
  uint32_t *ikey, *ikey2, *ival, *ival2;  // [IB] items
  int *iflag, *iscan;                     // [IB]
  int2* bab;                              // [NBB] block (a, b), a >= b
  int* boff;                              // [NBB+1]
  int *cidx, *bidx, *bpos;                // [N], [N], [kMaxBorder]
  // per iteration
  float* J;       // [E][32] per position: w[2] r[2] Jz[2] Ji[2][6] Jj[2][6]
  double *Qp, *up;  // [E] per patch
  double* Ev;     // [2E][6] per (patch, pose slot): E column block
  double* packed; // [6N] y, then [NBB][36] lower blocks of S
  double *D, *Lo0, *Lo1, *Y1, *Y2;  // superblock storage [SB2]
  double *R, *BT;                   // [SBR] rhs / solution, border columns
  double *Cb, *rb, *dXB;            // border system
  double* Pb;                       // [kBP][6 nB][1 + 6 nB] border Schur partials
  double* dX;                       // [6N]
  void* tmp;                        // rocPRIM temporary storage
  size_t tmp_bytes;
};

inline size_t al(size_t b) { return (b + 255) & ~(size_t)255; }

inline int item_bound(int E) { return kItemsPerEdge * E; }
inline int blk_bound(int E, int N) {
  const long long tri = (long long)N * (N + 1) / 2;
  return (int)std::min<long long>((long long)item_bound(E), tri > 0 ? tri : 1);
}
inline size_t sb2_bound(int N) { return (size_t)36 * kGCap * (N + kGCap); }
inline size_t sbr_bound(int N) { return (size_t)6 * (N + kGCap) * (1 + kMaxNB6); }
inline int key_bits(long long maxkey) {  // bits so that (1 << b) - 1 > maxkey
  int b = 1;
  while ((1LL << b) - 1 <= maxkey) b++;
  return b;
}

static size_t rocprim_tmp_bytes(int E) {
  const int IB = item_bound(E);
  size_t a = 0, b = 0, c = 0;
  uint32_t* u = nullptr;
  int* i = nullptr;
  if (rocprim::radix_sort_pairs(nullptr, a, u, u, u, u, (unsigned)IB, 0, 32) != hipSuccess)
    a = (size_t)16 * IB + (64u << 20);
  if (rocprim::inclusive_scan(nullptr, b, i, i, (size_t)IB, rocprim::plus<int>()) != hipSuccess)
    b = (size_t)8 * IB + (1u << 20);
  if (rocprim::exclusive_scan(nullptr, c, i, i, 0, (size_t)IB, rocprim::plus<int>()) !=
      hipSuccess)
    c = (size_t)8 * IB + (1u << 20);
  return std::max(a, std::max(b, c));
}

static size_t layout(int E, int N, char* base, Ws* w) {
  const int IB = item_bound(E), NBB = blk_bound(E, N);
  const int Np = N > 0 ? N : 1;
  size_t off = 0;
  auto take = [&](size_t bytes) -> char* {
    char* p = base ? base + off : nullptr;
    off += al(bytes);
    return p;
  };
  Ws t;
  t.meta = (Meta*)take(sizeof(Meta));
  t.pkey = (uint32_t*)take(4 * (size_t)E);
  t.pkey2 = (uint32_t*)take(4 * (size_t)E);
  t.pval = (uint32_t*)take(4 * (size_t)E);
  t.pval2 = (uint32_t*)take(4 * (size_t)E);
  t.flag = (int*)take(4 * (size_t)E);
  t.scan = (int*)take(4 * (size_t)E);
  t.poff = (int*)take(4 * ((size_t)E + 1));
  t.pkk = (int*)take(4 * (size_t)E);
  t.own = (uint8_t*)take((size_t)E);
  t.psetf = (int*)take(4 * (size_t)E * kMaxSet);
  t.pscnt = (int*)take(4 * (size_t)E);
  t.psoff = (int*)take(4 * (size_t)E);
  t.itcnt = (int*)take(4 * (size_t)E);
  t.itoff = (int*)take(4 * (size_t)E);
  t.ikey = (uint32_t*)take(4 * (size_t)IB);
  t.ikey2 = (uint32_t*)take(4 * (size_t)IB);
  t.ival = (uint32_t*)take(4 * (size_t)IB);
  t.ival2 = (uint32_t*)take(4 * (size_t)IB);
  t.iflag = (int*)take(4 * (size_t)IB);
  t.iscan = (int*)take(4 * (size_t)IB);
  t.bab = (int2*)take(8 * (size_t)NBB);
  t.boff = (int*)take(4 * ((size_t)NBB + 1));
  t.cidx = (int*)take(4 * (size_t)Np);
  t.bidx = (int*)take(4 * (size_t)Np);
  t.bpos = (int*)take(4 * (size_t)kMaxBorder);
  t.J = (float*)take(4 * 32 * (size_t)E);
  t.Qp = (double*)take(8 * (size_t)E);
  t.up = (double*)take(8 * (size_t)E);
  t.Ev = (double*)take(8 * 6 * 2 * (size_t)E);
  t.packed = (double*)take(8 * (6 * (size_t)Np + 36 * (size_t)NBB));
  const size_t SB2 = sb2_bound(Np), SBR = sbr_bound(Np);
  t.D = (double*)take(8 * SB2);
  t.Lo0 = (double*)take(8 * SB2);
  t.Lo1 = (double*)take(8 * SB2);
  t.Y1 = (double*)take(8 * SB2);
  t.Y2 = (double*)take(8 * SB2);
  t.R = (double*)take(8 * SBR);
  t.BT = (double*)take(8 * SBR);
  t.Cb = (double*)take(8 * (size_t)kMaxNB6 * kMaxNB6);
  t.rb = (double*)take(8 * (size_t)kMaxNB6);
  t.dXB = (double*)take(8 * (size_t)kMaxNB6);
  t.Pb = (double*)take(8 * (size_t)kBP * kMaxNB6 * (kMaxNB6 + 1));
  t.dX = (double*)take(8 * 6 * (size_t)Np);
  t.tmp_bytes = rocprim_tmp_bytes(E);
  t.tmp = take(t.tmp_bytes);
  if (w) *w = t;
  return off;
}

__device__ __forceinline__ double* y_of(const Ws& w) { return w.packed; }
__device__ __forceinline__ double* S_of(const Ws& w, int N) { return w.packed + 6 * N; }

// number of active superblocks at CR level lev
__device__ __forceinline__ int level_count(int nsb, int lev) {
  int n = nsb;
  for (int l = 0; l < lev; l++) n = (n + 1) >> 1;
  return n;
}

// ------------------------------------------------------------------- setup
__global__ void k_keys(const int64_t* __restrict__ kk, int E, int num_patches, Ws w) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e == 0) {
    Meta* m = w.meta;
    m->nuniq = m->nitems = m->nblk = m->nI = m->nB = m->nsb = 0;
    m->g = 1;
    m->m = 6;
    m->status = 0;
  }
  if (e >= E) return;
  int64_t k = kk[e];
  if (k < 0 || k >= num_patches) {
    k = k < 0 ? 0 : num_patches - 1;
    atomicOr(&w.meta->status, kStClamp);
  }
  w.pkey[e] = (uint32_t)k;
  w.pval[e] = (uint32_t)e;
}

__global__ void k_pflag(int E, Ws w) {
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= E) return;
  w.flag[p] = (p == 0 || w.pkey2[p] != w.pkey2[p - 1]) ? 1 : 0;
}

__global__ void k_pscatter(int E, Ws w) {
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= E) return;
  const int u = w.scan[p] - 1;  // inclusive scan
  if (w.flag[p]) {
    w.poff[u] = p;
    w.pkk[u] = (int)w.pkey2[p];
  }
  if (p == E - 1) {
    w.meta->nuniq = u + 1;
    w.poff[u + 1] = E;
  }
}

// pose set of each patch: free poses (ii - t0, jj - t0 in [0, N)) of its edges
__global__ void k_pset(const int64_t* __restrict__ ii, const int64_t* __restrict__ jj, int E,
                       int t0, int N, int PPF, int own_lo, int own_hi, Ws w) {
  const int u = blockIdx.x * blockDim.x + threadIdx.x;
  if (u >= E) return;
  const int nuniq = w.meta->nuniq;
  if (u >= nuniq) {
    w.pscnt[u] = 0;
    w.itcnt[u] = 0;
    return;
  }
  int set[kMaxSet];
  int s = 0;
  bool over = false;
  const int p0 = w.poff[u], p1 = w.poff[u + 1];
  for (int p = p0; p < p1; p++) {
    const int e = (int)w.pval2[p];
    const int64_t cand[2] = {ii[e] - t0, jj[e] - t0};
    for (int c = 0; c < 2; c++) {
      const int64_t a = cand[c];
      if (a < 0 || a >= N) continue;
      int pos = 0;
      while (pos < s && set[pos] < a) pos++;
      if (pos < s && set[pos] == a) continue;
      if (s == kMaxSet) {
        over = true;
        continue;
      }
      for (int q = s; q > pos; q--) set[q] = set[q - 1];
      set[pos] = (int)a;
      s++;
    }
  }
  if (over) atomicOr(&w.meta->status, kStSet);
  for (int q = 0; q < s; q++) w.psetf[(size_t)u * kMaxSet + q] = set[q];
  w.pscnt[u] = s;
  w.itcnt[u] = s * (s + 1) / 2;
  const int frame = PPF > 0 ? w.pkk[u] / PPF : 0;
  w.own[u] = (frame >= own_lo && frame < own_hi) ? 1 : 0;
}

__global__ void k_items(int E, int N, Ws w) {
  const int u = blockIdx.x * blockDim.x + threadIdx.x;
  if (u >= E) return;
  if (u == E - 1) w.meta->nitems = w.itoff[u] + w.itcnt[u];
  if (u >= w.meta->nuniq) return;
  const int s = w.pscnt[u];
  const int* set = w.psetf + (size_t)u * kMaxSet;
  int q = w.itoff[u];
  for (int sa = 0; sa < s; sa++)
    for (int sb = 0; sb <= sa; sb++) {
      w.ikey[q] = (uint32_t)lblk(set[sa], set[sb]);
      w.ival[q] = ((uint32_t)u << 10) | ((uint32_t)sa << 5) | (uint32_t)sb;
      q++;
    }
}

__global__ void k_ipad(int IB, uint32_t pad, Ws w) {
  const int q = blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= IB) return;
  if (q >= w.meta->nitems) {
    w.ikey[q] = pad;
    w.ival[q] = 0;
  }
}

__global__ void k_bflag(int IB, Ws w) {
  const int q = blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= IB) return;
  const int n = w.meta->nitems;
  w.iflag[q] = (q < n && (q == 0 || w.ikey2[q] != w.ikey2[q - 1])) ? 1 : 0;
}

__global__ void k_bscatter(int IB, Ws w) {
  const int q = blockIdx.x * blockDim.x + threadIdx.x;
  const int n = w.meta->nitems;
  if (q >= IB || q >= n) return;
  const int b = w.iscan[q] - 1;
  if (w.iflag[q]) {
    int a, c;
    tri_of((int)w.ikey2[q], a, c);
    w.bab[b] = make_int2(a, c);
    w.boff[b] = q;
  }
  if (q == n - 1) {
    w.meta->nblk = b + 1;
    w.boff[b + 1] = n;
  }
}

// band analysis (one workgroup): border poses, interior compression,
// superblock size.
__global__ void __launch_bounds__(1024) k_structure(int N, Ws w) {
  __shared__ int sflag[kMaxN];
  __shared__ int wsum[32];
  __shared__ int sg;
  const int tid = threadIdx.x, nt = blockDim.x;
  Meta* meta = w.meta;
  const int nblk = meta->nitems > 0 ? meta->nblk : 0;
  if (tid == 0) {
    if (meta->nitems == 0) meta->nblk = 0;
    sg = 1;
  }
  for (int a = tid; a < N; a += nt) sflag[a] = 0;
  __syncthreads();
  for (int b = tid; b < nblk; b += nt) {
    const int2 ab = w.bab[b];
    if (ab.x - ab.y > kGCap) sflag[ab.x] = 1;
  }
  __syncthreads();
  // border flags -> bidx (exclusive scan of flags), cidx (of !flags); serial
  // chunks per thread then a wave-level scan of the chunk sums.
  const int per = (N + nt - 1) / nt;
  const int lo = min(tid * per, N), hi = min(lo + per, N);
  int nb = 0;
  for (int a = lo; a < hi; a++) nb += sflag[a];
  // block exclusive scan of nb (nt <= 1024 = 16 waves)
  int x = nb;
  const int lane = tid & 63, wid = tid >> 6;
  for (int o = 1; o < 64; o <<= 1) {
    const int t = __shfl_up(x, o, 64);
    if (lane >= o) x += t;
  }
  if (lane == 63) wsum[wid] = x;
  __syncthreads();
  if (tid == 0) {
    int acc = 0;
    for (int q = 0; q < nt / 64; q++) {
      const int v = wsum[q];
      wsum[q] = acc;
      acc += v;
    }
    wsum[31] = acc;
  }
  __syncthreads();
  int bb = wsum[wid] + x - nb;  // border poses before lo
  const int nB = wsum[31];
  for (int a = lo; a < hi; a++) {
    if (sflag[a]) {
      w.bidx[a] = bb;
      w.cidx[a] = -1;
      if (bb < kMaxBorder) w.bpos[bb] = a;
      bb++;
    } else {
      w.bidx[a] = -1;
      w.cidx[a] = a - bb;
    }
  }
  __syncthreads();
  // superblock size: largest compressed distance of an interior coupling
  int gl = 1;
  for (int b = tid; b < nblk; b += nt) {
    const int2 ab = w.bab[b];
    const int ca = w.cidx[ab.x], cb = w.cidx[ab.y];
    if (ca >= 0 && cb >= 0) gl = max(gl, ca - cb);
  }
  atomicMax(&sg, gl);
  __syncthreads();
  if (tid == 0) {
    const int nI = N - nB, g = min(sg, kGCap);
    meta->nI = nI;
    meta->nB = nB;
    meta->g = g;
    meta->m = 6 * g;
    meta->nsb = (nI + g - 1) / g;
    if (nB > kMaxBorder) {  // unsupported coupling pattern: no solve, dX = 0
      meta->status |= kStBorder;
      meta->nsb = 0;
      meta->nB = 0;
    }
  }
}

// ------------------------------------------------------------ iteration
// thread per (owned) patch: linearise its edges in edge order
__global__ void k_lin(const float* __restrict__ poses, const float* __restrict__ patches,
                      const float* __restrict__ intrinsics, const float* __restrict__ target,
                      const float* __restrict__ weight, const float* __restrict__ lmbda,
                      const int64_t* __restrict__ ii, const int64_t* __restrict__ jj, int E,
                      int P, int num_poses, int t0, int N, Ws w) {
  const int u = blockIdx.x * blockDim.x + threadIdx.x;
  if (u >= E || u >= w.meta->nuniq || !w.own[u]) return;
  const float fx = intrinsics[0], fy = intrinsics[1], cx = intrinsics[2], cy = intrinsics[3];
  const int s = w.pscnt[u];
  const int* set = w.psetf + (size_t)u * kMaxSet;
  double* Ev = w.Ev + 6 * (size_t)w.psoff[u];
  for (int q = 0; q < 6 * s; q++) Ev[q] = 0.0;
  const float* pk = patches + (size_t)w.pkk[u] * 3 * P * P;
  const int c11 = P + 1;  // patches[k][*][1][1] (ba_cuda.cu:282-285)
  const float px = pk[c11], py = pk[P * P + c11], pd = pk[2 * P * P + c11];
  const float nx = (px - cx) / fx, ny = (py - cy) / fy;
  double C = 0.0, uu = 0.0;
  const int p0 = w.poff[u], p1 = w.poff[u + 1];
  for (int p = p0; p < p1; p++) {
    const int e = (int)w.pval2[p];
    const int64_t gi = ii[e], gj = jj[e];
    const int pi = (int)min<int64_t>(max<int64_t>(gi, 0), num_poses - 1);
    const int pj = (int)min<int64_t>(max<int64_t>(gj, 0), num_poses - 1);
    Lin L;
    lin_edge(poses + 7 * pi, poses + 7 * pj, nx, ny, pd, target[2 * e], target[2 * e + 1],
             weight[2 * e], weight[2 * e + 1], fx, fy, cx, cy, L);
    float* rec = w.J + 32 * (size_t)p;
    rec[0] = L.w[0];
    rec[1] = L.w[1];
    rec[2] = L.r[0];
    rec[3] = L.r[1];
    rec[4] = L.Jz[0];
    rec[5] = L.Jz[1];
#pragma unroll
    for (int r = 0; r < 2; r++)
#pragma unroll
      for (int a = 0; a < 6; a++) {
        rec[6 + 6 * r + a] = L.Ji[r][a];
        rec[18 + 6 * r + a] = L.Jj[r][a];
      }
    const int64_t ri = gi - t0, rj = gj - t0;
    int si = -1, sj = -1;
    for (int q = 0; q < s; q++) {
      if (set[q] == ri) si = q;
      if (set[q] == rj) sj = q;
    }
#pragma unroll
    for (int r = 0; r < 2; r++) {
      const double wr = L.w[r];
#pragma unroll
      for (int a = 0; a < 6; a++) {  // ba_cuda.cu:352-370
        if (si >= 0) Ev[6 * si + a] -= wr * L.Jz[r] * L.Ji[r][a];
        if (sj >= 0) Ev[6 * sj + a] += wr * L.Jz[r] * L.Jj[r][a];
      }
      C += wr * L.Jz[r] * L.Jz[r];  // :372-373
      uu += wr * L.r[r] * L.Jz[r];
    }
  }
  w.Qp[u] = 1.0 / (C + (double)lmbda[0]);  // :519
  w.up[u] = uu;
}

// wave per nonzero lower block of S: 36 entries (+ y of the pose for a
// diagonal block), fixed item order per lane + butterfly sum
constexpr int kBlkWaves = 4;
__global__ void __launch_bounds__(kBlkWaves* kWave)
    k_block(const int64_t* __restrict__ ii, const int64_t* __restrict__ jj, int t0, int N, Ws w) {
  const int lane = threadIdx.x & 63;
  const int b = blockIdx.x * kBlkWaves + (int)(threadIdx.x >> 6);
  if (b >= w.meta->nblk) return;
  const int2 ab = w.bab[b];
  const int A = ab.x, Bp = ab.y;
  const bool diag = A == Bp;
  double acc[42];
#pragma unroll
  for (int k = 0; k < 42; k++) acc[k] = 0.0;
  const int q1 = w.boff[b + 1];
  for (int q = w.boff[b] + lane; q < q1; q += kWave) {
    const uint32_t v = w.ival2[q];
    const int u = (int)(v >> 10), sa = (int)((v >> 5) & 31), sb = (int)(v & 31);
    if (!w.own[u]) continue;
    const double Qu = w.Qp[u];
    const double* Eb0 = w.Ev + 6 * (size_t)w.psoff[u];
    double ea[6], eb[6];
#pragma unroll
    for (int k = 0; k < 6; k++) {
      ea[k] = Eb0[6 * sa + k];
      eb[k] = Eb0[6 * sb + k];
    }
#pragma unroll
    for (int r = 0; r < 6; r++)
#pragma unroll
      for (int c = 0; c < 6; c++) acc[6 * r + c] -= ea[r] * Qu * eb[c];
    if (diag) {
      const double uq = w.up[u];
#pragma unroll
      for (int r = 0; r < 6; r++) acc[36 + r] -= ea[r] * Qu * uq;
    }
    const int p1 = w.poff[u + 1];
    for (int p = w.poff[u]; p < p1; p++) {
      const int e = (int)w.pval2[p];
      const int64_t ri = ii[e] - t0, rj = jj[e] - t0;
      const bool fi = ri == A || (!diag && ri == Bp), fj = rj == A || (!diag && rj == Bp);
      if (!(fi || fj)) continue;
      const float* rec = w.J + 32 * (size_t)p;
#pragma unroll
      for (int r = 0; r < 2; r++) {
        const double wr = rec[r], rr = rec[2 + r];
        const float* Ji = rec + 6 + 6 * r;
        const float* Jj = rec + 18 + 6 * r;
        if (diag) {
          if (ri == A) {
#pragma unroll
            for (int x = 0; x < 6; x++) {
#pragma unroll
              for (int y = 0; y < 6; y++) acc[6 * x + y] += wr * Ji[x] * Ji[y];
              acc[36 + x] -= wr * rr * Ji[x];
            }
          }
          if (rj == A) {
#pragma unroll
            for (int x = 0; x < 6; x++) {
#pragma unroll
              for (int y = 0; y < 6; y++) acc[6 * x + y] += wr * Jj[x] * Jj[y];
              acc[36 + x] += wr * rr * Jj[x];
            }
          }
          if (ri == A && rj == A) {
#pragma unroll
            for (int x = 0; x < 6; x++)
#pragma unroll
              for (int y = 0; y < 6; y++)
                acc[6 * x + y] -= wr * Ji[x] * Jj[y] + wr * Jj[x] * Ji[y];
          }
        } else {
          if (ri == A && rj == Bp) {
#pragma unroll
            for (int x = 0; x < 6; x++)
#pragma unroll
              for (int y = 0; y < 6; y++) acc[6 * x + y] -= wr * Ji[x] * Jj[y];
          }
          if (rj == A && ri == Bp) {
#pragma unroll
            for (int x = 0; x < 6; x++)
#pragma unroll
              for (int y = 0; y < 6; y++) acc[6 * x + y] -= wr * Jj[x] * Ji[y];
          }
        }
      }
    }
  }
#pragma unroll
  for (int k = 0; k < 42; k++) {
    double x = acc[k];
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) x += __shfl_xor(x, o, 64);
    acc[k] = x;
  }
  // every lane holds all sums; lane k stores entry k
  double mine = 0.0;
#pragma unroll
  for (int k = 0; k < 42; k++)
    if (lane == k) mine = acc[k];
  if (lane < 36) S_of(w, N)[36 * (size_t)b + lane] = mine;
  else if (diag && lane < 42) y_of(w)[6 * A + (lane - 36)] = mine;
}

__global__ void k_zero_y(int N, Ws w) {
  const int q = blockIdx.x * blockDim.x + threadIdx.x;
  if (q < 6 * N) y_of(w)[q] = 0.0;
}

// zero the superblock system (extent from the device-side structure) and
// put 1 on every diagonal entry (poses without any block, padding rows)
__global__ void k_sys_clear(Ws w) {
  const Meta* meta = w.meta;
  const int nsb = meta->nsb, m = meta->m, nb6 = 6 * meta->nB, nr = 1 + nb6;
  const size_t nD = (size_t)nsb * m * m, nR = (size_t)nsb * m * nr, nC = (size_t)nb6 * nb6;
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  for (size_t q = blockIdx.x * (size_t)blockDim.x + threadIdx.x; q < nD; q += stride) {
    const size_t r = (q / m) % m, c = q % m;
    w.D[q] = r == c ? 1.0 : 0.0;
    w.Lo0[q] = 0.0;
  }
  for (size_t q = blockIdx.x * (size_t)blockDim.x + threadIdx.x; q < nR; q += stride) {
    w.R[q] = 0.0;
    w.BT[q] = 0.0;
  }
  for (size_t q = blockIdx.x * (size_t)blockDim.x + threadIdx.x; q < nC; q += stride)
    w.Cb[q] = (q / nb6 == q % nb6) ? 1.0 : 0.0;
}

// damped blocks into the superblock system: wave per block, lane per entry
__global__ void __launch_bounds__(256) k_assemble(int N, Ws w) {
  const int lane = threadIdx.x & 63;
  const int b = blockIdx.x * 4 + (int)(threadIdx.x >> 6);
  const Meta* meta = w.meta;
  if (b >= meta->nblk || lane >= 36 || (meta->status & kStBorder)) return;
  const int g = meta->g, m = meta->m, nr = 1 + 6 * meta->nB;
  const int2 ab = w.bab[b];
  const int r = lane / 6, c = lane % 6;
  double s = S_of(w, N)[36 * (size_t)b + lane];
  if (ab.x == ab.y && r == c) s += 1e-4 * s + 1.0;  // ba_cuda.cu:560
  const int ca = w.cidx[ab.x], cb = w.cidx[ab.y];
  if (ca >= 0 && cb >= 0) {
    const int sa = ca / g, sb = cb / g;
    const int ra = (ca % g) * 6 + r, rb = (cb % g) * 6 + c;
    if (sa == sb) {
      double* Dk = w.D + (size_t)sa * m * m;
      Dk[(size_t)ra * m + rb] = s;
      if (ab.x != ab.y) Dk[(size_t)rb * m + ra] = s;
    } else {  // sa == sb + 1 by construction: L_sb = A[sb + 1, sb]
      w.Lo0[(size_t)sb * m * m + (size_t)ra * m + rb] = s;
    }
  } else if (ca >= 0 || cb >= 0) {
    // interior row, border column: BT[sb][row][col] = S[interior, border]
    const bool ai = ca >= 0;
    const int ci = ai ? ca : cb;
    const int bcol = 6 * (ai ? w.bidx[ab.y] : w.bidx[ab.x]) + (ai ? c : r);
    const int irow = (ci % g) * 6 + (ai ? r : c);
    const size_t q = (size_t)(ci / g) * m * nr + (size_t)irow * nr + 1 + bcol;
    w.BT[q] = s;
    w.R[q] = s;
  } else {
    const int nb6 = 6 * meta->nB;
    const int ba = 6 * w.bidx[ab.x] + r, bb = 6 * w.bidx[ab.y] + c;
    w.Cb[(size_t)ba * nb6 + bb] = s;
    if (ab.x != ab.y) w.Cb[(size_t)bb * nb6 + ba] = s;
  }
}

__global__ void k_assemble_y(int N, Ws w) {
  const int q = blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= 6 * N) return;
  const Meta* meta = w.meta;
  if (meta->status & kStBorder) return;
  const int a = q / 6, r = q % 6, g = meta->g, m = meta->m, nr = 1 + 6 * meta->nB;
  const double v = y_of(w)[q];
  const int ca = w.cidx[a];
  if (ca >= 0) {
    w.R[(size_t)(ca / g) * m * nr + (size_t)((ca % g) * 6 + r) * nr] = v;
  } else {
    w.rb[6 * w.bidx[a] + r] = v;
  }
}

// ------------------------------------------------- dense workgroup helpers
// In-place Gauss-Jordan inverse of an SPD n x n matrix (row stride lda), no
// pivoting; colk/rowk: 2 n scratch doubles (LDS).  Returns false if a pivot
// was not positive (the matrix is then garbage; callers discard the step).
__device__ bool wg_gj_inverse(double* A, int n, int lda, double* colk, double* rowk) {
  __shared__ int bad;
  const int tid = threadIdx.x, nt = blockDim.x;
  if (tid == 0) bad = 0;
  for (int k = 0; k < n; k++) {
    __syncthreads();
    for (int i = tid; i < n; i += nt) {
      colk[i] = A[(size_t)i * lda + k];
      rowk[i] = A[(size_t)k * lda + i];
    }
    __syncthreads();
    const double p = colk[k];
    if (!(p > 0.0)) {
      if (tid == 0) bad = 1;
    }
    const double ip = p > 0.0 ? 1.0 / p : 0.0;
    for (int q = tid; q < n * n; q += nt) {
      const int i = q / n, j = q % n;
      double* a = A + (size_t)i * lda + j;
      if (i != k && j != k) *a -= colk[i] * rowk[j] * ip;
      else if (i == k && j != k) *a = rowk[j] * ip;
      else if (i != k) *a = -colk[i] * ip;
      else *a = ip;
    }
  }
  __syncthreads();
  return bad == 0;
}

// Superblock kernels.  Each level of the reduction is a few launches whose
// workgroups do ONE round trip to HBM each: every operand a workgroup needs
// (an m x m factor, a 32-column panel) is loaded into LDS at once, then the
// work runs from LDS and registers.  kMaxM <= 96.
//   k_cr_inv   one 1024-thread workgroup per eliminated superblock: D^-1 in
//              place (register Gauss-Jordan, 32 x 32 threads x 3 x 3 entries)
//   k_cr_mul   (superblock, 32-column panel): Y1 = D^-1 A[o,l], Y2 = D^-1 A[o,r],
//              Z = D^-1 R_o
//   k_cr_b     (kept superblock, panel): Schur updates of D_e, R_e and the new
//              coupling
//   k_cr_back  (eliminated superblock, panel): x_o = Z_o - Y1 x_l - Y2 x_r
constexpr int kTB = 1024;
constexpr int kPW = 32;                        // panel width (columns)
constexpr int kPanelsM = (kMaxM + kPW - 1) / kPW;
constexpr int kPanelsR = (1 + kMaxNB6 + kPW - 1) / kPW;
static_assert(kMaxM <= 96, "register Gauss-Jordan tiles 96 x 96");

// --- one-round-trip panel products (1024 threads: tc = tid % 32 column,
// tr = tid / 32 row group, rows tr + 32 a, a < kRA)
constexpr int kPT = 1024;
constexpr int kRG = kPT / 32;                  // row groups
constexpr int kRA = (kMaxM + kRG - 1) / kRG;   // rows per thread
// Global -> LDS staging with the loads of 8 elements per thread issued back to
// back before any is waited on (a plain load/store loop waits once per element:
// one HBM round trip each).  src(q) gives the value of LDS element q.
// Every load is unconditional (index clamped into range, value selected
// afterwards): a conditional load compiles to a branch with its own wait.
template <typename F>
__device__ __forceinline__ void stage(double* dst, int total, F src) {
  const int nt = blockDim.x;
  for (int base = threadIdx.x; base < total; base += 8 * nt) {
    double v[8];
#pragma unroll
    for (int u = 0; u < 8; u++) v[u] = src(min(base + u * nt, total - 1));
#pragma unroll
    for (int u = 0; u < 8; u++) {
      const int q = base + u * nt;
      if (q < total) dst[q] = v[u];
    }
  }
}
// As <- op(A) (M x K, row stride K): A row-major (lda) or, with trans, A^T
// where A is stored K x M.  Loads only: the caller syncs.
__device__ __forceinline__ void stage_a(const double* A, int lda, bool trans, int M, int K,
                                        double* As) {
  stage(As, M * K, [&](int q) {
    const int r = q / K, k = q - r * K;
    return A[trans ? (size_t)k * lda + r : (size_t)r * lda + k];
  });
}
// Bs <- columns [c0, c0 + nc) of B (K x *, row-major ldb) or of B^T (B stored
// * x K) as K x kPW (zero-padded).  Loads only.
__device__ __forceinline__ void stage_b(const double* B, int ldb, bool trans, int K, int c0, int nc,
                                        double* Bs) {
  stage(Bs, K * kPW, [&](int q) {
    const int k = q / kPW, c = q - k * kPW, cc = min(c, nc - 1);
    const double v = B[trans ? (size_t)(c0 + cc) * ldb + k : (size_t)k * ldb + c0 + cc];
    return c < nc ? v : 0.0;
  });
}
// s[a] = sum_k As[r_a][k] Bs[k][tc], r_a = tr + kRG a, k ascending; K even.
// Branch-free: rows past M read row M - 1 (their sums are never stored); a
// row guard here compiles to one exec-masked block per row, each waiting on
// its own LDS read.
__device__ __forceinline__ void panel_dot(const double* As, int M, int K, const double* Bs,
                                          double s[kRA]) {
  const int tc = threadIdx.x & (kPW - 1), tr = threadIdx.x >> 5;
  const double* arow[kRA];
#pragma unroll
  for (int a = 0; a < kRA; a++) {
    s[a] = 0.0;
    arow[a] = As + min(tr + kRG * a, M - 1) * K;
  }
  for (int k = 0; k < K; k += 2) {
    const double b0 = Bs[k * kPW + tc], b1 = Bs[(k + 1) * kPW + tc];
#pragma unroll
    for (int a = 0; a < kRA; a++) {
      const double2 av = *reinterpret_cast<const double2*>(arow[a] + k);
      s[a] += av.x * b0;
      s[a] += av.y * b1;
    }
  }
}
// C[rows, c0 + tc] = (acc ? C : 0) (+ alpha * s1 if use1) (+ alpha * s2 if use2)
__device__ __forceinline__ void panel_store(double* C, int ldc, int M, int c0, int nc, double alpha,
                                            bool acc, const double (&s1)[kRA], bool use1,
                                            const double (&s2)[kRA], bool use2) {
  const int tc = threadIdx.x & (kPW - 1), tr = threadIdx.x >> 5;
  if (tc >= nc) return;
#pragma unroll
  for (int a = 0; a < kRA; a++) {
    const int r = tr + kRG * a;
    if (r < M) {
      double* cp = C + (size_t)r * ldc + c0 + tc;
      double v = acc ? *cp : 0.0;
      if (use1) v += alpha * s1[a];
      if (use2) v += alpha * s2[a];
      *cp = v;
    }
  }
}

// C[M x N] (ldc) = (acc ? C : 0) + alpha * A^T B with A stored [K x M] (lda),
// B [K x N] (ldb), K <= kMaxM: 64 x 64 output tiles, each with ONE staging
// round trip of its full-K operands; 256 threads, 4 x 4 outputs each.
constexpr int kTM = 64, kTN = 64;
__device__ void wg_gemm_tn(double* C, int ldc, const double* A, int lda, const double* B, int ldb,
                           int M, int N, int K, double alpha, bool acc, double* As, double* Bs) {
  const int tid = threadIdx.x;
  const int tr = tid / 16, tc = tid % 16;
  for (int i0 = 0; i0 < M; i0 += kTM)
    for (int j0 = 0; j0 < N; j0 += kTN) {
      __syncthreads();
      stage(As, K * kTM, [&](int q) {
        const int k = q / kTM, i = q % kTM;
        const double v = A[(size_t)k * lda + min(i0 + i, M - 1)];
        return (i0 + i < M) ? v : 0.0;
      });
      stage(Bs, K * kTN, [&](int q) {
        const int k = q / kTN, j = q % kTN;
        const double v = B[(size_t)k * ldb + min(j0 + j, N - 1)];
        return (j0 + j < N) ? v : 0.0;
      });
      __syncthreads();
      double s[4][4];
#pragma unroll
      for (int a = 0; a < 4; a++)
#pragma unroll
        for (int b = 0; b < 4; b++) s[a][b] = 0.0;
      for (int k = 0; k < K; k++) {
        double av[4], bv[4];
#pragma unroll
        for (int a = 0; a < 4; a++) av[a] = As[k * kTM + tr + 16 * a];
#pragma unroll
        for (int b = 0; b < 4; b++) bv[b] = Bs[k * kTN + tc + 16 * b];
#pragma unroll
        for (int a = 0; a < 4; a++)
#pragma unroll
          for (int b = 0; b < 4; b++) s[a][b] += av[a] * bv[b];
      }
#pragma unroll
      for (int a = 0; a < 4; a++)
#pragma unroll
        for (int b = 0; b < 4; b++) {
          const int gi = i0 + tr + 16 * a, gj = j0 + tc + 16 * b;
          if (gi < M && gj < N) {
            double* cp = C + (size_t)gi * ldc + gj;
            *cp = (acc ? *cp : 0.0) + alpha * s[a][b];
          }
        }
    }
  __syncthreads();
}

// LDS of the GJ kernels: inverse (kMaxM^2) | GJ vectors
inline size_t gj_lds_bytes() { return sizeof(double) * ((size_t)kMaxM * kMaxM + kBgjDoubles); }
// LDS of the panel kernels: A (kMaxM^2) | B panel (kMaxM x kPW)
constexpr size_t kPanelLds = sizeof(double) * ((size_t)kMaxM * kMaxM + (size_t)kMaxM * kPW);
// k_cr_b / k_cr_back stage both products' operands at once when they fit
constexpr size_t kPanelLds2 = 160 * 1024;
// (layout: A at 0, B at kMaxM^2, second A / B right after the first B)
__device__ __forceinline__ bool two_fit(int m) {
  return sizeof(double) * ((size_t)kMaxM * kMaxM + (size_t)m * m + 2 * (size_t)m * kPW) <=
         kPanelLds2;
}

// ------------------------------------------------- block cyclic reduction
// Level lev: active superblocks are k * 2^lev, k < n.  Odd k are eliminated.
// top: the last remaining superblock (index 0) at the end.
// Grids are sized by the host's bound and capped (kCrGrid); workgroups loop
// over the level's real items, so a level costs no empty-workgroup rounds.
constexpr int kCrGrid = 256;
__device__ __forceinline__ int cr_nelim(const Meta* meta, int lev, bool top) {
  if (top) return meta->nsb >= 1 ? 1 : 0;
  const int n = level_count(meta->nsb, lev);
  return n > 1 ? n / 2 : 0;
}
__device__ __forceinline__ int cr_nkept(const Meta* meta, int lev) {
  const int n = level_count(meta->nsb, lev);
  return n > 1 ? (n + 1) / 2 : 0;
}

__global__ void __launch_bounds__(kTB) k_cr_inv(int lev, int top, Ws w) {
  extern __shared__ __attribute__((aligned(16))) double lds[];
  Meta* meta = w.meta;
  const int cnt = cr_nelim(meta, lev, top), m = meta->m;
  for (int it = blockIdx.x; it < cnt; it += gridDim.x) {
    const int k = top ? 0 : 2 * it + 1, o = k << lev;
    double* D = w.D + (size_t)o * m * m;
    if (!wg_bgj_inverse(D, m, m, D, lds)) {  // in place: D_o is not read again
      if (threadIdx.x == 0) atomicOr(&meta->status, kStChol);
    }
  }
}

// grid (panel, superblock): panels [0, kPanelsM) -> Y1, [kPanelsM, 2 kPanelsM)
// -> Y2, then kPanelsR panels of R_o (in place).
__global__ void __launch_bounds__(kPT) k_cr_mul(int lev, int top, Ws w, const double* Lcur) {
  extern __shared__ __attribute__((aligned(16))) double lds[];
  const Meta* meta = w.meta;
  const int cnt = cr_nelim(meta, lev, top) * (2 * kPanelsM + kPanelsR);
  const int m = meta->m, nr = 1 + 6 * meta->nB, st = 1 << lev;
  const int n = level_count(meta->nsb, lev);
  const size_t mm = (size_t)m * m;
  double* As = lds;
  double* Bs = As + kMaxM * kMaxM;
  for (int it = blockIdx.x; it < cnt; it += gridDim.x) {
    const int e = it / (2 * kPanelsM + kPanelsR);
    int pnl = it - e * (2 * kPanelsM + kPanelsR), seg;
    const int k = top ? 0 : 2 * e + 1, o = k * st, l = (k - 1) * st;
    const bool has_r = !top && k + 1 < n;
    if (pnl < kPanelsM) seg = 0;
    else if (pnl < 2 * kPanelsM) seg = 1, pnl -= kPanelsM;
    else seg = 2, pnl -= 2 * kPanelsM;
    const int c0 = pnl * kPW, ncol = seg == 2 ? nr : m;
    if (c0 >= ncol || (top && seg < 2) || (seg == 1 && !has_r)) continue;  // block-uniform
    const int nc = min(kPW, ncol - c0);
    __syncthreads();
    stage_a(w.D + o * mm, m, false, m, m, As);  // D_o^-1
    double* Ro = w.R + (size_t)o * m * nr;
    if (seg == 0) stage_b(Lcur + l * mm, m, false, m, c0, nc, Bs);       // A[o, l] = L[l]
    else if (seg == 1) stage_b(Lcur + o * mm, m, true, m, c0, nc, Bs);   // A[o, r] = L[o]^T
    else stage_b(Ro, nr, false, m, c0, nc, Bs);
    __syncthreads();
    double s[kRA];
    panel_dot(As, m, m, Bs, s);
    if (seg == 0) panel_store(w.Y1 + o * mm, m, m, c0, nc, 1.0, false, s, true, s, false);
    else if (seg == 1) panel_store(w.Y2 + o * mm, m, m, c0, nc, 1.0, false, s, true, s, false);
    else panel_store(Ro, nr, m, c0, nc, 1.0, false, s, true, s, false);
  }
}

// grid (panel, kept superblock): [D_e | R_e | L'_e] column panels.
//   D_e -= L[ol] Y2[ol] + L[e]^T Y1[or];  R_e -= L[ol] R[ol] + L[e]^T R[or]
//   L'_e = -L[or] Y1[or]  (new coupling A'[r2, e])
__global__ void __launch_bounds__(kPT) k_cr_b(int lev, Ws w, const double* Lcur, double* Lnext) {
  extern __shared__ __attribute__((aligned(16))) double lds[];
  const Meta* meta = w.meta;
  constexpr int kP = 2 * kPanelsM + kPanelsR;
  const int n = level_count(meta->nsb, lev), cnt = cr_nkept(meta, lev) * kP;
  const int m = meta->m, nr = 1 + 6 * meta->nB, st = 1 << lev;
  const size_t mm = (size_t)m * m, mr = (size_t)m * nr;
  double* As = lds;
  double* Bs = As + kMaxM * kMaxM;
  for (int it = blockIdx.x; it < cnt; it += gridDim.x) {
    const int kq = it / kP;
    int pnl = it - kq * kP, seg;
    const int k = 2 * kq, e = k * st;
    const bool has_l = k >= 1, has_r = k + 1 < n, has_r2 = k + 2 < n;
    const int ol = (k - 1) * st, orr = (k + 1) * st;
    if (pnl < kPanelsM) seg = 0;
    else if (pnl < kPanelsM + kPanelsR) seg = 1, pnl -= kPanelsM;
    else seg = 2, pnl -= kPanelsM + kPanelsR;
    const int c0 = pnl * kPW, ncol = seg == 1 ? nr : m;
    if (c0 >= ncol || (seg == 2 && !has_r2) || (!has_l && !has_r)) continue;  // block-uniform
    const int nc = min(kPW, ncol - c0);
    double s1[kRA], s2[kRA];
    __syncthreads();
    if (seg == 2) {
      stage_a(Lcur + orr * mm, m, false, m, m, As);
      stage_b(w.Y1 + orr * mm, m, false, m, c0, nc, Bs);
      __syncthreads();
      panel_dot(As, m, m, Bs, s1);
      panel_store(Lnext + e * mm, m, m, c0, nc, -1.0, false, s1, true, s1, false);
      continue;
    }
    double* C = seg == 0 ? w.D + e * mm : w.R + e * mr;
    const int ldc = seg == 0 ? m : nr;
    // A[e, ol] = L[ol] (B: Y2[ol] | R[ol]); A[e, or] = L[e]^T (B: Y1[or] | R[or])
    const double* B1 = seg == 0 ? w.Y2 + ol * mm : w.R + ol * mr;
    const double* B2 = seg == 0 ? w.Y1 + orr * mm : w.R + orr * mr;
    const int ldb = seg == 0 ? m : nr;
    if (has_l && has_r && two_fit(m)) {  // one round trip for both products
      double* As2 = Bs + m * kPW;
      double* Bs2 = As2 + m * m;
      stage_a(Lcur + ol * mm, m, false, m, m, As);
      stage_b(B1, ldb, false, m, c0, nc, Bs);
      stage_a(Lcur + e * mm, m, true, m, m, As2);
      stage_b(B2, ldb, false, m, c0, nc, Bs2);
      __syncthreads();
      panel_dot(As, m, m, Bs, s1);
      panel_dot(As2, m, m, Bs2, s2);
    } else {
      if (has_l) {
        stage_a(Lcur + ol * mm, m, false, m, m, As);
        stage_b(B1, ldb, false, m, c0, nc, Bs);
        __syncthreads();
        panel_dot(As, m, m, Bs, s1);
      }
      if (has_r) {
        __syncthreads();
        stage_a(Lcur + e * mm, m, true, m, m, As);
        stage_b(B2, ldb, false, m, c0, nc, Bs);
        __syncthreads();
        panel_dot(As, m, m, Bs, s2);
      }
    }
    panel_store(C, ldc, m, c0, nc, -1.0, true, s1, has_l, s2, has_r);
  }
}

// grid (panel of R, eliminated superblock): x_o = Z_o - Y1 x_l - Y2 x_r
__global__ void __launch_bounds__(kPT) k_cr_back(int lev, Ws w) {
  extern __shared__ __attribute__((aligned(16))) double lds[];
  const Meta* meta = w.meta;
  const int n = level_count(meta->nsb, lev), cnt = cr_nelim(meta, lev, false) * kPanelsR;
  const int m = meta->m, nr = 1 + 6 * meta->nB, st = 1 << lev;
  const size_t mm = (size_t)m * m, mr = (size_t)m * nr;
  double* As = lds;
  double* Bs = As + kMaxM * kMaxM;
  for (int it = blockIdx.x; it < cnt; it += gridDim.x) {
    const int e = it / kPanelsR, c0 = (it - e * kPanelsR) * kPW;
    if (c0 >= nr) continue;  // block-uniform
    const int nc = min(kPW, nr - c0);
    const int k = 2 * e + 1, o = k * st, l = (k - 1) * st, r = (k + 1) * st;
    double s1[kRA], s2[kRA];
    __syncthreads();
    const bool has_r = k + 1 < n;
    if (has_r && two_fit(m)) {  // one round trip for both products
      double* As2 = Bs + m * kPW;
      double* Bs2 = As2 + m * m;
      stage_a(w.Y1 + o * mm, m, false, m, m, As);
      stage_b(w.R + l * mr, nr, false, m, c0, nc, Bs);
      stage_a(w.Y2 + o * mm, m, false, m, m, As2);
      stage_b(w.R + r * mr, nr, false, m, c0, nc, Bs2);
      __syncthreads();
      panel_dot(As, m, m, Bs, s1);
      panel_dot(As2, m, m, Bs2, s2);
    } else {
      stage_a(w.Y1 + o * mm, m, false, m, m, As);
      stage_b(w.R + l * mr, nr, false, m, c0, nc, Bs);
      __syncthreads();
      panel_dot(As, m, m, Bs, s1);
      if (has_r) {
        __syncthreads();
        stage_a(w.Y2 + o * mm, m, false, m, m, As);
        stage_b(w.R + r * mr, nr, false, m, c0, nc, Bs);
        __syncthreads();
        panel_dot(As, m, m, Bs, s2);
      }
    }
    panel_store(w.R + o * mr, nr, m, c0, nc, -1.0, true, s1, true, s2, has_r);
  }
}

// border Schur complement [Sb | rb] = [Cb | yB] - BT^T [X | z0], in two
// passes: workgroup g sums BT_sb^T [X_sb | z0_sb] over sb = g, g + kBP, ...
// into its own partial (no atomics), then a fixed-order sum over the groups.
__global__ void __launch_bounds__(256) k_border_part(Ws w) {
  extern __shared__ __attribute__((aligned(16))) double lds[];
  const Meta* meta = w.meta;
  const int nB = meta->nB, nsb = meta->nsb, m = meta->m;
  if (nB == 0 || nB > kMaxBorder) return;
  const int nb6 = 6 * nB, nr = 1 + nb6, g = blockIdx.x;
  double* part = w.Pb + (size_t)g * nb6 * nr;
  for (int sb = g; sb < nsb; sb += kBP) {
    const double* bt = w.BT + (size_t)sb * m * nr + 1;  // [m][nr], border columns 1..nb6
    const double* x = w.R + (size_t)sb * m * nr;
    wg_gemm_tn(part, nr, bt, nr, x, nr, nb6, nr, m, 1.0, sb != g, lds, lds + kMaxM * kTM);
  }
}

__global__ void k_border_reduce(Ws w) {
  const Meta* meta = w.meta;
  const int nB = meta->nB;
  if (nB == 0 || nB > kMaxBorder) return;
  const int nb6 = 6 * nB, nr = 1 + nb6, ng = min(meta->nsb, kBP);
  const int q = blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= nb6 * nr) return;
  const int r = q / nr, c = q % nr;  // c == 0: rhs, c >= 1: Sb column c - 1
  double s = 0.0;
#pragma unroll 8
  for (int g = 0; g < ng; g++) s += w.Pb[(size_t)g * nb6 * nr + q];
  if (c == 0) w.rb[r] -= s;
  else w.Cb[(size_t)r * nb6 + c - 1] -= s;
}

// dense border solve: register Gauss-Jordan for 6 nB <= kMaxM, else in place in HBM
__global__ void __launch_bounds__(kTB) k_border_solve(Ws w) {
  extern __shared__ __attribute__((aligned(16))) double lds[];
  Meta* meta = w.meta;
  const int nB = meta->nB;
  if (nB == 0 || nB > kMaxBorder) return;
  const int nb6 = 6 * nB;
  double* rb = lds + kMaxM * kMaxM + kBgjDoubles;
  const double* inv;
  bool ok;
  if (nb6 <= kMaxM) {
    for (int q = threadIdx.x; q < nb6; q += blockDim.x) rb[q] = w.rb[q];
    ok = wg_bgj_inverse(w.Cb, nb6, nb6, lds, lds + kMaxM * kMaxM);
    inv = lds;
  } else {
    ok = wg_gj_inverse(w.Cb, nb6, nb6, lds, lds + nb6);
    for (int q = threadIdx.x; q < nb6; q += blockDim.x) rb[q] = w.rb[q];
    __syncthreads();
    inv = w.Cb;
  }
  if (!ok && threadIdx.x == 0) atomicOr(&meta->status, kStChol);
  for (int r = threadIdx.x; r < nb6; r += blockDim.x) {
    double s = 0.0;
    for (int k = 0; k < nb6; k++) s += inv[(size_t)r * nb6 + k] * rb[k];
    w.dXB[r] = s;
  }
}

// dX in pose order: interior x = z0 - X dXB; border dXB.  Failed solve -> 0.
__global__ void __launch_bounds__(256) k_final_dx(int N, Ws w) {
  __shared__ double xb[kMaxNB6];
  const Meta* meta = w.meta;
  const int nB = min(meta->nB, kMaxBorder);
  for (int c = threadIdx.x; c < 6 * nB; c += blockDim.x) xb[c] = w.dXB[c];
  __syncthreads();
  const int q = blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= 6 * N) return;
  if (meta->status & (kStChol | kStBorder)) {
    w.dX[q] = 0.0;
    return;
  }
  const int a = q / 6, rr = q % 6, g = meta->g, m = meta->m, nr = 1 + 6 * nB;
  double v;
  const int ca = w.cidx[a];
  if (ca >= 0) {
    const double* x = w.R + (size_t)(ca / g) * m * nr + (size_t)((ca % g) * 6 + rr) * nr;
    v = x[0];
    for (int c = 0; c < 6 * nB; c++) v -= x[1 + c] * xb[c];
  } else {
    v = xb[6 * w.bidx[a] + rr];
  }
  w.dX[q] = v;
}

// pose retraction (threads < N) and patch depth update (owned patches)
__global__ void k_update(float* __restrict__ poses, float* __restrict__ patches, int E, int P,
                         int t0, int N, Ws w) {
  const int q = blockIdx.x * blockDim.x + threadIdx.x;
  if (q < N) {  // pose_retr_kernel (ba_cuda.cu:178-206)
    float* pt = poses + 7 * (size_t)(t0 + q);
    float xi[6], t1v[3], q1v[4];
#pragma unroll
    for (int a = 0; a < 6; a++) xi[a] = (float)w.dX[6 * q + a];
    retrSE3(xi, pt, pt + 3, t1v, q1v);
    pt[0] = t1v[0];
    pt[1] = t1v[1];
    pt[2] = t1v[2];
    pt[3] = q1v[0];
    pt[4] = q1v[1];
    pt[5] = q1v[2];
    pt[6] = q1v[3];
    return;
  }
  const int u = q - N;
  if (u >= E || u >= w.meta->nuniq || !w.own[u]) return;
  double s = w.up[u];  // dZ = Q (u - E^T dX) (:563); structure only: Q u
  if (N > 0) {
    const int ns = w.pscnt[u];
    const int* set = w.psetf + (size_t)u * kMaxSet;
    const double* Ev = w.Ev + 6 * (size_t)w.psoff[u];
    for (int t = 0; t < ns; t++)
      for (int a = 0; a < 6; a++) s -= Ev[6 * t + a] * w.dX[6 * set[t] + a];
  }
  const double dz = w.Qp[u] * s;
  float* pk = patches + (size_t)w.pkk[u] * 3 * P * P + 2 * P * P;  // patch_retr_kernel :209-229
  float d = pk[0];
  d = d + (float)dz;
  d = (d > 20) ? 1.0f : d;
  d = (float)fmax((double)d, 1e-4);
  for (int a = 0; a < P * P; a++) pk[a] = d;
}

__global__ void k_status_out(const Ws w, int* out) {
  if (threadIdx.x == 0 && blockIdx.x == 0) {
    const Meta* m = w.meta;
    out[0] = m->status;
    out[1] = m->nuniq;
    out[2] = m->nitems;
    out[3] = m->nblk;
    out[4] = m->nI;
    out[5] = m->nB;
    out[6] = m->g;
    out[7] = m->nsb;
  }
}

__global__ void k_status_or_out(const Ws w, int* acc) {
  if (threadIdx.x == 0 && blockIdx.x == 0) atomicOr(acc, w.meta->status);
}

__global__ void k_clear_chol(Ws w) {
  if (threadIdx.x == 0 && blockIdx.x == 0) w.meta->status &= ~kStChol;
}

inline int grid_of(long long n, int t = kT) { return (int)std::max<long long>(1, (n + t - 1) / t); }

inline int cr_levels(int N) {
  int n = N, L = 0;
  while (n > 1) {
    n = (n + 1) >> 1;
    L++;
  }
  return L;
}

static void ensure_attrs() {
  static bool done = false;
  if (done) return;
  for (const void* f : {(const void*)k_cr_inv, (const void*)k_border_solve})
    (void)hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize,
                              (int)(gj_lds_bytes() + sizeof(double) * kMaxNB6));
  for (const void* f : {(const void*)k_cr_mul, (const void*)k_border_part})
    (void)hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, (int)kPanelLds);
  for (const void* f : {(const void*)k_cr_b, (const void*)k_cr_back})
    (void)hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, (int)kPanelLds2);
  done = true;
}

}  // namespace gba

// ------------------------------------------------------------------ C ABI
using namespace gba;

size_t gba_workspace_bytes(int E, int N) { return layout(E, N, nullptr, nullptr); }

int gba_setup(const int64_t* ii, const int64_t* jj, const int64_t* kk, int E, int num_patches,
              int PPF, int t0, int t1, int own_lo, int own_hi, void* workspace,
              size_t workspace_bytes, void* stream) {
  const int N = t1 - t0;
  if (E <= 0) return DPVO_OK;
  if (!ii || !jj || !kk || !workspace || num_patches <= 0 || N < 0) return DPVO_ERR_INVALID;
  if (N > kMaxN || E > (1 << 22)) return DPVO_ERR_UNSUPPORTED;
  if (workspace_bytes < gba_workspace_bytes(E, N)) return DPVO_ERR_WORKSPACE;
  Ws w;
  layout(E, N, (char*)workspace, &w);
  hipStream_t s = as_stream(stream);
  const int IB = item_bound(E);
  hipLaunchKernelGGL(k_keys, dim3(grid_of(E)), dim3(kT), 0, s, kk, E, num_patches, w);
  size_t tb = w.tmp_bytes;
  const int pbits = key_bits(num_patches);
  if (rocprim::radix_sort_pairs(w.tmp, tb, w.pkey, w.pkey2, w.pval, w.pval2, (unsigned)E, 0, pbits,
                                s) != hipSuccess)
    return DPVO_ERR_LAUNCH;
  hipLaunchKernelGGL(k_pflag, dim3(grid_of(E)), dim3(kT), 0, s, E, w);
  tb = w.tmp_bytes;
  if (rocprim::inclusive_scan(w.tmp, tb, w.flag, w.scan, (size_t)E, rocprim::plus<int>(), s) !=
      hipSuccess)
    return DPVO_ERR_LAUNCH;
  hipLaunchKernelGGL(k_pscatter, dim3(grid_of(E)), dim3(kT), 0, s, E, w);
  hipLaunchKernelGGL(k_pset, dim3(grid_of(E)), dim3(kT), 0, s, ii, jj, E, t0, N, PPF, own_lo,
                     own_hi, w);
  tb = w.tmp_bytes;
  if (rocprim::exclusive_scan(w.tmp, tb, w.pscnt, w.psoff, 0, (size_t)E, rocprim::plus<int>(),
                              s) != hipSuccess)
    return DPVO_ERR_LAUNCH;
  tb = w.tmp_bytes;
  if (rocprim::exclusive_scan(w.tmp, tb, w.itcnt, w.itoff, 0, (size_t)E, rocprim::plus<int>(),
                              s) != hipSuccess)
    return DPVO_ERR_LAUNCH;
  hipLaunchKernelGGL(k_items, dim3(grid_of(E)), dim3(kT), 0, s, E, N, w);
  const long long maxkey = (long long)N * (N + 1) / 2;
  const int ibits = key_bits(maxkey);
  const uint32_t pad = (uint32_t)((1ull << ibits) - 1);
  hipLaunchKernelGGL(k_ipad, dim3(grid_of(IB)), dim3(kT), 0, s, IB, pad, w);
  tb = w.tmp_bytes;
  if (rocprim::radix_sort_pairs(w.tmp, tb, w.ikey, w.ikey2, w.ival, w.ival2, (unsigned)IB, 0,
                                ibits, s) != hipSuccess)
    return DPVO_ERR_LAUNCH;
  hipLaunchKernelGGL(k_bflag, dim3(grid_of(IB)), dim3(kT), 0, s, IB, w);
  tb = w.tmp_bytes;
  if (rocprim::inclusive_scan(w.tmp, tb, w.iflag, w.iscan, (size_t)IB, rocprim::plus<int>(), s) !=
      hipSuccess)
    return DPVO_ERR_LAUNCH;
  hipLaunchKernelGGL(k_bscatter, dim3(grid_of(IB)), dim3(kT), 0, s, IB, w);
  hipLaunchKernelGGL(k_structure, dim3(1), dim3(1024), 0, s, N, w);
  return launch_status();
}

int gba_build(const float* poses, const float* patches, const float* intrinsics,
              const float* target, const float* weight, const float* lmbda, const int64_t* ii,
              const int64_t* jj, int E, int P, int num_poses, int t0, int t1, void* workspace,
              void* stream) {
  const int N = t1 - t0;
  if (E <= 0) return DPVO_OK;
  Ws w;
  layout(E, N, (char*)workspace, &w);
  hipStream_t s = as_stream(stream);
  hipLaunchKernelGGL(k_clear_chol, dim3(1), dim3(64), 0, s, w);
  hipLaunchKernelGGL(k_lin, dim3(grid_of(E)), dim3(kT), 0, s, poses, patches, intrinsics, target,
                     weight, lmbda, ii, jj, E, P, num_poses, t0, N, w);
  if (N > 0) {
    hipLaunchKernelGGL(k_zero_y, dim3(grid_of(6 * N)), dim3(kT), 0, s, N, w);
    hipLaunchKernelGGL(k_block, dim3(grid_of(blk_bound(E, N), kBlkWaves)),
                       dim3(kBlkWaves * kWave), 0, s, ii, jj, t0, N, w);
  }
  return launch_status();
}

int gba_solve_update(float* poses, float* patches, int E, int P, int t0, int t1, void* workspace,
                     void* stream) {
  const int N = t1 - t0;
  if (E <= 0) return DPVO_OK;
  Ws w;
  layout(E, N, (char*)workspace, &w);
  ensure_attrs();
  hipStream_t s = as_stream(stream);
  if (N > 0) {
    hipLaunchKernelGGL(k_sys_clear, dim3(1024), dim3(kT), 0, s, w);
    hipLaunchKernelGGL(k_assemble, dim3(grid_of(blk_bound(E, N), 4)), dim3(256), 0, s, N, w);
    hipLaunchKernelGGL(k_assemble_y, dim3(grid_of(6 * N)), dim3(kT), 0, s, N, w);
    const int L = cr_levels(N);
    double* Lo[2] = {w.Lo0, w.Lo1};
    int n = N;  // upper bound of the superblock count at each level
    const size_t lg = gj_lds_bytes() + sizeof(double) * kMaxNB6;
    constexpr int kP = 2 * kPanelsM + kPanelsR;
    auto cap = [](long long v) { return (int)std::max(1LL, std::min<long long>(v, kCrGrid)); };
    for (int lev = 0; lev < L; lev++) {
      const int ne = n / 2, nk = (n + 1) / 2;
      hipLaunchKernelGGL(k_cr_inv, dim3(cap(ne)), dim3(kTB), lg, s, lev, 0, w);
      hipLaunchKernelGGL(k_cr_mul, dim3(cap((long long)ne * kP)), dim3(kPT), kPanelLds, s, lev, 0,
                         w, Lo[lev & 1]);
      hipLaunchKernelGGL(k_cr_b, dim3(cap((long long)nk * kP)), dim3(kPT), kPanelLds2, s, lev, w,
                         Lo[lev & 1], Lo[(lev + 1) & 1]);
      n = (n + 1) >> 1;
    }
    hipLaunchKernelGGL(k_cr_inv, dim3(1), dim3(kTB), lg, s, L, 1, w);
    hipLaunchKernelGGL(k_cr_mul, dim3(kP), dim3(kPT), kPanelLds, s, L, 1, w, Lo[L & 1]);
    n = N;
    int nl[32];
    for (int lev = 0; lev < L; lev++) {
      nl[lev] = n;
      n = (n + 1) >> 1;
    }
    for (int lev = L - 1; lev >= 0; lev--)
      hipLaunchKernelGGL(k_cr_back, dim3(cap((long long)(nl[lev] / 2) * kPanelsR)), dim3(kPT),
                         kPanelLds2, s, lev, w);
    hipLaunchKernelGGL(k_border_part, dim3(kBP), dim3(256), kPanelLds, s, w);
    hipLaunchKernelGGL(k_border_reduce, dim3(grid_of((long long)kMaxNB6 * (kMaxNB6 + 1))),
                       dim3(kT), 0, s, w);
    hipLaunchKernelGGL(k_border_solve, dim3(1), dim3(kTB), lg, s, w);
    hipLaunchKernelGGL(k_final_dx, dim3(grid_of(6 * N)), dim3(kT), 0, s, N, w);
  }
  hipLaunchKernelGGL(k_update, dim3(grid_of((long long)N + E)), dim3(kT), 0, s, poses, patches, E,
                     P, t0, N, w);
  return launch_status();
}

int gba_status_or(const void* workspace, int E, int N, int* acc, void* stream) {
  Ws w;
  layout(E, N, (char*)workspace, &w);
  hipLaunchKernelGGL(k_status_or_out, dim3(1), dim3(64), 0, as_stream(stream), w, acc);
  return launch_status();
}

int gba_status(const void* workspace, int E, int N, int* out, void* stream) {
  Ws w;
  layout(E, N, (char*)workspace, &w);
  hipLaunchKernelGGL(k_status_out, dim3(1), dim3(64), 0, as_stream(stream), w, out);
  return launch_status();
}

double* gba_dx(void* workspace, int E, int N) {
  Ws w;
  layout(E, N, (char*)workspace, &w);
  return w.dX;
}

double* gba_packed(void* workspace, int E, int N) {
  Ws w;
  layout(E, N, (char*)workspace, &w);
  return w.packed;
}

int gba_forward(float* poses, float* patches, const float* intrinsics, const float* target,
                const float* weight, const float* lmbda, const int64_t* ii, const int64_t* jj,
                const int64_t* kk, int E, int P, int num_poses, int num_patches, int PPF, int t0,
                int t1, int iterations, void* workspace, size_t workspace_bytes, void* stream) {
  int st = gba_setup(ii, jj, kk, E, num_patches, PPF, t0, t1, 0, 0x7fffffff, workspace,
                     workspace_bytes, stream);
  for (int it = 0; it < iterations && st == DPVO_OK; it++) {
    st = gba_build(poses, patches, intrinsics, target, weight, lmbda, ii, jj, E, P, num_poses, t0,
                   t1, workspace, stream);
    if (st == DPVO_OK) st = gba_solve_update(poses, patches, E, P, t0, t1, workspace, stream);
  }
  return st;
}

// ---------------------------------------------------------------- exports
static inline int gba_n(int t0, int t1) { return t1 > t0 ? t1 - t0 : 0; }

DPVO_EXPORT size_t dpvo_gba_workspace_bytes(int E, int t0, int t1) {
  return E > 0 ? gba_workspace_bytes(E, gba_n(t0, t1)) : 0;
}

DPVO_EXPORT int dpvo_gba_max_free_poses(void) { return kMaxN; }

DPVO_EXPORT int dpvo_gba_setup(const int64_t* ii, const int64_t* jj, const int64_t* kk, int E,
                               int num_patches, int PPF, int t0, int t1, int own_lo, int own_hi,
                               void* workspace, size_t workspace_bytes, void* stream) {
  if (t1 < t0) return DPVO_ERR_INVALID;
  return gba_setup(ii, jj, kk, E, num_patches, PPF, t0, t1, own_lo, own_hi, workspace,
                   workspace_bytes, stream);
}

DPVO_EXPORT int dpvo_gba_build(const float* poses, const float* patches, const float* intrinsics,
                               const float* target, const float* weight, const float* lmbda,
                               const int64_t* ii, const int64_t* jj, int E, int P, int num_poses,
                               int t0, int t1, void* workspace, void* stream) {
  if (E <= 0) return DPVO_OK;
  if (!poses || !patches || !intrinsics || !target || !weight || !lmbda || !ii || !jj ||
      !workspace || P < 2 || num_poses <= 0 || t1 < t0)
    return DPVO_ERR_INVALID;
  return gba_build(poses, patches, intrinsics, target, weight, lmbda, ii, jj, E, P, num_poses, t0,
                   t1, workspace, stream);
}

DPVO_EXPORT int dpvo_gba_solve_update(float* poses, float* patches, int E, int P, int t0, int t1,
                                      void* workspace, void* stream) {
  if (E <= 0) return DPVO_OK;
  if (!poses || !patches || !workspace || P < 2 || t1 < t0) return DPVO_ERR_INVALID;
  return gba_solve_update(poses, patches, E, P, t0, t1, workspace, stream);
}

DPVO_EXPORT int dpvo_gba_info(const void* workspace, int E, int t0, int t1, int* out,
                              void* stream) {
  if (!workspace || !out || E <= 0) return DPVO_ERR_INVALID;
  return gba_status(workspace, E, gba_n(t0, t1), out, stream);
}

DPVO_EXPORT size_t dpvo_gba_packed_offset(int E, int t0, int t1) {
  if (E <= 0) return 0;
  return (size_t)((char*)gba_packed((void*)4096, E, gba_n(t0, t1)) - (char*)4096);
}

}  // namespace dpvo
