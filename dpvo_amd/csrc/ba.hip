// ba.hip -- fastba on gfx950: F-BA (Schur bundle adjustment), F-REPROJ, F-NBR.
//
// Reference semantics: dpvo/fastba/ba_cuda.cu + block_e.cu + ba.cpp
// (cuteboyqq/DPVO).  One F-BA iteration (ba_cuda.cu:482-579):
//   per edge: residual + Jacobians (fp32, :265-333); B, E, C, v, u sums
//   Q = 1/(C+lmbda); S = B - E Q E^T; y = v - E Q u; S += I*(1e-4 S + 1)
//   dX = chol_solve(S, y); dZ = Q (u - E^T dX); pose / patch retraction.
//
// MI355X design (DESIGN.md "F-BA"), shaped by measured gfx950 costs
// (scripts/micro): barrier ~70 ns, dependent LDS load ~27 ns, dependent L2
// load ~60-175 ns, dependent fp64 FMA 36 cycles, back-to-back launch 2.4 us.
// A DPVO window is tiny (N <= 20 free poses, a few thousand edges), so one
// CU runs out of latency hiding long before it runs out of FLOPs; the work
// is spread over ~70 CUs and the launches are kept to 1 + iterations:
//
//   ba_setup_kernel (1 workgroup, once per call): counting sort of the
//       edges by patch in LDS (bitonic fallback for wide kk ranges) ->
//       "positions" grouped by patch (edge, ii, jj, kk records), unique
//       patches, per-patch free-pose masks and pose-block offsets.
//   ba_iter_kernel (one launch per iteration, NL + ceil(E/512) workgroups):
//     * one workgroup per lower 6x6 block (a, b) of S: every patch whose
//       mask holds a and b is re-linearised by one thread (the fp32 edge
//       math of the reference), which accumulates that patch's B, E Q E^T
//       (and y) terms in fp64 registers; a fixed DPP tree + ordered
//       cross-wave sum -> deterministic S block, no atomics;
//     * patch-owner workgroups: Q_u, U_u and the E column blocks c_{u,p}
//       of every patch (needed for dZ);
//     * the last workgroup to arrive (one atomic ticket, agent-scope
//       fences) damps S, runs the block Cholesky in LDS, the substitutions,
//       the pose retraction and dZ + patch retraction.
//   The split (build_schur -> all-reduce(S,y) -> solve_update) launches the
//   same code without / as the solve tail: the edge-sharded multi-GPU form
//   (SURVEY 8e).
#include "common.hpp"
#include "ba_device.hpp"  // bad::lin_edge: the one copy of the edge math

namespace dpvo {

constexpr int kSetupThreads = 1024;
constexpr int kIterThreads = 512;
constexpr int kIterWaves = kIterThreads / 64;
constexpr int kMaxSetupE = 16384;
constexpr int kMaxFree = 20;  // pose-block masks are 32-bit; lower S blocks of N=20: 59 KiB LDS
constexpr int kPerThread = kMaxSetupE / kSetupThreads;
constexpr int kCtlBytes = 512;
constexpr int kSetupLds = 160 * 1024;
constexpr int kMarks = 2432;  // [0, 128) phases; window kernel per workgroup: [128 + 256 it + g] assembled, [640 + 256 it + g] all partials seen, [1152 + g] setup, [1408 + g] it 0 pre-reduction; fused reproject + plan + insert launch: [1664 + 2b] / [1665 + 2b] start / end of workgroup b; window kernel [2176 + g] end of workgroup g
constexpr int kLaunchMarks = 1664;
constexpr int kNoPose = 31;
constexpr int kEC = 16;  // doubles per position record of E terms

struct BaWs {
  int4* srec;       // [E]   per position: edge id, ii, jj, kk (clamped to the patch buffer)
  int32_t* poff;    // [E+1] patch -> position range (positions grouped by patch, edges ascending)
  int32_t* pu;      // [E]   patch of each position
  uint32_t* pmask;  // [E]   free poses touched by each patch
  int32_t* meta;    // [8]   nuniq, status, -, num_patches, arrival ticket
  int64_t* kx;      // [E]   unique patch ids (ascending)
  float* J;         // [E][32]  per position: w[2] r[2] Jz[2] Ji[2][6] Jj[2][6]
  double* EC[2];    // [E][16]  per position: Ei[6] Ej[6] C u (E blocks, ba_cuda.cu:352-373),
                    //          ii - t0, jj - t0; double-buffered by iteration parity
  float* dbuf[2];   // [E]      per patch: inverse depth after iteration it (parity it & 1)
  double* S;        // [NL][36]
  double* y;        // [6N]
  double* dX;       // [6N]
  float* lam;       // [1]   lmbda of the last build (read by the update)
  int64_t* tmark;   // [kMarks]
  int64_t* wgt;     // [2 x grid] per-workgroup start / end stamps of the last Schur launch
};

struct BaArgs {
  float* poses;  // written in place; never restrict (read again after the update)
  float* patches;
  const float* intrinsics;
  const float* target;
  const float* weight;
  const float* lmbda;
  const int64_t* ii;
  const int64_t* jj;
  const int64_t* kk;
  int E, P, num_poses, num_patches, t0, N;
};

static inline size_t align_up(size_t v, size_t a) { return (v + a - 1) / a * a; }

static size_t ba_layout(int E, int N, char* base, BaWs* w) {
  const size_t NL = (size_t)N * (N + 1) / 2;
  size_t off = 0;
  auto take = [&](size_t bytes) -> char* {
    char* p = base ? base + off : nullptr;
    off = align_up(off + bytes, 256);
    return p;
  };
  BaWs t;
  t.srec = (int4*)take(sizeof(int4) * E);
  t.poff = (int32_t*)take(sizeof(int32_t) * (E + 1));
  t.pu = (int32_t*)take(sizeof(int32_t) * E);
  t.pmask = (uint32_t*)take(sizeof(uint32_t) * E);
  t.meta = (int32_t*)take(sizeof(int32_t) * 8);
  t.kx = (int64_t*)take(sizeof(int64_t) * E);
  t.J = (float*)take(sizeof(float) * 32 * E);
  t.EC[0] = (double*)take(sizeof(double) * kEC * E);
  t.EC[1] = (double*)take(sizeof(double) * kEC * E);
  t.dbuf[0] = (float*)take(sizeof(float) * E);
  t.dbuf[1] = (float*)take(sizeof(float) * E);
  t.S = (double*)take(sizeof(double) * 36 * (NL ? NL : 1));
  t.y = (double*)take(sizeof(double) * 6 * (N ? N : 1));
  t.dX = (double*)take(sizeof(double) * 6 * (N ? N : 1));
  t.lam = (float*)take(sizeof(float));
  t.tmark = (int64_t*)take(sizeof(int64_t) * kMarks);
  t.wgt = (int64_t*)take(sizeof(int64_t) * 2 * (NL + 8));
  if (w) *w = t;
  return off;
}

// LDS of the Schur / solve kernel: ctl | wave partials | solve tail:
// augmented [6N][6N+1] system, pivot inverse 6x6, column-block snapshot [6N][6]
static size_t iter_lds(int N) {
  const size_t n = 6 * (size_t)N;
  return kCtlBytes + sizeof(double) * (42 * kIterWaves + n * (n + 1) + 36 + 6 * n);
}

__device__ __forceinline__ int tri_row(int t) {  // a with a(a+1)/2 <= t < (a+1)(a+2)/2
  int r = (int)((sqrtf(8.0f * t + 1.0f) - 1.0f) * 0.5f);
  while (r * (r + 1) / 2 > t) r--;
  while ((r + 1) * (r + 2) / 2 <= t) r++;
  return r;
}
__device__ __forceinline__ int blk(int a, int b) { return a * (a + 1) / 2 + b; }  // a >= b

__device__ __forceinline__ void trace(int64_t* tmark, int slot) {
  if (tmark && threadIdx.x == 0 && slot < kMarks) tmark[slot] = (int64_t)wall_clock64();
}

// ---------------------------------------------------------------------------
// block-wide exclusive scan of data[0..n) in LDS (int), returns the total.
// Callers barrier before (data complete); the scan ends with a barrier.
// ---------------------------------------------------------------------------
__device__ int block_exclusive_scan(int* data, int n, int* scratch) {
  const int tid = threadIdx.x, nt = blockDim.x;
  const int per = (n + nt - 1) / nt;
  const int lo = min(tid * per, n), hi = min(lo + per, n);
  int s = 0;
  for (int i = lo; i < hi; i++) s += data[i];
  const int lane = tid & 63, wid = tid >> 6;
  int v = s;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int t = __shfl_up(v, o, 64);
    if (lane >= o) v += t;
  }
  if (lane == 63) scratch[wid] = v;
  __syncthreads();
  if (tid == 0) {
    int acc = 0;
    for (int w = 0; w < nt / 64; w++) {
      const int x = scratch[w];
      scratch[w] = acc;
      acc += x;
    }
    scratch[nt / 64] = acc;
  }
  __syncthreads();
  int run = scratch[wid] + v - s;
  for (int i = lo; i < hi; i++) {
    const int x = data[i];
    data[i] = run;
    run += x;
  }
  const int total = scratch[nt / 64];
  __syncthreads();
  return total;
}

// ---------------------------------------------------------------------------
// SETUP: unique/inverse of kk (torch::_unique(kk, sorted, inverse),
// ba_cuda.cu:447) -> positions grouped by patch, masks, pose blocks.
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(kSetupThreads) ba_setup_kernel(BaArgs A, BaWs w, int P2) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  const int tid = threadIdx.x, T = blockDim.x, lane = tid & 63, wid = tid >> 6;
  const int E = A.E, N = A.N, t0 = A.t0;
  int* ctl = reinterpret_cast<int*>(lds);  // [0] bad kk [1] kmin [2] kmax
  int* scr = ctl + 64;                     // scan scratch (T/64 + 1)
  int* red = ctl + 96;                     // per-wave min/max (2 x 16)
  char* mainp = lds + kCtlBytes;
  const int budget = (kSetupLds - kCtlBytes) / 4;  // ints
  trace(w.tmark, 40);
  // kk range (clamped to the patch buffer; out-of-range ids flag bit 1)
  int lmin = 0x7fffffff, lmax = -1, bad = 0;
  for (int i = tid; i < E; i += T) {
    int64_t v = A.kk[i];
    if (v < 0 || v >= A.num_patches) {
      bad = 1;
      v = v < 0 ? 0 : A.num_patches - 1;
    }
    lmin = min(lmin, (int)v);
    lmax = max(lmax, (int)v);
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    lmin = min(lmin, __shfl_xor(lmin, o, 64));
    lmax = max(lmax, __shfl_xor(lmax, o, 64));
    bad |= __shfl_xor(bad, o, 64);
  }
  if (lane == 0) {
    red[wid] = lmin;
    red[16 + wid] = lmax;
    red[32 + wid] = bad;
  }
  __syncthreads();
  if (tid == 0) {
    int a = 0x7fffffff, b = -1, c = 0;
    for (int k = 0; k < T / 64; k++) {
      a = min(a, red[k]);
      b = max(b, red[16 + k]);
      c |= red[32 + k];
    }
    ctl[0] = c;
    ctl[1] = a;
    ctl[2] = b;
  }
  __syncthreads();
  const int kmin = ctl[1], R = ctl[2] - ctl[1] + 1;
  const int kmaxc = A.num_patches - 1;
  int* pij;   // per position: free-pose code of ii | of jj << 8
  int* work;  // scratch ints (>= E)
  int nuniq;
  if (R + 3 * E <= budget) {
    // ---- counting sort: histogram, packed scan (start | rank << 16),
    // ticket placement, then each (small) bucket sorted by edge id
    int* hist = reinterpret_cast<int*>(mainp);
    int* spos = hist + R;
    pij = spos + E;
    work = pij + E;
    for (int v = tid; v < R; v += T) hist[v] = 0;
    __syncthreads();
    for (int i = tid; i < E; i += T) {
      const int v = (int)min(max(A.kk[i], (int64_t)0), (int64_t)kmaxc) - kmin;
      atomicAdd(&hist[v], 1);
    }
    __syncthreads();
    for (int v = tid; v < R; v += T) {
      const int c = hist[v];
      hist[v] = c | (c > 0 ? (1 << 16) : 0);
    }
    __syncthreads();
    const int tot = block_exclusive_scan(hist, R, scr);
    nuniq = tot >> 16;
    for (int v = tid; v < R; v += T) {
      const int h = hist[v];
      const int nxt = (v + 1 < R) ? hist[v + 1] : tot;
      if ((nxt >> 16) > (h >> 16)) {  // bucket v is not empty
        w.poff[h >> 16] = h & 0xffff;
        w.kx[h >> 16] = kmin + v;
      }
    }
    __syncthreads();
    for (int i = tid; i < E; i += T) {
      const int v = (int)min(max(A.kk[i], (int64_t)0), (int64_t)kmaxc) - kmin;
      spos[atomicAdd(&hist[v], 1) & 0xffff] = i;
    }
    if (tid == 0) w.poff[nuniq] = E;
    __syncthreads();
    for (int u = tid; u < nuniq; u += T) {  // insertion sort: edges ascending
      const int a = w.poff[u], b = w.poff[u + 1];
      for (int t = a + 1; t < b; t++) {
        const int x = spos[t];
        int s = t - 1;
        while (s >= a && spos[s] > x) {
          spos[s + 1] = spos[s];
          s--;
        }
        spos[s + 1] = x;
      }
      for (int t = a; t < b; t++) w.pu[t] = u;
    }
    __syncthreads();
    for (int i = tid; i < E; i += T) {
      const int e = spos[i];
      const int64_t gi = A.ii[e], gj = A.jj[e];
      const int64_t pi = gi - t0, pj = gj - t0;
      const int ci = (pi >= 0 && pi < N) ? (int)pi : kNoPose;
      const int cj = (pj >= 0 && pj < N) ? (int)pj : kNoPose;
      pij[i] = ci | (cj << 8);
      const int kv = (int)min(max(A.kk[e], (int64_t)0), (int64_t)kmaxc);
      w.srec[i] = make_int4(e, (int)gi, (int)gj, kv);
    }
  } else {
    // ---- bitonic sort of (kk << 32 | edge) keys, P2 <= 16384
    unsigned long long* keys = reinterpret_cast<unsigned long long*>(mainp);
    for (int i = tid; i < P2; i += T) {
      unsigned long long k = ~0ull;
      if (i < E) {
        const int64_t v = min(max(A.kk[i], (int64_t)0), (int64_t)kmaxc);
        k = ((unsigned long long)v << 32) | (unsigned)i;
      }
      keys[i] = k;
    }
    __syncthreads();
    for (int size = 2; size <= P2; size <<= 1) {
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
    }
    int pe[kPerThread], kv[kPerThread], hd[kPerThread];
#pragma unroll
    for (int k = 0; k < kPerThread; k++) {
      const int i = tid + k * T;
      pe[k] = kv[k] = hd[k] = 0;
      if (i < E) {
        const unsigned long long v = keys[i];
        pe[k] = (int)(v & 0xffffffffu);
        kv[k] = (int)(v >> 32);
        hd[k] = (i == 0 || (int)(keys[i - 1] >> 32) != kv[k]) ? 1 : 0;
      }
    }
    __syncthreads();
    pij = reinterpret_cast<int*>(mainp);
    work = pij + E;
#pragma unroll
    for (int k = 0; k < kPerThread; k++) {
      const int i = tid + k * T;
      if (i < E) {
        const int e = pe[k];
        const int64_t gi = A.ii[e], gj = A.jj[e];
        const int64_t pi = gi - t0, pj = gj - t0;
        const int ci = (pi >= 0 && pi < N) ? (int)pi : kNoPose;
        const int cj = (pj >= 0 && pj < N) ? (int)pj : kNoPose;
        pij[i] = ci | (cj << 8);
        work[i] = hd[k];
        w.srec[i] = make_int4(e, (int)gi, (int)gj, kv[k]);
      }
    }
    __syncthreads();
    nuniq = block_exclusive_scan(work, E, scr);
#pragma unroll
    for (int k = 0; k < kPerThread; k++) {
      const int i = tid + k * T;
      if (i < E) w.pu[i] = work[i] + hd[k] - 1;
      if (i < E && hd[k]) {
        w.kx[work[i]] = kv[k];
        w.poff[work[i]] = i;
      }
    }
    if (tid == 0) w.poff[nuniq] = E;
  }
  if (tid == 0) {
    w.meta[0] = nuniq;
    w.meta[1] = ctl[0] ? 2 : 0;
    w.meta[3] = A.num_patches;
    w.meta[4] = 0;  // arrival ticket of the Schur kernel
  }
  __syncthreads();
  trace(w.tmark, 41);
  // per patch: free-pose mask
  for (int u = tid; u < nuniq; u += T) {
    unsigned mask = 0;
    for (int t = w.poff[u]; t < w.poff[u + 1]; t++) {
      const int c = pij[t];
      if ((c & 0xff) != kNoPose) mask |= 1u << (c & 0xff);
      if ((c >> 8) != kNoPose) mask |= 1u << (c >> 8);
    }
    w.pmask[u] = mask;
  }
  trace(w.tmark, 42);
}

#pragma clang fp contract(off)
// The multi-kernel path's record layout [w(2), r(2), Jz(2), Ji(2x6), Jj(2x6)]
// over bad::lin_edge (ba_device.hpp), the same edge math the window kernel
// runs (ba_cuda.cu:265-333); only the patch-centre normalisation is here.
__device__ __forceinline__ void edge_linearize(const float* poses, const float* patches, int P,
                                               float fx, float fy, float cx, float cy, float tx,
                                               float ty, float wx, float wy, int ix, int jx,
                                               int64_t kx, bool use_depth, float depth, float* o) {
  const float* pk = patches + (size_t)kx * 3 * P * P;
  const int c11 = P + 1;  // patches[kx][*][1][1]  (ba_cuda.cu:282-285)
  const float nx = (pk[c11] - cx) / fx;
  const float ny = (pk[P * P + c11] - cy) / fy;
  const float dz = use_depth ? depth : pk[2 * P * P + c11];
  bad::Lin L;
  bad::lin_edge(poses + 7 * (size_t)ix, poses + 7 * (size_t)jx, nx, ny, dz, tx, ty, wx, wy, fx, fy,
                cx, cy, L);
  o[0] = L.w[0];
  o[1] = L.w[1];
  o[2] = L.r[0];
  o[3] = L.r[1];
  o[4] = L.Jz[0];
  o[5] = L.Jz[1];
#pragma unroll
  for (int a = 0; a < 6; a++) {
    o[6 + a] = L.Ji[0][a];
    o[12 + a] = L.Ji[1][a];
    o[18 + a] = L.Jj[0][a];
    o[24 + a] = L.Jj[1][a];
  }
}

// F-REPROJ (ba_cuda.cu:379-429): one thread per (edge, patch pixel).
__global__ void reproject_kernel(const float* __restrict__ poses, const float* __restrict__ patches,
                                 const float* __restrict__ intrinsics,
                                 const int64_t* __restrict__ ii, const int64_t* __restrict__ jj,
                                 const int64_t* __restrict__ kk, int E, int P, int num_poses,
                                 int num_patches, float* __restrict__ coords,
                                 int* __restrict__ order, int N2) {
  if (order && blockIdx.x == gridDim.x - 1) {  // extra workgroup: A-CORR edge order
    __shared__ int bins[kOrderBins + 1];
    const OrderIn q{poses, patches, intrinsics, ii, kk, P, num_poses, num_patches};
    edge_order_block(q, jj, E, N2, order, bins);
    return;
  }
  const int PP = P * P;
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= E * PP) return;
  reproject_pixel(poses, patches, intrinsics, ii, jj, kk, t / PP, t % PP, P, num_poses,
                  num_patches, coords);
}
#pragma clang fp contract(fast)

// ---------------------------------------------------------------------------
// Inverse-depth retraction of patch u (dZ = Q (u - E^T dX), ba_cuda.cu:563;
// patch_retr_kernel :209-229) from the E terms of the iteration that
// produced dX, applied to `base` (the depth that iteration used).
// ---------------------------------------------------------------------------
__device__ __forceinline__ float retract_depth(const BaWs& w, const double* EC, const double* dX,
                                               int t0, int N, double lam, int u, float base) {
  double C = 0.0, Uu = 0.0, ex = 0.0;  // ex = (E^T dX)_u
  const int p1 = w.poff[u + 1];
#pragma unroll 2
  for (int t = w.poff[u]; t < p1; t++) {
    const double* ec = EC + kEC * (size_t)t;
    const int pi = (int)ec[14], pj = (int)ec[15];
    C += ec[12];
    Uu += ec[13];
    if (pi >= 0 && pi < N)
#pragma unroll
      for (int k = 0; k < 6; k++) ex += ec[k] * dX[6 * pi + k];
    if (pj >= 0 && pj < N)
#pragma unroll
      for (int k = 0; k < 6; k++) ex += ec[6 + k] * dX[6 * pj + k];
  }
  const float dz = (float)((1.0 / (C + lam)) * (Uu - ex));  // Q = 1/(C + lmbda) (:519)
  float d = base + dz;
  d = (d > 20.0f) ? 1.0f : d;
  return (float)fmax((double)d, 1e-4);
}

// ---------------------------------------------------------------------------
// LINEARIZE (ba_lin_kernel, iteration `it`): thread per position.  For
// it > 0 the thread first retracts its patch's depth with the previous
// iteration's dX (every thread of a patch computes the same value; the
// patch's first position records it), then runs the fp32 edge math of the
// reference at that depth -> J, and the edge's E/C/u terms in fp64 -> EC.
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(256) ba_lin_kernel(BaArgs A, BaWs w, int it) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t == 0) w.lam[0] = A.lmbda[0];
  if (t >= A.E) return;
  const float fx = A.intrinsics[0], fy = A.intrinsics[1], cx = A.intrinsics[2],
              cy = A.intrinsics[3];
  const int4 r = w.srec[t];
  const int kmax = w.meta[3] - 1;
  float depth = 0.0f;
  if (it > 0) {
    const int u = w.pu[t], P = A.P;
    const float base = (it == 1)
                           ? A.patches[(size_t)min(r.w, kmax) * 3 * P * P + 2 * P * P]
                           : w.dbuf[(it - 1) & 1][u];
    depth = retract_depth(w, w.EC[(it - 1) & 1], w.dX, A.t0, A.N, (double)A.lmbda[0], u, base);
    if (t == w.poff[u]) w.dbuf[it & 1][u] = depth;
  }
  const float2 tg = reinterpret_cast<const float2*>(A.target)[r.x];
  const float2 wt = reinterpret_cast<const float2*>(A.weight)[r.x];
  const int ix = min(max(r.y, 0), A.num_poses - 1);  // memory guard (reference: unchecked)
  const int jx = min(max(r.z, 0), A.num_poses - 1);
  float o[30];
  edge_linearize(A.poses, A.patches, A.P, fx, fy, cx, cy, tg.x, tg.y, wt.x, wt.y, ix, jx,
                 (int64_t)min(r.w, kmax), it > 0, depth, o);
  float4* Jo = reinterpret_cast<float4*>(w.J + 32 * (size_t)t);
#pragma unroll
  for (int k = 0; k < 7; k++) Jo[k] = make_float4(o[4 * k], o[4 * k + 1], o[4 * k + 2], o[4 * k + 3]);
  reinterpret_cast<float2*>(Jo + 7)[0] = make_float2(o[28], o[29]);
  double ec[kEC];
#pragma unroll
  for (int k = 0; k < 14; k++) ec[k] = 0.0;
#pragma unroll
  for (int row = 0; row < 2; row++) {  // ba_cuda.cu:352-373
    const double wr = o[row];
    const float rr = o[2 + row], Jz = o[4 + row];
    const double wz = wr * Jz;
#pragma unroll
    for (int k = 0; k < 6; k++) {
      ec[k] -= wz * o[6 + 6 * row + k];
      ec[6 + k] += wz * o[18 + 6 * row + k];
    }
    ec[12] += wz * Jz;
    ec[13] += wr * rr * Jz;
  }
  ec[14] = (double)(r.y - A.t0);  // pose codes: free iff in [0, N)
  ec[15] = (double)(r.z - A.t0);
  double2* Eo = reinterpret_cast<double2*>(w.EC[it & 1] + kEC * (size_t)t);
#pragma unroll
  for (int k = 0; k < kEC / 2; k++) Eo[k] = make_double2(ec[2 * k], ec[2 * k + 1]);
}

// After the last iteration (`iters` of them): write every patch's final
// inverse depth to all P x P entries (patch_retr_kernel :225-228).
__global__ void __launch_bounds__(256) ba_apply_kernel(BaArgs A, BaWs w, int iters) {
  const int u = blockIdx.x * blockDim.x + threadIdx.x;
  if (u >= w.meta[0]) return;
  const int P = A.P, last = iters - 1;
  float* pk = A.patches + (size_t)w.kx[u] * 3 * P * P + 2 * P * P;
  const float base = (last == 0) ? pk[0] : w.dbuf[last & 1][u];
  const float d = retract_depth(w, w.EC[last & 1], w.dX, A.t0, A.N, (double)w.lam[0], u, base);
  for (int k = 0; k < P * P; k++) pk[k] = d;
}

// ---------------------------------------------------------------------------
// SCHUR block (a, b), a >= b: patch u's terms, gathered from J / EC.
// acc[0..36): row-major 6x6 block, acc[36..42): y_a (diagonal blocks).
// ---------------------------------------------------------------------------
__device__ __forceinline__ void patch_schur_terms(const BaWs& w, const double* EC, int t0,
                                                  double lam, int u, int a, int b, double* acc) {
  const bool diag = a == b;
  double C = 0.0, Uu = 0.0, ca[6], cc[6];
#pragma unroll
  for (int k = 0; k < 6; k++) ca[k] = cc[k] = 0.0;
  const int p1 = w.poff[u + 1];
#pragma unroll 2
  for (int t = w.poff[u]; t < p1; t++) {
    const double2* ep = reinterpret_cast<const double2*>(EC + kEC * (size_t)t);
    double ec[kEC];
#pragma unroll
    for (int k = 0; k < kEC / 2; k++) {
      const double2 v = ep[k];
      ec[2 * k] = v.x;
      ec[2 * k + 1] = v.y;
    }
    const int pi = (int)ec[14], pj = (int)ec[15];
    C += ec[12];
    Uu += ec[13];
    if (pi == a)
#pragma unroll
      for (int k = 0; k < 6; k++) ca[k] += ec[k];
    if (pj == a)
#pragma unroll
      for (int k = 0; k < 6; k++) ca[k] += ec[6 + k];
    if (!diag) {
      if (pi == b)
#pragma unroll
        for (int k = 0; k < 6; k++) cc[k] += ec[k];
      if (pj == b)
#pragma unroll
        for (int k = 0; k < 6; k++) cc[k] += ec[6 + k];
    }
    // B and v (ba_cuda.cu:339-370): only edges whose poses are (a, a) / {a, b}
    const bool inB = diag ? (pi == a || pj == a) : ((pi == a && pj == b) || (pi == b && pj == a));
    if (!inB) continue;
    const float4* J4 = reinterpret_cast<const float4*>(w.J + 32 * (size_t)t);
    float o[32];
#pragma unroll
    for (int k = 0; k < 8; k++) {
      const float4 v = J4[k];
      o[4 * k] = v.x;
      o[4 * k + 1] = v.y;
      o[4 * k + 2] = v.z;
      o[4 * k + 3] = v.w;
    }
    const bool rows_i = (pi == a);  // off-diagonal: rows follow pose a
#pragma unroll
    for (int row = 0; row < 2; row++) {
      const double wr = o[row];
      const double wrr = wr * o[2 + row];
      float Ji[6], Jj[6];
#pragma unroll
      for (int k = 0; k < 6; k++) {
        Ji[k] = o[6 + 6 * row + k];
        Jj[k] = o[18 + 6 * row + k];
      }
      if (diag) {
        if (pi == a) {
#pragma unroll
          for (int x = 0; x < 6; x++) {
            const double wx = wr * Ji[x];
#pragma unroll
            for (int z = 0; z < 6; z++) acc[6 * x + z] += wx * Ji[z];
            acc[36 + x] -= wrr * Ji[x];
          }
        }
        if (pj == a) {
#pragma unroll
          for (int x = 0; x < 6; x++) {
            const double wx = wr * Jj[x];
#pragma unroll
            for (int z = 0; z < 6; z++) acc[6 * x + z] += wx * Jj[z];
            acc[36 + x] += wrr * Jj[x];
          }
        }
        if (pi == a && pj == a) {
#pragma unroll
          for (int x = 0; x < 6; x++)
#pragma unroll
            for (int z = 0; z < 6; z++) acc[6 * x + z] -= wr * Ji[x] * Jj[z] + wr * Jj[x] * Ji[z];
        }
      } else {
        // rows follow pose a: Ji when ii == a, Jj when jj == a
#pragma unroll
        for (int x = 0; x < 6; x++) {
          const double wx = wr * (rows_i ? Ji[x] : Jj[x]);
#pragma unroll
          for (int z = 0; z < 6; z++) acc[6 * x + z] -= wx * (rows_i ? Jj[z] : Ji[z]);
        }
      }
    }
  }
  // - E Q E^T and - E Q u (:554-558)
  const double q = 1.0 / (C + lam);  // :519
  const double* cr = diag ? ca : cc;
#pragma unroll
  for (int x = 0; x < 6; x++) {
    const double cq = ca[x] * q;
#pragma unroll
    for (int z = 0; z < 6; z++) acc[6 * x + z] -= cq * cr[z];
  }
  if (diag) {
    const double qu = q * Uu;
#pragma unroll
    for (int x = 0; x < 6; x++) acc[36 + x] -= ca[x] * qu;
  }
}

// ---------------------------------------------------------------------------
// Deterministic wave sum to lane 63 with DPP row shifts + row broadcasts
// (no LDS traffic); fp64 values move as two 32-bit halves.
// ---------------------------------------------------------------------------
template <int CTRL, int ROW_MASK, int BANK_MASK>
__device__ __forceinline__ double dpp_f64(double v) {
  const int lo = __builtin_amdgcn_update_dpp(0, __double2loint(v), CTRL, ROW_MASK, BANK_MASK, true);
  const int hi = __builtin_amdgcn_update_dpp(0, __double2hiint(v), CTRL, ROW_MASK, BANK_MASK, true);
  return __hiloint2double(hi, lo);
}

__device__ __forceinline__ double wave_sum_to_63(double v) {
  v += dpp_f64<0x111, 0xf, 0xf>(v);  // row_shr:1
  v += dpp_f64<0x112, 0xf, 0xf>(v);  // row_shr:2
  v += dpp_f64<0x114, 0xf, 0xf>(v);  // row_shr:4
  v += dpp_f64<0x118, 0xf, 0xf>(v);  // row_shr:8  -> lane 15 of each row: row sum
  v += dpp_f64<0x142, 0xa, 0xf>(v);  // row_bcast:15 -> rows 1, 3
  v += dpp_f64<0x143, 0xc, 0xf>(v);  // row_bcast:31 -> rows 2, 3: lane 63 = total
  return v;
}

// sum of NV per-thread values over the workgroup in a fixed order -> red[]
// (LDS).  Only waves below `active_waves` hold non-zero values (the
// compacted patch list fills threads from 0); the others skip the DPP tree.
// part: (blockDim/64) * NV doubles of LDS.
template <int NV>
__device__ __forceinline__ void block_sum(const double* v, double* part, double* red,
                                          int active_waves) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int nw = min((int)(blockDim.x >> 6), max(active_waves, 1));
  if (wid < nw) {
#pragma unroll
    for (int i = 0; i < NV; i++) {
      const double s = wave_sum_to_63(v[i]);
      if (lane == 63) part[wid * NV + i] = s;
    }
  }
  __syncthreads();
  if (threadIdx.x < NV) {
    double s = 0.0;
    for (int k = 0; k < nw; k++) s += part[k * NV + threadIdx.x];
    red[threadIdx.x] = s;
  }
  __syncthreads();
}

// ---------------------------------------------------------------------------
// SOLVE tail: damped S x = y by block Gauss-Jordan (6x6 pivot blocks) on the
// augmented system in LDS -- SPD, no pivoting needed; the elimination of
// every row block at each step folds the back substitution in, so the
// critical path is one 6x6 inversion per pose.
// ---------------------------------------------------------------------------
__device__ __forceinline__ double rcp_d(double x) {  // estimate + one Newton step
  const double r = __builtin_amdgcn_rcp(x);
  return __builtin_fma(r, __builtin_fma(-x, r, 1.0), r);
}

// one lane: in-place Gauss-Jordan inverse of an SPD 6x6 block (registers)
__device__ __forceinline__ bool invert6(const double* M, int ld, double* Pinv) {
  double a[6][6];
#pragma unroll
  for (int r = 0; r < 6; r++)
#pragma unroll
    for (int c = 0; c < 6; c++) a[r][c] = M[r * ld + c];
  bool ok = true;
#pragma unroll
  for (int c = 0; c < 6; c++) {
    const double piv = a[c][c];
    ok = ok && (piv > 0.0);
    const double r = rcp_d(piv);
    a[c][c] = 1.0;
#pragma unroll
    for (int j = 0; j < 6; j++) a[c][j] *= r;
#pragma unroll
    for (int i = 0; i < 6; i++) {
      if (i == c) continue;
      const double f = a[i][c];
      a[i][c] = 0.0;
#pragma unroll
      for (int j = 0; j < 6; j++) a[i][j] -= f * a[c][j];
    }
  }
#pragma unroll
  for (int r = 0; r < 6; r++)
#pragma unroll
    for (int c = 0; c < 6; c++) Pinv[6 * r + c] = a[r][c];
  return ok;
}

struct TailLds {
  int* ctl;      // [0] last-arrival flag, [1] failure
  double* part;  // kIterWaves x 42
  double* M;     // [n][n+1] augmented system
  double* Pinv;  // [36]
  double* Cb;    // [n][6] snapshot of the pivot column block
};
__device__ __forceinline__ TailLds tail_carve(char* lds, int N) {
  const int n = 6 * N;
  TailLds s;
  s.ctl = reinterpret_cast<int*>(lds);
  s.part = reinterpret_cast<double*>(lds + kCtlBytes);
  s.M = s.part + 42 * kIterWaves;
  s.Pinv = s.M + (size_t)n * (n + 1);
  s.Cb = s.Pinv + 36;
  return s;
}

// x overwrites column n of M; returns failure
__device__ int ba_solve_gj(int N, const TailLds& L, int64_t* tr) {
  const int tid = threadIdx.x, T = blockDim.x, n = 6 * N, ld = n + 1;
  double* M = L.M;
  if (tid == 0) L.ctl[1] = invert6(M, ld, L.Pinv) ? 0 : 1;
  __syncthreads();
  trace(tr, 50);
  for (int k = 0; k < N; k++) {
    const int k0 = 6 * k, c0 = k0 + 6;  // columns left of c0 are already eliminated
    // (1) pivot rows: row block k <- Pinv * row block k (columns c0..n);
    //     snapshot the pivot column block of the other rows
    for (int c = c0 + tid; c <= n; c += T) {
      double v[6], o[6];
#pragma unroll
      for (int q = 0; q < 6; q++) v[q] = M[(k0 + q) * ld + c];
#pragma unroll
      for (int r = 0; r < 6; r++) {
        double s = 0.0;
#pragma unroll
        for (int q = 0; q < 6; q++) s += L.Pinv[6 * r + q] * v[q];
        o[r] = s;
      }
#pragma unroll
      for (int r = 0; r < 6; r++) M[(k0 + r) * ld + c] = o[r];
    }
    for (int t = tid; t < 6 * n; t += T) L.Cb[t] = M[(t / 6) * ld + k0 + t % 6];
    __syncthreads();
    trace(tr, 60 + 2 * k);
    // (2) eliminate the pivot column block from every other row.  Wave 0
    //     first updates the next pivot block (k+1, k+1) and inverts it
    //     (look-ahead) while the other waves eliminate everything else: a
    //     thread owns one column and a strided group of rows, 4 rows per
    //     batch of independent loads.
    const int ncol = n + 1 - c0, nrow = n - 6;
    const bool ahead = (k + 1 < N);
    if (ahead && tid < 64) {
      if (tid < 36) {
        const int r = c0 + tid / 6, c = c0 + tid % 6;
        const double* f = L.Cb + 6 * r;
        double v = M[r * ld + c];
#pragma unroll
        for (int q = 0; q < 6; q++) v -= f[q] * M[(k0 + q) * ld + c];
        M[r * ld + c] = v;
      }
      wave_lds_sync();
      if (tid == 0 && !invert6(M + (size_t)c0 * ld + c0, ld, L.Pinv)) L.ctl[1] = 1;
    }
    const int T2 = ahead ? T - 64 : T, tid2 = ahead ? tid - 64 : tid;
    const int G = max(1, min(nrow, T2 / ncol));
    if (tid2 >= 0) {
      for (int task = tid2; task < ncol * G; task += T2) {
        const int c = c0 + task % ncol, g = task / ncol;
        double tq[6];
#pragma unroll
        for (int q = 0; q < 6; q++) tq[q] = M[(k0 + q) * ld + c];
        for (int i0 = g; i0 < nrow; i0 += 4 * G) {
          int rows[4];
          double v[4];
#pragma unroll
          for (int j = 0; j < 4; j++) {
            const int i = i0 + j * G;
            rows[j] = (i < nrow) ? i + ((i >= k0) ? 6 : 0) : -1;
            // the look-ahead block was already updated by wave 0
            if (ahead && rows[j] >= c0 && rows[j] < c0 + 6 && c < c0 + 6) rows[j] = -1;
            v[j] = rows[j] >= 0 ? M[rows[j] * ld + c] : 0.0;
          }
#pragma unroll
          for (int j = 0; j < 4; j++) {
            if (rows[j] < 0) continue;
            const double* f = L.Cb + 6 * rows[j];
            double x = v[j];
#pragma unroll
            for (int q = 0; q < 6; q++) x -= f[q] * tq[q];
            M[rows[j] * ld + c] = x;
          }
        }
      }
    }
    __syncthreads();
    trace(tr, 61 + 2 * k);
  }
  trace(tr, 51);
  return L.ctl[1];
}

// ---------------------------------------------------------------------------
// POSE UPDATE: dX out, pose_retr_kernel (:178-206).  x: dX (6N, stride xs).
// The patch retraction happens in the next ba_lin_kernel / ba_apply_kernel.
// ---------------------------------------------------------------------------
__device__ void ba_pose_update(const BaArgs& A, const BaWs& w, const double* x, int xs, int fail,
                               double* dX_out) {
  const int tid = threadIdx.x, T = blockDim.x, N = A.N;
  for (int i = tid; i < 6 * N; i += T) {
    const double v = fail ? 0.0 : x[i * xs];  // failed factorisation: dX = 0 (dpvo/ba.py:17-21)
    w.dX[i] = v;
    if (dX_out) dX_out[i] = v;
  }
  if (tid == 0) w.meta[1] = (w.meta[1] & ~1) | (fail ? 1 : 0);
  for (int i = tid; i < N; i += T) {
    const int t = A.t0 + i;
    if (t < 0 || t >= A.num_poses) continue;
    float* pt = A.poses + 7 * (size_t)t;
    float xi[6], t1[3], q1[4];
#pragma unroll
    for (int k = 0; k < 6; k++) xi[k] = fail ? 0.0f : (float)x[(6 * i + k) * xs];
    float tt[3] = {pt[0], pt[1], pt[2]}, qq[4] = {pt[3], pt[4], pt[5], pt[6]};
    retrSE3(xi, tt, qq, t1, q1);
    pt[0] = t1[0]; pt[1] = t1[1]; pt[2] = t1[2];
    pt[3] = q1[0]; pt[4] = q1[1]; pt[5] = q1[2]; pt[6] = q1[3];
  }
}

// the solve tail: S (lower blocks), y from global -> augmented system in
// LDS, damping, Gauss-Jordan, update
__device__ void ba_solve_tail(const BaArgs& A, const BaWs& w, const double* S_in,
                              const double* y_in, double* dX_out, const TailLds& L, int64_t* tr) {
  const int N = A.N, n = 6 * N, ld = n + 1;
  int fail = 0;
  if (N > 0) {
    // batches of 16 independent loads per thread (one latency per batch)
    constexpr int B = 16;
    for (int t0 = threadIdx.x; t0 < n * n; t0 += B * blockDim.x) {
      double v[B];
#pragma unroll
      for (int j = 0; j < B; j++) {
        const int t = t0 + j * blockDim.x;
        v[j] = 0.0;
        if (t < n * n) {
          const int r = t / n, c = t % n, ar = r / 6, ac = c / 6;
          // lower blocks hold (a, b), a >= b; the upper half is the transpose
          v[j] = (ar >= ac) ? S_in[36 * blk(ar, ac) + 6 * (r % 6) + c % 6]
                            : S_in[36 * blk(ac, ar) + 6 * (c % 6) + r % 6];
        }
      }
#pragma unroll
      for (int j = 0; j < B; j++) {
        const int t = t0 + j * blockDim.x;
        if (t < n * n) {
          const int r = t / n, c = t % n;
          double x = v[j];
          if (r == c) x += 1e-4 * x + 1.0;  // S += I * (1e-4 S + 1)  (ba_cuda.cu:560)
          L.M[r * ld + c] = x;
        }
      }
    }
    for (int r = threadIdx.x; r < n; r += blockDim.x) L.M[r * ld + n] = y_in[r];
    __syncthreads();
    fail = ba_solve_gj(N, L, tr);
  }
  ba_pose_update(A, w, L.M + n, ld, fail, dX_out);
}

// Schur blocks + (do_solve) the last-arrival solve tail.  One workgroup per
// lower 6x6 block (a, b) of S.
__global__ void __launch_bounds__(kIterThreads)
    ba_schur_kernel(BaArgs A, BaWs w, double* S_out, double* y_out, double* dX_out, int do_solve,
                    int it, int trace_it) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  const TailLds L = tail_carve(lds, A.N);
  const int tid = threadIdx.x;
  int64_t* tr = trace_it ? w.tmark : nullptr;
  if (tid == 0) w.wgt[2 * blockIdx.x] = (int64_t)wall_clock64();
  {
    const int d = blockIdx.x, a = tri_row(d), b = d - a * (a + 1) / 2;
    const double lam = (double)A.lmbda[0];
    const int nuniq = w.meta[0];
    double acc[42];  // 36 S entries + 6 y entries
#pragma unroll
    for (int i = 0; i < 42; i++) acc[i] = 0.0;
    // compact the patches whose mask holds a and b (ballots, in patch order)
    int* rp = reinterpret_cast<int*>(L.M);  // free until the tail
    int* wc = L.ctl + 8;                    // per-wave counts
    const int lane = tid & 63, wid = tid >> 6, nw = blockDim.x >> 6;
    int nrel = 0;
    for (int base = 0; base < nuniq; base += blockDim.x) {
      const int u = base + tid;
      bool rel = false;
      if (u < nuniq) {
        const unsigned mask = w.pmask[u];
        rel = ((mask >> a) & 1u) && ((mask >> b) & 1u);
      }
      const unsigned long long m = __ballot(rel);
      if (lane == 0) wc[wid] = __popcll(m);
      __syncthreads();
      int before = 0, total = 0;
      for (int k = 0; k < nw; k++) {
        const int c = wc[k];
        before += (k < wid) ? c : 0;
        total += c;
      }
      if (rel) rp[nrel + before + __popcll(m & ((1ull << lane) - 1ull))] = u;
      nrel += total;
      __syncthreads();
    }
    int64_t* trw = (blockIdx.x == 0) ? tr : (blockIdx.x == gridDim.x - 1 && tr ? tr + 5 : nullptr);
    trace(trw, 100);
    const double* EC = w.EC[it & 1];
    for (int i = tid; i < nrel; i += blockDim.x)
      patch_schur_terms(w, EC, A.t0, lam, rp[i], a, b, acc);
    __syncthreads();  // rp is overwritten by the sums below
    trace(trw, 101);
    double* red = L.M;  // 42 doubles, free until the tail
    // every thread with data has tid < nrel (one patch per thread when
    // nrel <= blockDim, more otherwise: then all waves are active)
    const int active = nrel >= (int)blockDim.x ? (int)(blockDim.x >> 6) : (nrel + 63) / 64;
    block_sum<42>(acc, L.part, red, active);
    if (tid < 36) S_out[36 * d + tid] = red[tid];
    if (a == b && tid >= 36 && tid < 42) y_out[6 * a + tid - 36] = red[tid];
    trace(trw, 102);
  }
  __syncthreads();
  if (tid == 0) w.wgt[2 * blockIdx.x + 1] = (int64_t)wall_clock64();
  if (!do_solve) return;
  // last-arrival election.  Every wave drains its stores (workgroup-scope
  // release: s_waitcnt), then ONE lane writes the XCD L2 back (agent-scope
  // release, ~1.7 us -- per workgroup, not per thread) and takes a ticket.
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  __syncthreads();
  if (tid == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    L.ctl[0] = (atomicAdd(&w.meta[4], 1) == (int)gridDim.x - 1) ? 1 : 0;
    if (L.ctl[0]) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");  // this CU's L1
  }
  __syncthreads();
  if (!L.ctl[0]) return;  // the last one reads every other workgroup's S blocks and y
  trace(tr, 49);
  ba_solve_tail(A, w, S_out, y_out, dX_out, L, tr);
  trace(tr, 52);
  if (tid == 0) w.meta[4] = 0;  // ticket for the next launch
}

// split form, step 3 (and N == 0): solve + update from an (all-reduced) S, y
__global__ void __launch_bounds__(kIterThreads)
    ba_solve_kernel(BaArgs A, BaWs w, const double* S_in, const double* y_in, double* dX_out) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  const TailLds L = tail_carve(lds, A.N);
  ba_solve_tail(A, w, S_in, y_in, dX_out, L, nullptr);
}

// ---------------------------------------------------------------------------
// F-NBR (ba.cpp:59-97): for edge e, among edges f with ii[f] == ii[e] ordered
// by (jj, index) (= stable sort by jj), ix = predecessor, jx = successor.
// O(E^2) comparisons, tiled through LDS: no size limit, no sort state.
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(256)
    neighbors_kernel(const int64_t* __restrict__ ii, const int64_t* __restrict__ jj, int E,
                     int64_t* __restrict__ ix, int64_t* __restrict__ jx) {
  __shared__ int64_t si[256], sj[256];
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  const bool act = e < E;
  const int64_t ie = act ? ii[e] : 0, je = act ? jj[e] : 0;
  int64_t best_prev = -1, best_next = -1;
  int64_t pj_ = 0, nj_ = 0;
  for (int base = 0; base < E; base += 256) {
    const int f = base + threadIdx.x;
    si[threadIdx.x] = f < E ? ii[f] : 0;
    sj[threadIdx.x] = f < E ? jj[f] : 0;
    __syncthreads();
    const int lim = min(256, E - base);
    if (act) {
      for (int k = 0; k < lim; k++) {
        const int g = base + k;
        if (g == e || si[k] != ie) continue;
        const int64_t jg = sj[k];
        const bool before = jg < je || (jg == je && g < e);
        if (before) {
          if (best_prev < 0 || jg > pj_ || (jg == pj_ && g > best_prev)) { best_prev = g; pj_ = jg; }
        } else {
          if (best_next < 0 || jg < nj_ || (jg == nj_ && g < best_next)) { best_next = g; nj_ = jg; }
        }
      }
    }
    __syncthreads();
  }
  if (act) {
    ix[e] = best_prev;
    jx[e] = best_next;
  }
}


// ba_window.hip: plan kernel + persistent per-block workgroups, solve in every workgroup
size_t ba_window_scratch_bytes(int E, int N);
bool ba_window_supported(int E, int N, int P);
int ba_window_launch(float* poses, float* patches, const float* intrinsics, const float* target,
                     const float* weight, const float* lmbda, const int64_t* ii, const int64_t* jj,
                     const int64_t* kk, int E, int P, int num_poses, int num_patches, int t0, int t1,
                     int iterations, char* scratch, int* status, int64_t* marks, double* dxo,
                     void* stream);
int ba_window_plan(const int64_t* ii, const int64_t* jj, const int64_t* kk, int E, int num_patches,
                   int num_poses, int t0, int t1, char* scratch, int* status, void* stream,
                   const int* t0d);
void ba_window_plan_offsets(int E, int64_t* out);
int ba_window_reproject_plan(const float* poses, const float* patches, const float* intrinsics,
                             const int64_t* ii, const int64_t* jj, const int64_t* kk, int E, int P,
                             int num_poses, int num_patches, int N2, float* coords, int* order,
                             int t0, int t1, char* scratch, int* status, void* stream,
                             const int* t0d);
int ba_window_reproject_plan_insert(const float* poses, const float* patches,
                                    const float* intrinsics, const int64_t* ii, const int64_t* jj,
                                    const int64_t* kk, int E, int P, int num_poses,
                                    int num_patches, int N2, float* coords, int* order, int t0,
                                    int t1, char* scratch, int* status, const void* src,
                                    void* const* dst, const int* scale, int L, int C, int H, int W,
                                    int half, int64_t* marks, void* stream);
int ba_window_run(float* poses, float* patches, const float* intrinsics, const float* target,
                  const float* weight, const float* lmbda, const int64_t* ii, const int64_t* jj,
                  const int64_t* kk, int E, int P, int num_poses, int num_patches, int t0, int t1,
                  int iterations, char* scratch, int* status, int64_t* marks, double* dxo,
                  void* stream, const int* t0d);
// ba_large.hip: large graphs (global BA, cfg4)
size_t gba_workspace_bytes(int E, int N);
int gba_forward(float* poses, float* patches, const float* intrinsics, const float* target,
                const float* weight, const float* lmbda, const int64_t* ii, const int64_t* jj,
                const int64_t* kk, int E, int P, int num_poses, int num_patches, int PPF, int t0,
                int t1, int iterations, void* workspace, size_t workspace_bytes, void* stream);
double* gba_dx(void* workspace, int E, int N);

}  // namespace dpvo

namespace {
// 0 auto (window), 2 multi-kernel, 4 large-graph path, 5 window (1 / 3 removed)
int g_ba_path = 0;
// instrumentation: phase marks stamped by the window kernel (dpvo_ba_set_marks)
bool g_ba_marks = false;
}

using namespace dpvo;

// Kernels whose LDS exceeds the 64 KiB default opt in to the 160 KiB of a CU.
static void ensure_lds_limits() {
  static bool done = false;
  if (done) return;
  (void)hipFuncSetAttribute((const void*)ba_setup_kernel,
                            hipFuncAttributeMaxDynamicSharedMemorySize, kSetupLds);
  (void)hipFuncSetAttribute((const void*)ba_schur_kernel,
                            hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  (void)hipFuncSetAttribute((const void*)ba_solve_kernel,
                            hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  done = true;
}

static int pow2_at_least(int v) {
  int p = 1;
  while (p < v) p <<= 1;
  return p;
}

static BaArgs make_args(float* poses, float* patches, const float* intrinsics, const float* target,
                        const float* weight, const float* lmbda, const int64_t* ii,
                        const int64_t* jj, const int64_t* kk, int E, int P, int num_poses,
                        int num_patches, int t0, int t1) {
  BaArgs a;
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
  a.N = t1 - t0;
  return a;
}

static int schur_grid(int N) { return N * (N + 1) / 2; }
static int lin_grid(int E) { return (E + 255) / 256; }

// the window paths (blocks / fused / multi-kernel) cover E <= kMaxSetupE and
// N <= kMaxFree; anything larger (global BA, cfg4) runs ba_large.hip
static bool window_path_ok(int E, int N) { return E <= kMaxSetupE && N <= kMaxFree; }
static bool use_large(int E, int N) { return g_ba_path == 4 || !window_path_ok(E, N); }

DPVO_EXPORT size_t dpvo_ba_workspace_bytes(int E, int t0, int t1) {
  const int N = t1 > t0 ? t1 - t0 : 0;
  const int Ep = E > 0 ? E : 1;
  size_t bytes = 0;
  if (window_path_ok(Ep, N)) {
    size_t a = 0;
    if (ba_window_supported(Ep, N, 3)) {
      const size_t c = ba_window_scratch_bytes(Ep, N);
      a = a > c ? a : c;
    }
    bytes = ba_layout(Ep, N, nullptr, nullptr) + a;
  }
  if (use_large(Ep, N)) {
    const size_t g = gba_workspace_bytes(Ep, N);
    bytes = g > bytes ? g : bytes;
  }
  return bytes;
}

DPVO_EXPORT int dpvo_ba_select_path(int mode) {
  if (mode < 0 || mode > 5 || mode == 1 || mode == 3) return DPVO_ERR_INVALID;
  g_ba_path = mode;
  return DPVO_OK;
}


DPVO_EXPORT int dpvo_ba_max_free_poses(void) { return dpvo_gba_max_free_poses(); }

DPVO_EXPORT int dpvo_ba_setup(const int64_t* ii, const int64_t* jj, const int64_t* kk, int E,
                              int num_patches, int t0, int t1, void* workspace,
                              size_t workspace_bytes, void* stream) {
  if (E <= 0) return DPVO_OK;
  if (t1 < t0 || !ii || !jj || !kk || !workspace || num_patches <= 0) return DPVO_ERR_INVALID;
  const int N = t1 - t0;
  if (E > kMaxSetupE || N > kMaxFree) return DPVO_ERR_UNSUPPORTED;
  if (workspace_bytes < dpvo_ba_workspace_bytes(E, t0, t1)) return DPVO_ERR_WORKSPACE;
  BaWs w;
  ba_layout(E, N, (char*)workspace, &w);
  ensure_lds_limits();
  BaArgs a = make_args(nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, ii, jj, kk, E, 0, 0,
                       num_patches, t0, t1);
  hipLaunchKernelGGL(ba_setup_kernel, dim3(1), dim3(kSetupThreads), kSetupLds, as_stream(stream),
                     a, w, pow2_at_least(E < 2 ? 2 : E));
  return launch_status();
}

DPVO_EXPORT int dpvo_ba_build_schur(const float* poses, const float* patches,
                                    const float* intrinsics, const float* target,
                                    const float* weight, const float* lmbda, const int64_t* ii,
                                    const int64_t* jj, const int64_t* kk, int E, int P,
                                    int num_poses, int t0, int t1, void* workspace,
                                    double* S_lower, double* y, void* stream) {
  if (E <= 0) return DPVO_OK;
  if (P < 2 || num_poses <= 0 || t1 < t0 || !workspace) return DPVO_ERR_INVALID;
  const int N = t1 - t0;
  if (N > kMaxFree || E > kMaxSetupE) return DPVO_ERR_UNSUPPORTED;
  BaWs w;
  ba_layout(E, N, (char*)workspace, &w);
  ensure_lds_limits();
  BaArgs a = make_args(const_cast<float*>(poses), const_cast<float*>(patches), intrinsics, target,
                       weight, lmbda, ii, jj, kk, E, P, num_poses, 0, t0, t1);
  hipStream_t s = as_stream(stream);
  hipLaunchKernelGGL(ba_lin_kernel, dim3(lin_grid(E)), dim3(256), 0, s, a, w, 0);
  int st = launch_status();
  if (st || N == 0) return st;
  hipLaunchKernelGGL(ba_schur_kernel, dim3(schur_grid(N)), dim3(kIterThreads), iter_lds(N), s, a,
                     w, S_lower ? S_lower : w.S, y ? y : w.y, nullptr, 0, 0, 0);
  return launch_status();
}

DPVO_EXPORT int dpvo_ba_solve_update(float* poses, float* patches, const double* S_lower,
                                     const double* y, int E, int P, int num_poses, int t0, int t1,
                                     void* workspace, double* dX_out, void* stream) {
  if (E <= 0) return DPVO_OK;
  if (P < 2 || t1 < t0 || !workspace) return DPVO_ERR_INVALID;
  const int N = t1 - t0;
  if (N > kMaxFree) return DPVO_ERR_UNSUPPORTED;
  BaWs w;
  ba_layout(E, N, (char*)workspace, &w);
  ensure_lds_limits();
  // the patch retraction reads lmbda (Q = 1/(C + lmbda)) from the workspace
  // copy the build step made
  BaArgs a = make_args(poses, patches, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr,
                       nullptr, E, P, num_poses, 0, t0, t1);
  hipStream_t s = as_stream(stream);
  hipLaunchKernelGGL(ba_solve_kernel, dim3(1), dim3(kIterThreads), iter_lds(N), s, a, w,
                     S_lower ? S_lower : w.S, y ? y : w.y, dX_out);
  int st = launch_status();
  if (st) return st;
  hipLaunchKernelGGL(ba_apply_kernel, dim3(lin_grid(E)), dim3(256), 0, s, a, w, 1);
  return launch_status();
}

DPVO_EXPORT int dpvo_ba_last_status(const void* workspace, int E, int t0, int t1, int* out,
                                    void* stream) {
  if (!workspace || !out || E <= 0) return DPVO_ERR_INVALID;
  BaWs w;
  ba_layout(E, t1 > t0 ? t1 - t0 : 0, (char*)workspace, &w);
  return hipMemcpyAsync(out, w.meta + 1, sizeof(int), hipMemcpyDeviceToDevice,
                        as_stream(stream)) == hipSuccess
             ? DPVO_OK
             : DPVO_ERR_LAUNCH;
}

namespace dpvo {
int gba_status_or(const void* workspace, int E, int N, int* acc, void* stream);
}
namespace {
__global__ void k_status_or(const int* src, int* acc) {
  if (threadIdx.x == 0) atomicOr(acc, *src);
}
}  // namespace

namespace dpvo {
void ba_set_status_sink(int* sink);
}
DPVO_EXPORT int dpvo_ba_set_status_sink(int* acc) {
  dpvo::ba_set_status_sink(acc);
  return DPVO_OK;
}

DPVO_EXPORT int dpvo_ba_status_accumulate(const void* workspace, int E, int t0, int t1, int* acc,
                                          void* stream) {
  if (!workspace || !acc) return DPVO_ERR_INVALID;
  if (E <= 0) return DPVO_OK;
  const int N = t1 > t0 ? t1 - t0 : 0;
  if (use_large(E, N)) return gba_status_or(workspace, E, N, acc, stream);
  // the window kernels OR their status into the registered sink themselves
  if ((g_ba_path == 0 || g_ba_path == 5) && ba_window_supported(E, N, 3)) return DPVO_OK;
  BaWs w;
  ba_layout(E, N, (char*)workspace, &w);
  hipLaunchKernelGGL(k_status_or, dim3(1), dim3(64), 0, as_stream(stream), w.meta + 1, acc);
  return launch_status();
}

DPVO_EXPORT int dpvo_ba_phase_marks(const void* workspace, int E, int t0, int t1, int64_t* out,
                                    void* stream) {
  if (!workspace || !out || E <= 0) return DPVO_ERR_INVALID;
  BaWs w;
  ba_layout(E, t1 > t0 ? t1 - t0 : 0, (char*)workspace, &w);
  return hipMemcpyAsync(out, w.tmark, sizeof(int64_t) * kMarks, hipMemcpyDeviceToDevice,
                        as_stream(stream)) == hipSuccess
             ? DPVO_OK
             : DPVO_ERR_LAUNCH;
}

DPVO_EXPORT int dpvo_ba_set_marks(int on) {
  g_ba_marks = on != 0;
  return DPVO_OK;
}

DPVO_EXPORT int dpvo_ba_last_dx(const void* workspace, int E, int t0, int t1, double* out,
                                void* stream) {
  if (!workspace || !out || E <= 0 || t1 < t0) return DPVO_ERR_INVALID;
  const int N = t1 - t0;
  if (N == 0) return DPVO_OK;
  const double* src;
  if (use_large(E, N)) {
    src = gba_dx(const_cast<void*>(workspace), E, N);
  } else {
    BaWs w;
    ba_layout(E, N, (char*)workspace, &w);
    src = w.dX;
  }
  return hipMemcpyAsync(out, src, sizeof(double) * 6 * N, hipMemcpyDeviceToDevice,
                        as_stream(stream)) == hipSuccess
             ? DPVO_OK
             : DPVO_ERR_LAUNCH;
}

// instrumentation: per-workgroup start/end stamps of the last iteration launch
DPVO_EXPORT int dpvo_ba_workgroup_marks(const void* workspace, int E, int t0, int t1, int64_t* out,
                                        void* stream) {
  if (!workspace || !out || E <= 0) return DPVO_ERR_INVALID;
  const int N = t1 > t0 ? t1 - t0 : 0;
  BaWs w;
  ba_layout(E, N, (char*)workspace, &w);
  return hipMemcpyAsync(out, w.wgt, sizeof(int64_t) * 2 * schur_grid(N),
                        hipMemcpyDeviceToDevice, as_stream(stream)) == hipSuccess
             ? DPVO_OK
             : DPVO_ERR_LAUNCH;
}

DPVO_EXPORT int dpvo_ba_forward(float* poses, float* patches, const float* intrinsics,
                                const float* target, const float* weight, const float* lmbda,
                                const int64_t* ii, const int64_t* jj, const int64_t* kk, int E,
                                int P, int num_poses, int num_patches, int PPF, int t0, int t1,
                                int iterations, int eff_impl, void* workspace,
                                size_t workspace_bytes, void* stream) {
  (void)PPF;
  (void)eff_impl;  // one block-sparse implementation serves both reference paths
  if (E <= 0 || iterations <= 0) return DPVO_OK;
  if (P < 2 || num_poses <= 0 || num_patches <= 0 || t1 < t0 || !workspace || !poses ||
      !patches || !intrinsics || !target || !weight || !lmbda || !ii || !jj || !kk)
    return DPVO_ERR_INVALID;
  const int N = t1 - t0;
  if (workspace_bytes < dpvo_ba_workspace_bytes(E, t0, t1)) return DPVO_ERR_WORKSPACE;
  if (use_large(E, N))
    return gba_forward(poses, patches, intrinsics, target, weight, lmbda, ii, jj, kk, E, P,
                       num_poses, num_patches, PPF, t0, t1, iterations, workspace,
                       workspace_bytes, stream);
  BaWs w;
  const size_t base_bytes = ba_layout(E, N, (char*)workspace, &w);
  if ((g_ba_path == 0 || g_ba_path == 5) && ba_window_supported(E, N, P))
    return ba_window_launch(poses, patches, intrinsics, target, weight, lmbda, ii, jj, kk, E, P,
                            num_poses, num_patches, t0, t1, iterations,
                            (char*)workspace + base_bytes, w.meta + 1,
                            g_ba_marks ? w.tmark : nullptr, w.dX, stream);
  ensure_lds_limits();
  hipStream_t s = as_stream(stream);
  BaArgs a = make_args(poses, patches, intrinsics, target, weight, lmbda, ii, jj, kk, E, P,
                       num_poses, num_patches, t0, t1);
  hipLaunchKernelGGL(ba_setup_kernel, dim3(1), dim3(kSetupThreads), kSetupLds, s, a, w,
                     pow2_at_least(E < 2 ? 2 : E));
  int st = launch_status();
  for (int it = 0; it < iterations && st == DPVO_OK; it++) {
    hipLaunchKernelGGL(ba_lin_kernel, dim3(lin_grid(E)), dim3(256), 0, s, a, w, it);
    if (N > 0)  // N == 0 (structure only): dZ = Q u, applied by the next lin / apply kernel
      hipLaunchKernelGGL(ba_schur_kernel, dim3(schur_grid(N)), dim3(kIterThreads), iter_lds(N), s,
                         a, w, w.S, w.y, nullptr, 1, it, it == 0 ? 1 : 0);
    st = launch_status();
  }
  if (st == DPVO_OK) {
    hipLaunchKernelGGL(ba_apply_kernel, dim3(lin_grid(E)), dim3(256), 0, s, a, w, iterations);
    st = launch_status();
  }
  return st;
}

DPVO_EXPORT int dpvo_ba_plan_supported(int E, int t0, int t1, int P) {
  return (g_ba_path == 0 || g_ba_path == 5) && ba_window_supported(E, t1 - t0, P) ? 1 : 0;
}

DPVO_EXPORT int dpvo_ba_plan_offsets(int E, int t0, int t1, int64_t* out) {
  if (E <= 0 || t1 < t0 || !out) return DPVO_ERR_INVALID;
  if (!ba_window_supported(E, t1 - t0, 3)) return DPVO_ERR_UNSUPPORTED;
  const int64_t base = (int64_t)ba_layout(E, t1 - t0, nullptr, nullptr);
  ba_window_plan_offsets(E, out);
  for (int k = 0; k < 5; k++) out[k] += base;
  return DPVO_OK;
}

DPVO_EXPORT int dpvo_ba_plan(const int64_t* ii, const int64_t* jj, const int64_t* kk, int E,
                             int num_patches, int num_poses, int t0, int t1, void* workspace,
                             size_t workspace_bytes, void* stream) {
  if (E <= 0) return DPVO_OK;
  if (!ii || !jj || !kk || !workspace || num_patches <= 0 || num_poses <= 0 || t1 < t0)
    return DPVO_ERR_INVALID;
  if (!ba_window_supported(E, t1 - t0, 3)) return DPVO_ERR_UNSUPPORTED;
  if (workspace_bytes < dpvo_ba_workspace_bytes(E, t0, t1)) return DPVO_ERR_WORKSPACE;
  BaWs w;
  const size_t base_bytes = ba_layout(E, t1 - t0, (char*)workspace, &w);
  return ba_window_plan(ii, jj, kk, E, num_patches, num_poses, t0, t1,
                        (char*)workspace + base_bytes, w.meta + 1, stream, nullptr);
}

DPVO_EXPORT int dpvo_ba_forward_planned(float* poses, float* patches, const float* intrinsics,
                                        const float* target, const float* weight,
                                        const float* lmbda, const int64_t* ii, const int64_t* jj,
                                        const int64_t* kk, int E, int P, int num_poses,
                                        int num_patches, int t0, int t1, int iterations,
                                        void* workspace, size_t workspace_bytes, void* stream) {
  if (E <= 0 || iterations <= 0) return DPVO_OK;
  if (P < 2 || num_poses <= 0 || num_patches <= 0 || t1 < t0 || !workspace || !poses ||
      !patches || !intrinsics || !target || !weight || !lmbda || !ii || !jj || !kk)
    return DPVO_ERR_INVALID;
  if (!ba_window_supported(E, t1 - t0, P)) return DPVO_ERR_UNSUPPORTED;
  if (workspace_bytes < dpvo_ba_workspace_bytes(E, t0, t1)) return DPVO_ERR_WORKSPACE;
  BaWs w;
  const size_t base_bytes = ba_layout(E, t1 - t0, (char*)workspace, &w);
  return ba_window_run(poses, patches, intrinsics, target, weight, lmbda, ii, jj, kk, E, P,
                       num_poses, num_patches, t0, t1, iterations, (char*)workspace + base_bytes,
                       w.meta + 1, g_ba_marks ? w.tmark : nullptr, w.dX, stream, nullptr);
}

DPVO_EXPORT int dpvo_ba_forward_planned_dev(float* poses, float* patches, const float* intrinsics,
                                            const float* target, const float* weight,
                                            const float* lmbda, const int64_t* ii,
                                            const int64_t* jj, const int64_t* kk, int E, int P,
                                            int num_poses, int num_patches, const int32_t* t0_dev,
                                            int N, int iterations, void* workspace,
                                            size_t workspace_bytes, void* stream) {
  if (E <= 0 || iterations <= 0) return DPVO_OK;
  if (P < 2 || num_poses <= 0 || num_patches <= 0 || N < 0 || !t0_dev || !workspace || !poses ||
      !patches || !intrinsics || !target || !weight || !lmbda || !ii || !jj || !kk)
    return DPVO_ERR_INVALID;
  if (!ba_window_supported(E, N, P)) return DPVO_ERR_UNSUPPORTED;
  if (workspace_bytes < dpvo_ba_workspace_bytes(E, 0, N)) return DPVO_ERR_WORKSPACE;
  BaWs w;
  const size_t base_bytes = ba_layout(E, N, (char*)workspace, &w);
  return ba_window_run(poses, patches, intrinsics, target, weight, lmbda, ii, jj, kk, E, P,
                       num_poses, num_patches, 0, N, iterations, (char*)workspace + base_bytes,
                       w.meta + 1, g_ba_marks ? w.tmark : nullptr, w.dX, stream, t0_dev);
}

DPVO_EXPORT int dpvo_reproject(const float* poses, const float* patches, const float* intrinsics,
                               const int64_t* ii, const int64_t* jj, const int64_t* kk, int E,
                               int P, int num_poses, int num_patches, float* coords, void* stream) {
  if (E <= 0) return DPVO_OK;
  if (P <= 0 || num_poses <= 0 || num_patches <= 0) return DPVO_ERR_INVALID;
  const int total = E * P * P;
  hipLaunchKernelGGL(reproject_kernel, dim3((total + 255) / 256), dim3(256), 0,
                     as_stream(stream), poses, patches, intrinsics, ii, jj, kk, E, P, num_poses,
                     num_patches, coords, (int*)nullptr, 0);
  return launch_status();
}

DPVO_EXPORT int dpvo_reproject_ordered(const float* poses, const float* patches,
                                       const float* intrinsics, const int64_t* ii,
                                       const int64_t* jj, const int64_t* kk, int E, int P,
                                       int num_poses, int num_patches, int N2, float* coords,
                                       int32_t* order, void* stream) {
  if (E <= 0) return DPVO_OK;
  if (P <= 0 || num_poses <= 0 || num_patches <= 0 || !order) return DPVO_ERR_INVALID;
  const int total = E * P * P;
  // one more workgroup than the reprojection needs: it writes the edge order
  hipLaunchKernelGGL(reproject_kernel, dim3((total + 255) / 256 + 1), dim3(256), 0,
                     as_stream(stream), poses, patches, intrinsics, ii, jj, kk, E, P, num_poses,
                     num_patches, coords, (int*)order, N2);
  return launch_status();
}

DPVO_EXPORT int dpvo_reproject_ordered_plan(const float* poses, const float* patches,
                                            const float* intrinsics, const int64_t* ii,
                                            const int64_t* jj, const int64_t* kk, int E, int P,
                                            int num_poses, int num_patches, int N2, float* coords,
                                            int32_t* order, int t0, int t1, void* workspace,
                                            size_t workspace_bytes, void* stream) {
  if (E <= 0) return DPVO_OK;
  if (P <= 0 || num_poses <= 0 || num_patches <= 0 || !order || !coords || !poses || !patches ||
      !intrinsics || !ii || !jj || !kk || !workspace || t1 < t0)
    return DPVO_ERR_INVALID;
  if (!ba_window_supported(E, t1 - t0, P)) return DPVO_ERR_UNSUPPORTED;
  if (workspace_bytes < dpvo_ba_workspace_bytes(E, t0, t1)) return DPVO_ERR_WORKSPACE;
  BaWs w;
  const size_t base_bytes = ba_layout(E, t1 - t0, (char*)workspace, &w);
  return ba_window_reproject_plan(poses, patches, intrinsics, ii, jj, kk, E, P, num_poses,
                                  num_patches, N2, coords, (int*)order, t0, t1,
                                  (char*)workspace + base_bytes, w.meta + 1, stream, nullptr);
}

DPVO_EXPORT int dpvo_reproject_ordered_plan_insert(
    const float* poses, const float* patches, const float* intrinsics, const int64_t* ii,
    const int64_t* jj, const int64_t* kk, int E, int P, int num_poses, int num_patches, int N2,
    float* coords, int32_t* order, int t0, int t1, void* workspace, size_t workspace_bytes,
    const void* src, void* const* dst, const int* scale, int L, int C, int H, int W, int dtype,
    void* stream) {
  if (E <= 0) return DPVO_OK;
  if (P <= 0 || num_poses <= 0 || num_patches <= 0 || !order || !coords || !poses || !patches ||
      !intrinsics || !ii || !jj || !kk || !workspace || t1 < t0 || !src || !dst || !scale ||
      L <= 0 || C <= 0 || H <= 0 || W <= 0)
    return DPVO_ERR_INVALID;
  if ((dtype != DPVO_F32 && dtype != DPVO_F16) || L > 4) return DPVO_ERR_UNSUPPORTED;
  for (int l = 0; l < L; l++) {
    if (!dst[l]) return DPVO_ERR_INVALID;
    if (scale[l] != 1 && scale[l] != 2 && scale[l] != 4 && scale[l] != 8)
      return DPVO_ERR_UNSUPPORTED;
  }
  if (!ba_window_supported(E, t1 - t0, P)) return DPVO_ERR_UNSUPPORTED;
  if (workspace_bytes < dpvo_ba_workspace_bytes(E, t0, t1)) return DPVO_ERR_WORKSPACE;
  BaWs w;
  const size_t base_bytes = ba_layout(E, t1 - t0, (char*)workspace, &w);
  return ba_window_reproject_plan_insert(poses, patches, intrinsics, ii, jj, kk, E, P, num_poses,
                                         num_patches, N2, coords, (int*)order, t0, t1,
                                         (char*)workspace + base_bytes, w.meta + 1, src, dst,
                                         scale, L, C, H, W, dtype == DPVO_F16 ? 1 : 0,
                                         g_ba_marks ? w.tmark + kLaunchMarks : nullptr, stream);
}

DPVO_EXPORT int dpvo_reproject_ordered_plan_dev(const float* poses, const float* patches,
                                                const float* intrinsics, const int64_t* ii,
                                                const int64_t* jj, const int64_t* kk, int E, int P,
                                                int num_poses, int num_patches, int N2,
                                                float* coords, int32_t* order,
                                                const int32_t* t0_dev, int N, void* workspace,
                                                size_t workspace_bytes, void* stream) {
  if (E <= 0) return DPVO_OK;
  if (P <= 0 || num_poses <= 0 || num_patches <= 0 || !order || !coords || !poses || !patches ||
      !intrinsics || !ii || !jj || !kk || !workspace || !t0_dev || N < 0)
    return DPVO_ERR_INVALID;
  if (!ba_window_supported(E, N, P)) return DPVO_ERR_UNSUPPORTED;
  if (workspace_bytes < dpvo_ba_workspace_bytes(E, 0, N)) return DPVO_ERR_WORKSPACE;
  BaWs w;
  const size_t base_bytes = ba_layout(E, N, (char*)workspace, &w);
  return ba_window_reproject_plan(poses, patches, intrinsics, ii, jj, kk, E, P, num_poses,
                                  num_patches, N2, coords, (int*)order, 0, N,
                                  (char*)workspace + base_bytes, w.meta + 1, stream, t0_dev);
}

DPVO_EXPORT int dpvo_neighbors_max_edges(void) { return 1 << 30; }

DPVO_EXPORT int dpvo_neighbors(const int64_t* ii, const int64_t* jj, int E, int64_t* ix,
                               int64_t* jx, void* stream) {
  if (E <= 0) return DPVO_OK;
  hipLaunchKernelGGL(neighbors_kernel, dim3((E + 255) / 256), dim3(256), 0, as_stream(stream), ii,
                     jj, E, ix, jx);
  return launch_status();
}
