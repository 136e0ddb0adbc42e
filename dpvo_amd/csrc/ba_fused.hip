// ba_fused.hip -- F-BA for DPVO-sized windows in ONE single-workgroup launch.
//
// Reference semantics: dpvo/fastba/ba_cuda.cu:433-582 (cuda_ba) with the
// EfficentE Schur complement of block_e.cu:188-300: per iteration
//   per edge: residual + Jacobians in fp32 (ba_cuda.cu:265-333)
//   B, E, C, v, u sums (:339-373); Q = 1/(C + lmbda) (:519)
//   S = B - E Q E^T, y = v - E Q u (:554-558), S += I (1e-4 S + 1) (:560)
//   dX = chol_solve(S, y) (:561-562), dZ = Q (u - E^T dX) (:563)
//   pose_retr_kernel (:178-206), patch_retr_kernel (:209-229).
//
// Why one workgroup: a DPVO window (N <= 16 free poses, a few thousand edges)
// is latency-bound -- the fp64 work per iteration is ~0.6 MFLOP and the dense
// 6N x 6N solve is a chain of N dependent 6x6 pivots.  Spreading it over many
// CUs costs a cross-XCD handoff (L2 writeback + invalidate, ~2 us) per sync,
// two syncs per iteration, plus a launch per iteration.  Here the whole call
// (setup + every iteration + the final write-back) is one launch on one CU;
// every intermediate lives in LDS, syncs are 512-thread barriers (~70 ns).
//
// Structure (DESIGN.md "F-BA fused"):
//   setup   counting sort of the edges by patch (kk), (jj, edge) inside a
//           patch -> "positions"; patch table; pose table (free poses
//           t0..t1 plus nearby fixed ones) in LDS; a second counting sort of
//           positions by pose pair (ii, jj) -> chunks of <= kCB positions.
//   per iteration
//     E  thread per patch: linearise its edges -> C, u and the E column
//        block at the patch's source pose ("prim"), Q; other E entries
//        (target poses) to a per-position global scratch.
//     BS thread per pair chunk: re-linearise -> B blocks (ii,ii), (jj,jj),
//        (ii,jj), v, plus the Schur terms keyed by the same pair
//        (-Q e_j a^T, -Q e_j e_j^T, -Q u e_j) in 90 fp64 registers; one LDS
//        atomic flush per chunk.
//     D  (prim, prim) Schur terms -Q a a^T, -Q u a per run of patches.
//     X  cross terms -Q e_x e_y^T between different edges of one patch.
//     solve block LDL^T elimination with look-ahead pivot inversion, block
//        back substitution (lower 6x6 blocks in LDS, fp64).
//     update poses (LDS table + HBM), inverse depths (LDS patch table).
//   end  write every patch's inverse depth to all P x P entries.
// Per-edge arithmetic is the reference's fp32 (no FMA contraction, identical
// to the C oracle); every product of it and every sum is fp64.
#include "ba_device.hpp"

namespace dpvo {
namespace {
using namespace bad;

constexpr int kFT = 512;          // threads: 8 waves, 256 VGPRs for the 90 fp64 accumulators
constexpr int kFMaxN = 12;        // free poses handled by the fused path
constexpr int kFMaxE = 2048;      // edges handled by the fused path
constexpr int kPoseSlots = 64;    // LDS pose table: N free + nearby fixed poses
constexpr int kCB = 4;            // positions per pair chunk
constexpr int kSeg = 16;          // patches per (prim, prim) segment
constexpr int kHistMax = 8192;    // counting-sort range of kk (else bitonic)
constexpr int kFLds = 160 * 1024;
constexpr unsigned kFree = 0xFF;  // pose code of a fixed pose
constexpr unsigned kGlob = 0xFE;  // pose slot: read the pose from HBM
constexpr int kMarks = 64;

struct FArgs {
  float* poses;
  float* patches;
  const float* intrinsics;
  const float* target;
  const float* weight;
  const float* lmbda;
  const int64_t* ii;
  const int64_t* jj;
  const int64_t* kk;
  int E, P, num_poses, num_patches, t0, N, iters;
  // global scratch (workspace)
  double* PAg;      // [E][8]  per patch: Q, u, a[6] (when LDS is short)
  double* EJ;       // [E][12] per position: e_j[6], e_i[6] (entries off the prim pose)
  int* gidx;        // [E][2]  global pose indices (slot kGlob)
  int* kxg;         // [E]     patch id of each unique patch
  float* dbase;     // [E]     first-iteration retraction base (patch[2][0][0])
  double* dXg;      // [6N]    last dX
  int* meta;        // [8]     [1] status bits, [0] nuniq
  int64_t* marks;   // [kMarks] wall clock stamps (may be null)
};

__device__ __forceinline__ void stamp(int64_t* m, int slot) {
  if (m && threadIdx.x == 0) m[slot] = (int64_t)wall_clock64();
}


// ---------------------------------------------------------------------------
// LDS layout.  Fixed part (sized by E, N) then, after the sort, the patch
// table, the pair chunks and a band of per-patch sums; setup temporaries live
// at the top of the 160 KiB and are dead before the dynamic part is written.
// ---------------------------------------------------------------------------
struct FL {
  int* ctl;              // [64] control words (see kCtl*), [16..] scan scratch
  float* pose;           // [kPoseSlots][8] free poses t0.. then nearby fixed ones
  double* S;             // [NB][36] lower 6x6 blocks; diagonal blocks: lower triangle only
  double* y;             // [6N]
  double* piv;           // [N][36] LDL^T of the pivot blocks: L strictly lower, 1/D diagonal
  double* wv;            // [6N] L_k^-1 y_k of every pivot
  double* tt;            // [6N] back-substitution right-hand sides
  double* dX;            // [6N]
  double* PV;            // [N][36] panel V_i = S_ik L_k^-T D_k^-1 of the current step
  unsigned short* pu;    // [E] patch of each position
  unsigned short* pc;    // [E] pose slot of ii | slot of jj << 8
  unsigned short* pp;    // [E] pair order -> position
  float4* tw;            // [E] target.x, target.y, weight.x, weight.y per position
  // dynamic
  unsigned short* poff;  // [nuniq + 1] first position of each patch
  unsigned char* prim;   // [nuniq] free code of the patch's source pose
  float2* nxy;           // [nuniq] ((x - cx) / fx, (y - cy) / fy) of the patch centre
  float* dep;            // [nuniq] current inverse depth
  int* chunk;            // [nchunks] start | len << 16 (pair order)
  int* bchunk;           // [nbands + 1] first chunk of each band
  double* PA;            // [band size][8] Q, u, a[6] of the current band
};

enum {
  kCtlNuniq = 0, kCtlNchunks = 1, kCtlStatus = 2, kCtlFail = 3, kCtlKmin = 4, kCtlKmax = 5,
  kCtlFmin = 6, kCtlBad = 7, kCtlBand = 8, kCtlNbands = 9, kCtlScan = 16
};

__device__ __forceinline__ size_t aup(size_t v) { return (v + 15) & ~(size_t)15; }

struct Carver {
  char* base;
  size_t o;
  __device__ char* take(size_t b) {
    char* p = base + o;
    o = aup(o + b);
    return p;
  }
};

__device__ size_t carve_fixed(char* base, int E, int N, FL& L) {
  Carver c{base, 0};
  const int NB = N * (N + 1) / 2, N1 = N > 0 ? N : 1;
  L.ctl = (int*)c.take(sizeof(int) * 64);
  L.pose = (float*)c.take(sizeof(float) * 8 * kPoseSlots);
  L.S = (double*)c.take(sizeof(double) * 36 * (NB > 0 ? NB : 1));
  L.y = (double*)c.take(sizeof(double) * 6 * N1);
  L.piv = (double*)c.take(sizeof(double) * 36 * N1);
  L.wv = (double*)c.take(sizeof(double) * 6 * N1);
  L.tt = (double*)c.take(sizeof(double) * 6 * N1);
  L.dX = (double*)c.take(sizeof(double) * 6 * N1);
  L.PV = (double*)c.take(sizeof(double) * 36 * N1);
  L.pu = (unsigned short*)c.take(sizeof(unsigned short) * E);
  L.pc = (unsigned short*)c.take(sizeof(unsigned short) * E);
  L.pp = (unsigned short*)c.take(sizeof(unsigned short) * E);
  L.tw = (float4*)c.take(sizeof(float4) * E);
  return c.o;
}

__device__ __forceinline__ unsigned code_of(unsigned slot, int N) {
  return slot < (unsigned)N ? slot : kFree;
}

// ---------------------------------------------------------------------------
// accumulation helpers (LDS fp64 atomics; diagonal blocks keep the lower
// triangle only)
// ---------------------------------------------------------------------------
__device__ __forceinline__ void add_diag_lower(const FL& L, int a, const double* l21) {
  double* b = L.S + 36 * lblk(a, a);
  int k = 0;
#pragma unroll
  for (int x = 0; x < 6; x++)
#pragma unroll
    for (int z = 0; z <= x; z++) atomicAdd(b + 6 * x + z, l21[k++]);
}

// pair contribution: S gets M at (a, b) and M^T at (b, a); M row-major 6x6
__device__ __forceinline__ void add_pair(const FL& L, int a, int b, const double* M) {
  if (a > b) {
    double* p = L.S + 36 * lblk(a, b);
#pragma unroll
    for (int k = 0; k < 36; k++) atomicAdd(p + k, M[k]);
  } else if (a < b) {
    double* p = L.S + 36 * lblk(b, a);
#pragma unroll
    for (int x = 0; x < 6; x++)
#pragma unroll
      for (int z = 0; z < 6; z++) atomicAdd(p + 6 * z + x, M[6 * x + z]);
  } else {
    double* p = L.S + 36 * lblk(a, a);
#pragma unroll
    for (int x = 0; x < 6; x++)
#pragma unroll
      for (int z = 0; z <= x; z++)
        atomicAdd(p + 6 * x + z, (x == z) ? 2.0 * M[6 * x + z] : M[6 * x + z] + M[6 * z + x]);
  }
}

// pair contribution s u v^T at (a, b) (and its transpose at (b, a))
__device__ __forceinline__ void add_pair_outer(const FL& L, int a, int b, double s,
                                               const double* u, const double* v) {
  if (a > b) {
    double* p = L.S + 36 * lblk(a, b);
#pragma unroll
    for (int x = 0; x < 6; x++) {
      const double su = s * u[x];
#pragma unroll
      for (int z = 0; z < 6; z++) atomicAdd(p + 6 * x + z, su * v[z]);
    }
  } else if (a < b) {
    double* p = L.S + 36 * lblk(b, a);
#pragma unroll
    for (int x = 0; x < 6; x++) {
      const double su = s * u[x];
#pragma unroll
      for (int z = 0; z < 6; z++) atomicAdd(p + 6 * z + x, su * v[z]);
    }
  } else {
    double* p = L.S + 36 * lblk(a, a);
#pragma unroll
    for (int x = 0; x < 6; x++)
#pragma unroll
      for (int z = 0; z <= x; z++) {
        const double m = (s * u[x]) * v[z], mt = (s * u[z]) * v[x];
        atomicAdd(p + 6 * x + z, (x == z) ? 2.0 * m : m + mt);
      }
  }
}

__device__ __forceinline__ const float* pose_ptr(const FArgs& A, const FL& L, unsigned slot,
                                                 int p, int which) {
  return slot == kGlob ? A.poses + 7 * (size_t)A.gidx[2 * p + which] : L.pose + 8 * slot;
}


// ---------------------------------------------------------------------------
// the kernel
// ---------------------------------------------------------------------------
constexpr int kRE = kFMaxE / kFT;  // edges per thread in the setup

__global__ void __launch_bounds__(kFT) ba_fused_kernel(FArgs A) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  const int tid = threadIdx.x, T = kFT, lane = tid & 63, wid = tid >> 6;
  const int E = A.E, N = A.N, t0 = A.t0, P = A.P, PP = P * P;
  FL L;
  const size_t fixed_end = carve_fixed(lds, E, N, L);
  int* ctl = L.ctl;
  int* scr = ctl + kCtlScan;
  const float fx = A.intrinsics[0], fy = A.intrinsics[1], cx = A.intrinsics[2],
              cy = A.intrinsics[3];
  const int kmaxc = A.num_patches - 1;
  stamp(A.marks, 0);

  // ============================ setup ============================
  // S1: every thread keeps its edges e = tid + r T in registers
  int ekv[kRE], egi[kRE], egj[kRE];
  float4 etw[kRE];
  {
    int lmin = 0x7fffffff, lmax = -1, bad = 0, fmin = 0x7fffffff;
#pragma unroll
    for (int r = 0; r < kRE; r++) {
      const int e = tid + r * T;
      ekv[r] = 0;
      egi[r] = egj[r] = 0;
      if (e < E) {
        int64_t v = A.kk[e];
        if (v < 0 || v > kmaxc) {
          bad = 1;
          v = v < 0 ? 0 : kmaxc;
        }
        ekv[r] = (int)v;
        const int64_t gi = A.ii[e], gj = A.jj[e];
        // free poses keep their code; others are clamped for memory safety
        egi[r] = (gi >= t0 && gi < t0 + N) ? (int)gi
                                           : (int)min(max(gi, (int64_t)0), (int64_t)A.num_poses - 1);
        egj[r] = (gj >= t0 && gj < t0 + N) ? (int)gj
                                           : (int)min(max(gj, (int64_t)0), (int64_t)A.num_poses - 1);
        if (!(gi >= t0 && gi < t0 + N)) fmin = min(fmin, egi[r]);
        if (!(gj >= t0 && gj < t0 + N)) fmin = min(fmin, egj[r]);
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
      ctl[kCtlKmin] = 0x7fffffff;
      ctl[kCtlKmax] = -1;
      ctl[kCtlFmin] = 0x7fffffff;
      ctl[kCtlBad] = 0;
      ctl[kCtlFail] = 0;
    }
    __syncthreads();
    if (lane == 0) {
      atomicMin(&ctl[kCtlKmin], lmin);
      atomicMax(&ctl[kCtlKmax], lmax);
      atomicMin(&ctl[kCtlFmin], fmin);
      atomicOr(&ctl[kCtlBad], bad);
    }
    __syncthreads();
  }
  const int kmin = ctl[kCtlKmin], R = ctl[kCtlKmax] - kmin + 1, fmin = ctl[kCtlFmin];
  auto slot_of = [&](int g) -> unsigned {
    if (g >= t0 && g < t0 + N) return (unsigned)(g - t0);
    const int k = g - fmin;
    return (k >= 0 && k < kPoseSlots - N) ? (unsigned)(N + k) : kGlob;
  };
  // S2: positions = edges sorted by (kk, jj, edge); epos[e] = position of e
  char* top = lds + kFLds;
  int* epos = (int*)(top - sizeof(int) * kFMaxE);
  int* ehead = epos - kFMaxE;     // heads -> patch index (scan)
  int* spos = ehead - kFMaxE;     // sort keys / sorted edge per position
  {
    if (R <= kHistMax) {
      int* hist = spos - kHistMax;
      for (int v = tid; v < R; v += T) hist[v] = 0;
      __syncthreads();
#pragma unroll
      for (int r = 0; r < kRE; r++)
        if (tid + r * T < E) atomicAdd(&hist[ekv[r] - kmin], 1);
      __syncthreads();
      fscan(hist, R, scr);  // bucket starts
#pragma unroll
      for (int r = 0; r < kRE; r++) {
        const int e = tid + r * T;
        if (e < E) {
          const int jc = min(max(egj[r], 0), 32767);
          spos[atomicAdd(&hist[ekv[r] - kmin], 1)] = (jc << 16) | e;
        }
      }
      __syncthreads();
      // hist[v] = end of bucket v: insertion-sort each bucket, mark heads
      for (int v = tid; v < R; v += T) {
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
      unsigned long long* keys = (unsigned long long*)(spos - 2 * kFMaxE);
      for (int i = tid; i < P2; i += T) keys[i] = ~0ull;
      __syncthreads();
#pragma unroll
      for (int r = 0; r < kRE; r++) {
        const int e = tid + r * T;
        if (e < E) {
          const int jc = min(max(egj[r], 0), 32767);
          keys[e] = ((unsigned long long)ekv[r] << 32) | ((unsigned)jc << 16) | (unsigned)e;
        }
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
    __syncthreads();
  }
  // S3: per-position tables (edge owners scatter), patch index of each position
  const int nuniq = fscan(ehead, E, scr) ;  // ehead[p] = #heads before p
  {
#pragma unroll
    for (int r = 0; r < kRE; r++) {
      const int e = tid + r * T;
      if (e < E) {
        const int p = epos[e];
        const unsigned si = slot_of(egi[r]), sj = slot_of(egj[r]);
        L.pc[p] = (unsigned short)(si | (sj << 8));
        L.tw[p] = etw[r];
        A.gidx[2 * p] = egi[r];
        A.gidx[2 * p + 1] = egj[r];
      }
    }
    __syncthreads();  // pc complete (read for prim below)
  }
  // per position: patch index; per head: patch record (registers until the
  // setup temporaries are dead)
  int hu[kRE], hp[kRE], hkx[kRE];
#pragma unroll
  for (int r = 0; r < kRE; r++) {
    const int p = tid + r * T;
    hu[r] = -1;
    if (p < E) {
      const int nx = (p + 1 < E) ? ehead[p + 1] : nuniq;
      const int u = nx - 1;
      L.pu[p] = (unsigned short)u;
      if (ehead[p] != nx) {  // p is the first position of patch u
        hu[r] = u;
        hp[r] = p;
        hkx[r] = min(max((int)A.kk[spos[p] & 0xffff], 0), kmaxc);
      }
    }
  }
  __syncthreads();  // setup temporaries dead from here
  int nchunks, nbands, bsz;
  {
    Carver c{lds, fixed_end};
    L.poff = (unsigned short*)c.take(sizeof(unsigned short) * (nuniq + 1));
    L.prim = (unsigned char*)c.take(nuniq);
    L.nxy = (float2*)c.take(sizeof(float2) * nuniq);
    L.dep = (float*)c.take(sizeof(float) * nuniq);
    // patch records
#pragma unroll
    for (int r = 0; r < kRE; r++) {
      if (hu[r] < 0) continue;
      const int u = hu[r], p = hp[r], kx = hkx[r];
      L.poff[u] = (unsigned short)p;
      L.prim[u] = (unsigned char)code_of(L.pc[p] & 0xff, N);
      const float* pk = A.patches + (size_t)kx * 3 * PP;
      const int c11 = P + 1;  // [*][1][1] (ba_cuda.cu:282-285)
      L.nxy[u] = make_float2((pk[c11] - cx) / fx, (pk[PP + c11] - cy) / fy);  // (:282-285)
      L.dep[u] = pk[2 * PP + c11];
      A.dbase[u] = pk[2 * PP];  // patch_retr_kernel reads [2][0][0] (:225)
      A.kxg[u] = kx;
    }
    if (tid == 0) L.poff[nuniq] = (unsigned short)E;
    // pose table
    for (int k = tid; k < kPoseSlots * 8; k += T) {
      const int sl = k >> 3, cc = k & 7;
      const int g = (sl < N) ? t0 + sl : fmin + (sl - N);
      float v = (cc == 6) ? 1.0f : 0.0f;
      if (cc < 7 && g >= 0 && g < A.num_poses && (sl < N || fmin != 0x7fffffff))
        v = A.poses[7 * (size_t)g + cc];
      L.pose[k] = v;
    }
    // bands of patches whose sums (Q, u, a) fit in LDS next to the chunks
    const int NK = (N + 1) * (N + 1);
    const size_t after_patch = c.o;
    const size_t chunk_bytes = aup(sizeof(int) * (E + 8 * NK + 8));
    bsz = (int)((kFLds - aup(after_patch + chunk_bytes)) / (8 * sizeof(double)));
    bsz = max(1, min(bsz, nuniq));
    nbands = (nuniq + bsz - 1) / bsz;
    L.chunk = (int*)c.take(sizeof(int) * E);
    L.bchunk = (int*)c.take(sizeof(int) * (nbands + 1));
    L.PA = (double*)(lds + aup(after_patch + chunk_bytes));
    // pair order.  key = band * NK + code(ci) * (N + 1) + code(cj) (fixed
    // pose -> N); positions without a free pose are dropped.  The counters
    // alias the per-patch sums (setup only).
    const int K = nbands * NK;
    int* kc = (int*)L.PA;
    int* kn = kc + K;
    int* kfill = kn + K;
    for (int k = tid; k < K; k += T) kc[k] = 0;
    __syncthreads();
    auto key_of = [&](int p) -> int {
      const unsigned b = L.pc[p];
      const unsigned ci = code_of(b & 0xff, N), cj = code_of(b >> 8, N);
      if (ci == kFree && cj == kFree) return -1;
      return (L.pu[p] / bsz) * NK + (ci == kFree ? N : (int)ci) * (N + 1) +
             (cj == kFree ? N : (int)cj);
    };
    for (int p = tid; p < E; p += T) {
      const int key = key_of(p);
      if (key >= 0) atomicAdd(&kc[key], 1);
    }
    __syncthreads();
    for (int k = tid; k < K; k += T) kn[k] = (kc[k] + kCB - 1) / kCB;
    __syncthreads();
    const int npair = fscan(kc, K, scr);
    nchunks = fscan(kn, K, scr);
    for (int k = tid; k < K; k += T) kfill[k] = kc[k];
    __syncthreads();
    for (int p = tid; p < E; p += T) {
      const int key = key_of(p);
      if (key >= 0) L.pp[atomicAdd(&kfill[key], 1)] = (unsigned short)p;
    }
    for (int k = tid; k < K; k += T) {
      const int st = kc[k], n = ((k + 1 < K) ? kc[k + 1] : npair) - st;
      for (int q = 0; q * kCB < n; q++)
        L.chunk[kn[k] + q] = (st + q * kCB) | (min(kCB, n - q * kCB) << 16);
    }
    for (int b = tid; b <= nbands; b += T) L.bchunk[b] = (b < nbands) ? kn[b * NK] : nchunks;
    if (tid == 0) {
      ctl[kCtlNuniq] = nuniq;
      ctl[kCtlNchunks] = nchunks;
      ctl[kCtlStatus] = ctl[kCtlBad] ? 2 : 0;
    }
    __syncthreads();
  }
  stamp(A.marks, 1);

  const double lam = (double)A.lmbda[0];
  const int NB = N * (N + 1) / 2;
  // ============================ iterations ============================
  for (int it = 0; it < A.iters; it++) {
    const int mb = 2 + 8 * it;
    for (int k = tid; k < 36 * NB; k += T) L.S[k] = 0.0;
    for (int k = tid; k < 6 * N; k += T) L.y[k] = 0.0;
    for (int band = 0; band < nbands; band++) {
      const int u0 = band * bsz, u1 = min(u0 + bsz, nuniq);
      __syncthreads();
      // ---- E: thread per patch -> Q, u, a (entries at the source pose) ----
      for (int u = u0 + tid; u < u1; u += T) {
        const unsigned pr = L.prim[u];
        const float2 nxy = L.nxy[u];
        const float dp = L.dep[u];
        double C = 0.0, U = 0.0, a[6] = {0, 0, 0, 0, 0, 0};
        const int p1 = L.poff[u + 1];
        for (int p = L.poff[u]; p < p1; p++) {
          const unsigned b = L.pc[p];
          const unsigned si = b & 0xff, sj = b >> 8;
          const unsigned ci = code_of(si, N), cj = code_of(sj, N);
          const float4 tw = L.tw[p];
          Lin o;
          lin_edge(pose_ptr(A, L, si, p, 0), pose_ptr(A, L, sj, p, 1), nxy.x, nxy.y, dp, tw.x,
                   tw.y, tw.z, tw.w, fx, fy, cx, cy, o);
          double ei[6] = {0, 0, 0, 0, 0, 0}, ej[6] = {0, 0, 0, 0, 0, 0};
#pragma unroll
          for (int row = 0; row < 2; row++) {  // ba_cuda.cu:352-373
            const double wr = o.w[row];
            const double wz = wr * (double)o.Jz[row];
#pragma unroll
            for (int k = 0; k < 6; k++) {
              ei[k] -= wz * (double)o.Ji[row][k];
              ej[k] += wz * (double)o.Jj[row][k];
            }
            C += wz * (double)o.Jz[row];
            U += (wr * (double)o.r[row]) * (double)o.Jz[row];
          }
          const bool ipr = ci != kFree && ci == pr, jpr = cj != kFree && cj == pr;
#pragma unroll
          for (int k = 0; k < 6; k++) a[k] += (ipr ? ei[k] : 0.0) + (jpr ? ej[k] : 0.0);
          const bool ej_on = cj != kFree && !jpr, ei_on = ci != kFree && !ipr;
          if (ej_on || ei_on) {  // entries off the source pose: cross terms, depth update
            double2* out = reinterpret_cast<double2*>(A.EJ + 12 * (size_t)p);
#pragma unroll
            for (int k = 0; k < 3; k++) {
              out[k] = make_double2(ej_on ? ej[2 * k] : 0.0, ej_on ? ej[2 * k + 1] : 0.0);
              out[3 + k] = make_double2(ei_on ? ei[2 * k] : 0.0, ei_on ? ei[2 * k + 1] : 0.0);
            }
          }
        }
        double* pa = L.PA + 8 * (size_t)(u - u0);
        pa[0] = 1.0 / (C + lam);  // Q (:519)
        pa[1] = U;
#pragma unroll
        for (int k = 0; k < 6; k++) pa[2 + k] = a[k];
        if (nbands > 1) {
          double2* g = reinterpret_cast<double2*>(A.PAg + 8 * (size_t)u);
#pragma unroll
          for (int k = 0; k < 4; k++) g[k] = make_double2(pa[2 * k], pa[2 * k + 1]);
        }
      }
      __syncthreads();
      if (band == nbands - 1) stamp(A.marks, mb + 0);
      if (N == 0) continue;

      // ---- BS: thread per pair chunk of this band ----
      const int c0 = L.bchunk[band], nc = L.bchunk[band + 1] - c0;
      int cstride = max(1, nc / 64 + 1);  // spread one pair's chunks over lanes
      {
        auto gcd = [](int a, int b) {
          while (b) {
            const int t = a % b;
            a = b;
            b = t;
          }
          return a;
        };
        while (nc > 0 && gcd(cstride, nc) != 1) cstride++;
      }
      for (int t = tid; t < nc; t += T) {
        const int cw = L.chunk[c0 + (int)(((long long)t * cstride) % nc)];
        const int cs = cw & 0xffff, cl = cw >> 16;
        const unsigned b0 = L.pc[L.pp[cs]];
        const unsigned ci = code_of(b0 & 0xff, N), cj = code_of(b0 >> 8, N);
        const bool fi = ci != kFree, fj = cj != kFree;
        double Bii[21], Bjj[21], Bij[36], vi[6], vj[6];
#pragma unroll
        for (int k = 0; k < 21; k++) Bii[k] = Bjj[k] = 0.0;
#pragma unroll
        for (int k = 0; k < 36; k++) Bij[k] = 0.0;
#pragma unroll
        for (int k = 0; k < 6; k++) vi[k] = vj[k] = 0.0;
        for (int q = 0; q < cl; q++) {
          const int p = L.pp[cs + q];
          const int u = L.pu[p];
          const unsigned b = L.pc[p];
          const float4 tw = L.tw[p];
          const float2 nxy = L.nxy[u];
          Lin o;
          lin_edge(pose_ptr(A, L, b & 0xff, p, 0), pose_ptr(A, L, b >> 8, p, 1), nxy.x, nxy.y,
                   L.dep[u], tw.x, tw.y, tw.z, tw.w, fx, fy, cx, cy, o);
          // B and v (ba_cuda.cu:339-370)
#pragma unroll
          for (int row = 0; row < 2; row++) {
            const double wr = o.w[row];
            const double wrr = wr * (double)o.r[row];
            int k = 0;
#pragma unroll
            for (int x = 0; x < 6; x++) {
              const double ti = wr * (double)o.Ji[row][x];
              const double tj = wr * (double)o.Jj[row][x];
#pragma unroll
              for (int z = 0; z <= x; z++, k++) {
                Bii[k] += ti * (double)o.Ji[row][z];
                Bjj[k] += tj * (double)o.Jj[row][z];
              }
#pragma unroll
              for (int z = 0; z < 6; z++) Bij[6 * x + z] -= ti * (double)o.Jj[row][z];
              vi[x] -= wrr * (double)o.Ji[row][x];
              vj[x] += wrr * (double)o.Jj[row][x];
            }
          }
          // Schur terms of this edge's E entries (entries at fixed poses dropped)
          const unsigned pr = L.prim[u];
          const bool ej_on = fj && cj != pr, ei_on = fi && ci != pr;
          if (ej_on || ei_on) {
            const double* pa = L.PA + 8 * (size_t)(u - u0);
            const double Q = pa[0], QU = pa[0] * pa[1];
            double ej[6] = {0, 0, 0, 0, 0, 0}, ei[6] = {0, 0, 0, 0, 0, 0};
#pragma unroll
            for (int row = 0; row < 2; row++) {  // same sums as the E phase
              const double wz = (double)o.w[row] * (double)o.Jz[row];
#pragma unroll
              for (int k = 0; k < 6; k++) {
                ei[k] -= wz * (double)o.Ji[row][k];
                ej[k] += wz * (double)o.Jj[row][k];
              }
            }
            if (ej_on) {  // -Q e_j e_j^T, -Q u e_j, -Q e_j a^T at (cj, prim)
              int k = 0;
#pragma unroll
              for (int x = 0; x < 6; x++) {
                const double qe = Q * ej[x];
#pragma unroll
                for (int z = 0; z <= x; z++, k++) Bjj[k] -= qe * ej[z];
                vj[x] -= QU * ej[x];
              }
              if (fi && ci == pr) {  // rows ci of the (ci, cj) pair block
#pragma unroll
                for (int x = 0; x < 6; x++) {
                  const double qa = Q * pa[2 + x];
#pragma unroll
                  for (int z = 0; z < 6; z++) Bij[6 * x + z] -= qa * ej[z];
                }
              } else if (pr != kFree) {
                add_pair_outer(L, (int)cj, (int)pr, -Q, ej, pa + 2);
              }
            }
            if (ei_on) {  // source-pose entry off the patch's prim (general graphs)
              int k = 0;
#pragma unroll
              for (int x = 0; x < 6; x++) {
                const double qe = Q * ei[x];
#pragma unroll
                for (int z = 0; z <= x; z++, k++) Bii[k] -= qe * ei[z];
                vi[x] -= QU * ei[x];
              }
              if (pr != kFree) add_pair_outer(L, (int)ci, (int)pr, -Q, ei, pa + 2);
              if (ej_on)  // the edge's two entries: (ci, cj) pair block
#pragma unroll
                for (int x = 0; x < 6; x++) {
                  const double qe = Q * ei[x];
#pragma unroll
                  for (int z = 0; z < 6; z++) Bij[6 * x + z] -= qe * ej[z];
                }
            }
          }
        }
        // flush (fixed poses dropped, ba_cuda.cu:341-345)
        if (fi) {
          add_diag_lower(L, (int)ci, Bii);
#pragma unroll
          for (int x = 0; x < 6; x++) atomicAdd(&L.y[6 * ci + x], vi[x]);
        }
        if (fj) {
          add_diag_lower(L, (int)cj, Bjj);
#pragma unroll
          for (int x = 0; x < 6; x++) atomicAdd(&L.y[6 * cj + x], vj[x]);
        }
        if (fi && fj) add_pair(L, (int)ci, (int)cj, Bij);
      }

      // ---- D: (prim, prim) terms -Q a a^T, -Q u a; thread per (segment, row) ----
      const int nseg = (u1 - u0 + kSeg - 1) / kSeg;
      for (int t = tid; t < 6 * nseg; t += T) {
        const int sg = t / 6, x = t % 6;
        const int s0 = u0 + sg * kSeg, s1 = min(s0 + kSeg, u1);
        unsigned cur = L.prim[s0];
        double acc[6] = {0, 0, 0, 0, 0, 0}, yacc = 0.0;
        for (int u = s0; u <= s1; u++) {
          const unsigned pr = (u < s1) ? L.prim[u] : 0xFFFFu;
          if (pr != cur) {
            if (cur != kFree) {
              double* bk = L.S + 36 * lblk((int)cur, (int)cur) + 6 * x;
              for (int z = 0; z <= x; z++) atomicAdd(bk + z, acc[z]);
              atomicAdd(&L.y[6 * cur + x], yacc);
            }
#pragma unroll
            for (int z = 0; z < 6; z++) acc[z] = 0.0;
            yacc = 0.0;
            cur = pr;
          }
          if (u == s1 || pr == kFree) continue;
          const double* pa = L.PA + 8 * (size_t)(u - u0);
          const double qa = pa[0] * pa[2 + x];
#pragma unroll
          for (int z = 0; z < 6; z++) acc[z] -= qa * pa[2 + z];  // (:554-556)
          yacc -= (pa[0] * pa[1]) * pa[2 + x];                   // (:557-558)
        }
      }
      // ---- X: cross terms between entries of different edges of a patch ----
      for (int u = u0 + tid; u < u1; u += T) {
        const int p0 = L.poff[u], p1 = L.poff[u + 1];
        if (p1 - p0 < 2) continue;
        const unsigned pr = L.prim[u];
        const double Q = L.PA[8 * (size_t)(u - u0)];
        for (int p = p0; p < p1; p++) {
          const unsigned bp = L.pc[p];
          const unsigned cpi = code_of(bp & 0xff, N), cpj = code_of(bp >> 8, N);
          const bool pj_on = cpj != kFree && cpj != pr, pi_on = cpi != kFree && cpi != pr;
          if (!pj_on && !pi_on) continue;
          for (int q = p + 1; q < p1; q++) {
            const unsigned bq = L.pc[q];
            const unsigned cqi = code_of(bq & 0xff, N), cqj = code_of(bq >> 8, N);
            const bool qj_on = cqj != kFree && cqj != pr, qi_on = cqi != kFree && cqi != pr;
            if (!qj_on && !qi_on) continue;
            for (int xs = 0; xs < 2; xs++) {
              if (!(xs == 0 ? pj_on : pi_on)) continue;
              double ex[6];
              load6(A.EJ + 12 * (size_t)p + 6 * xs, ex);
              const int ax = (int)(xs == 0 ? cpj : cpi);
              for (int ys = 0; ys < 2; ys++) {
                if (!(ys == 0 ? qj_on : qi_on)) continue;
                double ey[6];
                load6(A.EJ + 12 * (size_t)q + 6 * ys, ey);
                add_pair_outer(L, ax, (int)(ys == 0 ? cqj : cqi), -Q, ex, ey);
              }
            }
          }
        }
      }
    }
    __syncthreads();
    stamp(A.marks, mb + 1);

    // ============================ solve ============================
    int fail = 0;
    if (N > 0) {
      for (int k = tid; k < 6 * N; k += T) {  // S += I (1e-4 S + 1) (ba_cuda.cu:560)
        double* d = L.S + 36 * lblk(k / 6, k / 6) + 7 * (k % 6);
        *d += 1e-4 * *d + 1.0;
      }
      __syncthreads();
      if (tid == 0 && !ldl6(L.S, L.y, L.piv, L.wv)) ctl[kCtlFail] = 1;
      __syncthreads();
      // block LDL^T elimination, step k:
      //   W_i = S_ik L_k^-T (stored in S_ik), V_i = W_i D_k^-1, y_i -= V_i w_k   (i > k)
      //   S_ij -= V_i W_j^T                                              (k < j <= i)
      // the pivot block k+1 is finished and factored first (wave 0, look-ahead).
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
        for (int t = tid; t < 6 * (m * (m + 1) / 2); t += T) {
          const int x = t % 6;
          int a, b;
          tri_of(t / 6, a, b);
          const int i = k + 1 + a, j = k + 1 + b;
          const double* Vi = L.PV + 36 * i + 6 * x;
          const double* Wj = L.S + 36 * lblk(j, k);
          double* Sij = L.S + 36 * lblk(i, j) + 6 * x;
          double v[6];
#pragma unroll
          for (int q = 0; q < 6; q++) v[q] = Vi[q];
          const int zn = (i == j) ? x + 1 : 6;  // diagonal blocks: lower triangle
          for (int z = 0; z < zn; z++) {
            double s = Sij[z];
#pragma unroll
            for (int q = 0; q < 6; q++) s -= v[q] * Wj[6 * z + q];
            Sij[z] = s;
          }
        }
        if (m > 0 && wid == 0) {  // tasks 0..5 = rows of block (k+1, k+1): wave 0
          wave_lds_sync();
          if (tid == 0 && !ldl6(L.S + 36 * lblk(k + 1, k + 1), L.y + 6 * (k + 1),
                                L.piv + 36 * (k + 1), L.wv + 6 * (k + 1)))
            ctl[kCtlFail] = 1;
        }
        __syncthreads();
      }
      // back substitution: x_k = L_k^-T D_k^-1 (w_k - sum_{i>k} W_ik^T x_i)
      for (int k = tid; k < 6 * N; k += T) L.tt[k] = L.wv[k];
      __syncthreads();
      for (int i = N - 1; i >= 0; i--) {
        const double* pi_ = L.piv + 36 * i;
        for (int t = tid; t < 6 * (i + 1); t += T) {
          const int k = t / 6, x = t % 6;
          double xi[6];
#pragma unroll
          for (int q = 5; q >= 0; q--) {
            double s = L.tt[6 * i + q] * pi_[7 * q];
#pragma unroll
            for (int pq = q + 1; pq < 6; pq++) s -= pi_[6 * pq + q] * xi[pq];
            xi[q] = s;
          }
          if (k == i) {
            L.dX[6 * i + x] = xi[x];
          } else {
            const double* Wik = L.S + 36 * lblk(i, k);
            double s = L.tt[6 * k + x];
#pragma unroll
            for (int q = 0; q < 6; q++) s -= Wik[6 * q + x] * xi[q];
            L.tt[6 * k + x] = s;
          }
        }
        __syncthreads();
      }
      fail = ctl[kCtlFail];
      if (fail)
        for (int k = tid; k < 6 * N; k += T) L.dX[k] = 0.0;  // dX = 0 (dpvo/ba.py:17-21)
      __syncthreads();
      // pose retraction (pose_retr_kernel :178-206)
      for (int i = tid; i < N; i += T) {
        float xi[6], tt[3], qq[4], t1[3], q1[4];
#pragma unroll
        for (int k = 0; k < 6; k++) xi[k] = (float)L.dX[6 * i + k];
        float* pl = L.pose + 8 * i;
        tt[0] = pl[0]; tt[1] = pl[1]; tt[2] = pl[2];
        qq[0] = pl[3]; qq[1] = pl[4]; qq[2] = pl[5]; qq[3] = pl[6];
        retrSE3(xi, tt, qq, t1, q1);
        pl[0] = t1[0]; pl[1] = t1[1]; pl[2] = t1[2];
        pl[3] = q1[0]; pl[4] = q1[1]; pl[5] = q1[2]; pl[6] = q1[3];
        const int g = t0 + i;
        if (g >= 0 && g < A.num_poses) {
          float* pg = A.poses + 7 * (size_t)g;
#pragma unroll
          for (int c = 0; c < 7; c++) pg[c] = pl[c];
        }
      }
      for (int k = tid; k < 6 * N; k += T) A.dXg[k] = L.dX[k];
    }
    stamp(A.marks, mb + 2);
    // ---- inverse depths: dZ = Q (u - E^T dX) (:563), patch_retr_kernel ----
    for (int u = tid; u < nuniq; u += T) {
      double pa[8];
      const double* src = (nbands == 1) ? L.PA + 8 * (size_t)u : A.PAg + 8 * (size_t)u;
#pragma unroll
      for (int k = 0; k < 8; k++) pa[k] = src[k];
      const unsigned pr = L.prim[u];
      double ex = 0.0;
      if (N > 0) {
        if (pr != kFree)
#pragma unroll
          for (int k = 0; k < 6; k++) ex += pa[2 + k] * L.dX[6 * pr + k];
        for (int p = L.poff[u]; p < L.poff[u + 1]; p++) {
          const unsigned b = L.pc[p];
          const unsigned ci = code_of(b & 0xff, N), cj = code_of(b >> 8, N);
          const bool ej_on = cj != kFree && cj != pr, ei_on = ci != kFree && ci != pr;
          if (!ej_on && !ei_on) continue;
          double e6[6];
          if (ej_on) {
            load6(A.EJ + 12 * (size_t)p, e6);
#pragma unroll
            for (int k = 0; k < 6; k++) ex += e6[k] * L.dX[6 * cj + k];
          }
          if (ei_on) {
            load6(A.EJ + 12 * (size_t)p + 6, e6);
#pragma unroll
            for (int k = 0; k < 6; k++) ex += e6[k] * L.dX[6 * ci + k];
          }
        }
      }
      const float dz = (float)(pa[0] * (pa[1] - ex));
      const float base = (it == 0) ? A.dbase[u] : L.dep[u];
      float d = base + dz;
      d = (d > 20.0f) ? 1.0f : d;
      L.dep[u] = (float)fmax((double)d, 1e-4);
    }
    if (tid == 0) ctl[kCtlStatus] = (ctl[kCtlStatus] & ~1) | (fail ? 1 : 0);
    __syncthreads();
    stamp(A.marks, mb + 3);
  }
  // ============================ write back ============================
  for (int k = tid; k < nuniq * PP; k += T) {
    const int u = k / PP, c = k % PP;
    A.patches[(size_t)A.kxg[u] * 3 * PP + 2 * PP + c] = L.dep[u];
  }
  if (tid == 0) {
    A.meta[0] = nuniq;
    A.meta[1] = ctl[kCtlStatus];
  }
  stamp(A.marks, 63);
}

}  // namespace

// host side ------------------------------------------------------------------
size_t ba_fused_scratch_bytes(int E, int N) {
  auto al = [](size_t v) { return (v + 255) / 256 * 256; };
  return al(sizeof(double) * 8 * E) + al(sizeof(double) * 12 * E) + al(sizeof(int) * 2 * E) +
         al(sizeof(int) * E) + al(sizeof(float) * E) + al(sizeof(double) * 6 * (N > 0 ? N : 1));
}

bool ba_fused_supported(int E, int N, int P) {
  return E > 0 && E <= kFMaxE && N >= 0 && N <= kFMaxN && P >= 2 && P * P <= 64;
}

int ba_fused_launch(float* poses, float* patches, const float* intrinsics, const float* target,
                    const float* weight, const float* lmbda, const int64_t* ii, const int64_t* jj,
                    const int64_t* kk, int E, int P, int num_poses, int num_patches, int t0, int t1,
                    int iterations, char* scratch, int* meta, int64_t* marks, void* stream) {
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)ba_fused_kernel,
                              hipFuncAttributeMaxDynamicSharedMemorySize, kFLds);
    attr = true;
  }
  auto al = [](size_t v) { return (v + 255) / 256 * 256; };
  FArgs a;
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
  a.iters = iterations;
  char* s = scratch;
  a.PAg = (double*)s;
  s += al(sizeof(double) * 8 * E);
  a.EJ = (double*)s;
  s += al(sizeof(double) * 12 * E);
  a.gidx = (int*)s;
  s += al(sizeof(int) * 2 * E);
  a.kxg = (int*)s;
  s += al(sizeof(int) * E);
  a.dbase = (float*)s;
  s += al(sizeof(float) * E);
  a.dXg = (double*)s;
  a.meta = meta;
  a.marks = marks;
  hipLaunchKernelGGL(ba_fused_kernel, dim3(1), dim3(kFT), kFLds, as_stream(stream), a);
  return launch_status();
}

}  // namespace dpvo
