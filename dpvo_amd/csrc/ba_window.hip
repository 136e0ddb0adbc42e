// ba_window.hip -- F-BA for DPVO local-BA windows (N <= 16 free poses,
// E <= 10240 edges, DPVO MAX_EDGES = 10000): the default path of
// cuda_ba.forward for those shapes.
//
// Reference semantics: dpvo/fastba/ba_cuda.cu:433-582 (block_e.cu:188-300 for
// the block-sparse E):
//   per edge: residual + Jacobians in fp32 (ba_cuda.cu:265-333)
//   B, E, C, v, u (:339-373); Q = 1/(C + lmbda) (:519)
//   S = B - E Q E^T, y = v - E Q u (:554-558), S += I (1e-4 S + 1) (:560)
//   dX = chol_solve(S, y) (:561-562), dZ = Q (u - E^T dX) (:563)
//   pose_retr_kernel (:178-206), patch_retr_kernel (:209-229).
//
// MI355X design (DESIGN.md "F-BA for DPVO windows").  A window is
// latency-bound (~0.5 MB of compulsory traffic per call), so the aim is the
// shortest dependency chain, not bandwidth:
//   * ba_plan_kernel (one 512-thread workgroup, depends on ii/jj/kk only):
//     groups the edges by patch ONCE (counting sort on kk in LDS, bitonic if
//     the kk range is too wide; deterministic order inside a patch) and
//     writes patch offsets + free-pose masks.  Because it reads no pose,
//     target or weight it can run concurrently with A-CORR.
//   * ba_window_kernel: persistent, one workgroup per (lower 6x6 block (a, b)
//     of S, share `sub` of its patches).  Each workgroup keeps the patches
//     whose free-pose mask holds both a and b, re-linearises their edges each
//     iteration (fp32 edge math, fp64 products), reduces its block in a fixed
//     order (no atomics: deterministic) and publishes 42 doubles.  EVERY
//     workgroup then gathers all partial blocks (fixed order -> identical
//     bits everywhere), solves S dX = y itself (ba_solve.hpp, fp32 blocked
//     Cholesky + fp64 refinement) and applies the same pose retraction and
//     the depth update of its own patches.  One grid-wide exchange per
//     iteration; no solve -> broadcast hand-off.
//   * Grid <= 256 workgroups (one per CU, all co-resident); flags are
//     epoch-tagged (graph-replayable) and every spin-wait has a wall-clock
//     timeout (status bit 16) so the grid always drains.
#include <unistd.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <random>
#include <cstdlib>
#include <map>
#include <mutex>

#include "ba_solve.hpp"
#include "pyr_insert.hpp"

namespace dpvo {
namespace {
using namespace bad;

constexpr int kWT = 256;                // iteration kernel threads
constexpr int kPT = 512;                // plan kernel threads
constexpr int kWMaxN = 16;
constexpr int kWMaxE = 10240;           // DPVO MAX_EDGES = 10000 (config.py:42)
constexpr int kWMaxG = 256;
constexpr int kWLds = 160 * 1024;
constexpr int kHistMax = 12288;         // counting-sort range of kk
constexpr int kWSlots = 64;             // LDS pose table slots
constexpr unsigned kFix = 0xFF;         // pose code: fixed pose
constexpr unsigned kHbm = 0xFE;         // pose slot: read from HBM
constexpr int kChunk = 256;             // relevant edges per pass-1 chunk
constexpr int kPart = 42;               // doubles per published partial block
constexpr int kPartPad = 48;            // slot stride: 384 B = 3 whole 128-B lines per slot
constexpr int kGranPad = 48;            // granule slot stride: 768 B = 6 whole 128-B lines
constexpr long long kSpin = 2000000;    // 20 ms of the 100 MHz wall clock
constexpr int kEpochWord = kWMaxG;      // flags[kWMaxG]: epoch of the last call
constexpr int kFlagWords = kWMaxG + 8;
constexpr int kRefine = 1;              // fp64 refinement steps of the solve
// raw buffer resources (gfx950 dword 3) and the buffer builtins' cache-policy
// bit for sc1 (agent-coherent: bypasses the CU's L1; stores write through L2)
constexpr int kBufDword3 = 0x00020000;
constexpr int kSc1 = 16;

// status bits (shared with the other BA paths; see dpvo_hot.h)
constexpr int kStChol = 1, kStClamp = 2, kStTimeout = 16, kStCap = 32;

typedef unsigned v4u __attribute__((ext_vector_type(4)));

// plan meta (ints): [0] nuniq, [1] fmin, [2] status, [3] shards that wrote
// block-work partials; [16, 34) int64 phase stamps + 2 shader clocks; [kMetaWork + lblk(a, b)
// * kPlanShardMax + s] edges of the patches whose free poses hold a and b, from
// shard s (ba_window_kernel gives each lower block workgroups in proportion;
// a block's 16 shard counts are one 64-B run: four 16-B loads)
constexpr int kWMaxNB = kWMaxN * (kWMaxN + 1) / 2;
constexpr int kPlanShardMax = 16;
constexpr int kMetaWork = 64;
constexpr size_t kMetaBytes = sizeof(int) * (kMetaWork + (size_t)kPlanShardMax * kWMaxNB);

struct Plan {          // written by ba_plan_kernel, read by ba_window_kernel
  int* epos;           // [E] edge index at sorted position p (grouped by patch)
  int* poff;           // [E + 1] first position of patch u
  unsigned* pmask;     // [E] free-pose bitmask of patch u
  int* pkk;            // [E] patch id (kk) of patch u
  int* meta;           // [kMetaBytes / 4]: nuniq, fmin, status, shards, stamps, block work
  int* status;         // the workspace status word, reset here
  int* sink;           // caller's sticky status word or null
  const int* t0d;      // device t0 (graph-replayed updates: t0 moves per frame) or null
};

struct WArgs {
  float* poses;
  float* patches;
  const float* intrinsics;
  const float* target;
  const float* weight;
  const float* lmbda;
  const int64_t* ii;
  const int64_t* jj;
  const int64_t* kk;
  int E, P, num_poses, num_patches, t0, N, iters, NB, Sd, So, G;
  Plan plan;
  double* part;      // [2][G][kPartPad] (workspace layout only: the exchange uses gran)
  v4u* gran;         // [2][G][kGranPad] published partial blocks as 16-B granules, by iteration parity
  long long* flags;  // persistent [kFlagWords]
  float* ejg;        // [2][E][12] E entries by edge and iteration parity (fp32), HBM fallback
  int* status;       // [1] OR of status bits (workspace meta)
  int* sink;         // caller's sticky status word (dpvo_ba_set_status_sink) or null
  int64_t* marks;    // [2432] wall-clock stamps (instrumentation, dpvo_ba_set_marks): [0, 64)
                     // phases of workgroup 0, [128 + 256 it + g] / [640 + 256 it + g] per
                     // workgroup assembled / all partials seen, [1152 + g] setup done,
                     // [1408 + g] iteration 0 assembled (before the reduction); null on
                     // product calls
  double* dxo;       // [6N] dX of the latest iteration (workgroup 0; dpvo_ba_last_dx) or null
  const int* t0d;    // device t0 or null (then t0)
  unsigned long long salt;  // per-process random granule-key salt (see granule())
};

__device__ __forceinline__ size_t al16(size_t v) { return (v + 15) & ~(size_t)15; }
typedef double f64x2 __attribute__((ext_vector_type(2)));

// threadIdx.x through an empty asm: code inside the BA iteration loop that
// derives from it is not loop-invariant, so the compiler does not hoist it
// (addresses, masks of every phase) before the loop and keep it live across
// the loop in spilled registers (2.5 us of hoisted work at the loop entry).
__device__ __forceinline__ int opaque_tid() {
  int t = threadIdx.x;
  asm volatile("" : "+v"(t));
  return t;
}

__device__ __forceinline__ void mark(const WArgs& A, int slot) {
  if (A.marks && blockIdx.x == 0 && threadIdx.x == 0) A.marks[slot] = (int64_t)wall_clock64();
}


// ===========================================================================
// plan: group edges by patch (one workgroup, 512 threads)
// ===========================================================================
// per-edge capacity of a plan sized for E edges, and its LDS bytes
__host__ __device__ constexpr int plan_cap(int E) { return (E + 15) & ~15; }
// U: hd + mask (8 cap B) or the bitonic keys (u64 up to 8192 entries, u32 above)
__host__ __device__ constexpr size_t plan_u_bytes(int cap) {
  size_t p2 = 1;
  while (p2 < (size_t)cap) p2 <<= 1;
  const size_t keys = p2 <= 8192 ? 8 * p2 : 4 * p2;
  return keys > 8 * (size_t)cap ? keys : 8 * (size_t)cap;
}
__host__ __device__ constexpr size_t plan_lds_bytes(int cap) {
  return 256 + 6 * (size_t)cap + (((size_t)cap + 15) & ~(size_t)15) + plan_u_bytes(cap);
}
static_assert(plan_lds_bytes(kWMaxE) <= (size_t)kWLds, "plan LDS");

// rank of edge e among the members s[a, b) of its bucket (how many are smaller):
// 8 LDS reads in flight per step instead of one dependent read per member
__device__ __forceinline__ int bucket_rank(const unsigned short* s, int a, int b, int e) {
  int rank = 0;
  for (int t = a; t < b; t += 8) {
    int v[8];
#pragma unroll
    for (int k = 0; k < 8; k++) v[k] = s[min(t + k, b - 1)];
#pragma unroll
    for (int k = 0; k < 8; k++) rank += (t + k < b && v[k] < e) ? 1 : 0;
  }
  return rank;
}

constexpr int kPlanPer = kWMaxE / kPT;  // edges per plan thread: e = tid + r * kPT
// The plan's pass over the edge list: clamped kk of the thread's edges into
// kv (registers), pose codes into code[e] (LDS), and the block-wide kmin / kmax
// (ctl[0], ctl[1]), fmin (ctl[2], the smallest fixed pose) and status (ctl[3]).
// Loads in rounds of kPlanRound edges per thread, every load of a round issued
// before its first use (one global round trip per round, and only the rounds
// that hold edges); indices are clamped instead of guarded (a guarded load is
// a branch with its own wait).  Ends with a barrier.
template <int kPer = kPlanPer>
__device__ __forceinline__ void plan_edges_pass(const int64_t* __restrict__ ii,
                                                const int64_t* __restrict__ jj,
                                                const int64_t* __restrict__ kk, int E,
                                                int num_patches, int num_poses, int t0, int N,
                                                int* ctl, unsigned short* code, int (&kv)[kPer]) {
  const int tid = threadIdx.x, lane = tid & 63, T = kPT;
  const int kmaxc = num_patches - 1;
  if (tid == 0) {
    ctl[0] = 0x7fffffff;  // kmin
    ctl[1] = -1;          // kmax
    ctl[2] = 0x7fffffff;  // fmin
    ctl[3] = 0;           // status
  }
  __syncthreads();
  constexpr int kPlanRound = kPer % 5 == 0 ? 5 : kPer;
  static_assert(kPer % kPlanRound == 0, "load rounds");
  int kmin = 0x7fffffff, kmax = -1, fmin = 0x7fffffff, bad = 0;
#pragma unroll
  for (int r = 0; r < kPer; r++) kv[r] = 0;
  if (E > 0) {
#pragma unroll
    for (int r0 = 0; r0 < kPer; r0 += kPlanRound) {
      if (r0 * T >= E) break;  // block-uniform: only the rounds that hold edges (one at cfg2)
      int64_t vk[kPlanRound], vi[kPlanRound], vj[kPlanRound];
#pragma unroll
      for (int r = 0; r < kPlanRound; r++) {
        const int e = min(tid + (r0 + r) * T, E - 1);
        vk[r] = kk[e];
        vi[r] = ii[e];
        vj[r] = jj[e];
      }
#pragma unroll
      for (int r = 0; r < kPlanRound; r++) {
        const int e = tid + (r0 + r) * T;
        if (e >= E) continue;
        int64_t v = vk[r];
        if (v < 0 || v > kmaxc) {
          bad = 1;
          v = v < 0 ? 0 : kmaxc;
        }
        kmin = min(kmin, (int)v);
        kmax = max(kmax, (int)v);
        kv[r0 + r] = (int)v;
        const int64_t gi = vi[r], gj = vj[r];
        const bool fi = gi >= t0 && gi < t0 + N, fj = gj >= t0 && gj < t0 + N;
        const int ci = fi ? (int)(gi - t0) : (int)kFix, cj = fj ? (int)(gj - t0) : (int)kFix;
        if (!fi) fmin = min(fmin, (int)min(max(gi, (int64_t)0), (int64_t)num_poses - 1));
        if (!fj) fmin = min(fmin, (int)min(max(gj, (int64_t)0), (int64_t)num_poses - 1));
        code[e] = (unsigned short)((ci & 0xff) | ((cj & 0xff) << 8));
      }
    }
  }
  kmin = wave_min_i(kmin);
  kmax = wave_max_i(kmax);
  fmin = wave_min_i(fmin);
  bad = wave_max_i(bad);
  if (lane == 0) {
    atomicMin(&ctl[0], kmin);
    atomicMax(&ctl[1], kmax);
    atomicMin(&ctl[2], fmin);
    if (bad) atomicOr(&ctl[3], kStClamp);
  }
  __syncthreads();
}

// Block work of a set of patches (plan side): wl[lblk(a, b)] += edges of
// every patch whose free-pose mask holds a and b; patch(t) -> (count, mask)
// for t < n.  wl: kWMaxNB ints of LDS, zeroed by the caller before a barrier.
template <typename F>
__device__ __forceinline__ void plan_block_work(int n, F patch, int* wl) {
  for (int t = threadIdx.x; t < n; t += blockDim.x) {
    int c;
    unsigned m;
    patch(t, c, m);
    if (c <= 0) continue;
    for (unsigned ma = m; ma; ma &= ma - 1) {
      const int x = __builtin_ctz(ma);
      for (unsigned mb = m & ((2u << x) - 1u); mb; mb &= mb - 1)  // y <= x
        atomicAdd(&wl[lblk(x, __builtin_ctz(mb))], c);
    }
  }
}
__device__ __forceinline__ void plan_store_work(const Plan& plan, const int* wl, int s, int N) {
  const int nb = N * (N + 1) / 2;
  for (int t = threadIdx.x; t < nb; t += blockDim.x)
    plan.meta[kMetaWork + t * kPlanShardMax + s] = wl[t];
}

__device__ __forceinline__ void plan_block(const int64_t* __restrict__ ii,
                                           const int64_t* __restrict__ jj,
                                           const int64_t* __restrict__ kk, int E, int num_patches,
                                           int num_poses, int t0, int N, const Plan& plan,
                                           char* lds, int cap = kWMaxE) {
  if (plan.t0d) t0 = *plan.t0d;
  // LDS (plan_lds_bytes(cap), cap >= E; 153.9 KB at kWMaxE = 10240): per-edge
  // arrays as u16 / u8, one union
  //   [ctl 256 B | code u16[cap] | key u16[cap] -> ranked | spos u16[cap] | head u8[cap] | U]
  //   U (>= 16 cap B): counting sort hist int[R], later hd int[E] + mask u32[E];
  //      bitonic sort keys (u64 for E <= 8192, u32 (key << 14 | e) above)
  const int tid = threadIdx.x, T = kPT;
  const int kmaxc = num_patches - 1;
  int* ctl = (int*)lds;                  // [64]
  int* scr = ctl + 16;                   // scan scratch [>= 17]
  unsigned short* code = (unsigned short*)(lds + 256);           // ci | cj << 8 (5 bits each)
  unsigned short* key = code + cap;                              // kk - kmin, later ranked edges
  unsigned short* spos = key + cap;                              // edge at position p
  unsigned char* head = (unsigned char*)(spos + cap);            // head flags
  char* U = (char*)head + al16(cap);
  int kv[kPlanPer];  // clamped kk of this thread's edges e = tid + r * kPT (registers)
  plan_edges_pass(ii, jj, kk, E, num_patches, num_poses, t0, N, ctl, code, kv);
  int kmin = ctl[0];
  const int R = ctl[1] - kmin + 1;
  if (R <= kHistMax && (size_t)(R + E) * 4 <= plan_u_bytes(cap) && E < (1 << 14)) {
    // ---- counting sort in ONE scan (no second pass over positions) ----
    // hist[v] counts bucket v; one packed exclusive scan turns it into
    // (first position << 14 | patch index) -- buckets are patches in
    // ascending kk, so position and patch index of a bucket come from the
    // same prefix; the scatter then bumps the position part.  The free-pose
    // mask of each patch is an LDS OR over its edges.  Order inside a patch =
    // ascending edge index (a rank over the bucket's members), deterministic.
    int* hist = (int*)U;                                   // [R]
    unsigned* pm = reinterpret_cast<unsigned*>(hist + R);  // [E]
    for (int v = tid; v < R; v += T) hist[v] = 0;
    for (int u = tid; u < E; u += T) pm[u] = 0u;
    __syncthreads();
#pragma unroll
    for (int r = 0; r < kPlanPer; r++) {
      const int e = tid + r * T;
      if (e < E) atomicAdd(&hist[kv[r] - kmin], 1);
    }
    __syncthreads();
    const int nuniq = fscan(hist, R, scr, 14) & 0x3fff;  // hist[v] = start << 14 | patch
#pragma unroll
    for (int r = 0; r < kPlanPer; r++) {
      const int e = tid + r * T;
      if (e >= E) continue;
      const int old = atomicAdd(&hist[kv[r] - kmin], 1 << 14);
      spos[old >> 14] = (unsigned short)e;
      const unsigned c = code[e], ci = c & 0xff, cj = c >> 8;
      const unsigned m = (ci != kFix ? 1u << ci : 0u) | (cj != kFix ? 1u << cj : 0u);
      if (m) atomicOr(&pm[old & 0x3fff], m);
    }
    __syncthreads();
    // hist[v] >> 14 is now the END of bucket v (= the start of bucket v + 1);
    // the patch index bits are unchanged
#pragma unroll
    for (int r = 0; r < kPlanPer; r++) {
      const int e = tid + r * T;
      if (e >= E) continue;
      const int v = kv[r] - kmin, hv = hist[v];
      const int b = hv >> 14, a = (v == 0) ? 0 : (hist[v - 1] >> 14);
      const int rank = bucket_rank(spos, a, b, e);
      plan.epos[a + rank] = e;
      if (rank == 0) {
        const int u = hv & 0x3fff;
        plan.poff[u] = a;
        plan.pkk[u] = kv[r];
        plan.pmask[u] = pm[u];
      }
    }
    if (tid == 0) {
      plan.poff[nuniq] = E;
      plan.meta[0] = nuniq;
      plan.meta[1] = ctl[2];
      plan.meta[2] = ctl[3];
      plan.meta[3] = 0;  // no block-work partials: the iteration kernel splits blocks evenly
      if (ctl[3] && plan.sink) atomicOr(plan.sink, ctl[3]);
      *plan.status = 0;  // this call's status word (ORed by the iteration kernel)
    }
    return;
  }
  unsigned short* pos_edge = spos;  // the sorted order, wherever it ends up
  if (R <= kHistMax && (size_t)R * 4 <= plan_u_bytes(cap)) {
    int* hist = (int*)U;  // [R]
    for (int v = tid; v < R; v += T) hist[v] = 0;
    for (int p = tid; p < E; p += T) head[p] = 0;
    __syncthreads();
#pragma unroll
    for (int r = 0; r < kPlanPer; r++) {
      const int e = tid + r * T;
      if (e < E) atomicAdd(&hist[kv[r] - kmin], 1);
    }
    __syncthreads();
    fscan(hist, R, scr);  // hist[v] = first position of bucket v
    for (int v = tid; v < R; v += T) {
      const int a = hist[v], b = (v + 1 < R) ? hist[v + 1] : E;
      if (b > a) head[a] = 1;
    }
    // every bucket start must be read before any wave bumps it below (without
    // this barrier a fast wave's scatter moved a slow wave's head flag into the
    // middle of a bucket: patches split or merged, a wrong Schur complement)
    __syncthreads();
#pragma unroll
    for (int r = 0; r < kPlanPer; r++) {
      const int e = tid + r * T;
      if (e < E) spos[atomicAdd(&hist[kv[r] - kmin], 1)] = (unsigned short)e;
    }
    __syncthreads();
    // deterministic order inside a patch (ascending edge index): every edge
    // counts the smaller edges of its bucket, all edges in parallel; the
    // ranked order overwrites the keys (no longer read) after a barrier
    int dst[kPlanPer];
#pragma unroll
    for (int r = 0; r < kPlanPer; r++) {
      const int e = tid + r * T;
      dst[r] = -1;
      if (e >= E) continue;
      const int v = kv[r] - kmin;
      const int b = hist[v], a = (v == 0) ? 0 : hist[v - 1];  // hist[v]: end of bucket v now
      dst[r] = a + bucket_rank(spos, a, b, e);
    }
    __syncthreads();
#pragma unroll
    for (int r = 0; r < kPlanPer; r++)
      if (dst[r] >= 0) key[dst[r]] = (unsigned short)(tid + r * T);
    pos_edge = key;
  } else {
    // wide kk range: bitonic sort over the next power of two of (key, e):
    // u64 (key << 32 | e) up to E = 8192, else u32 (key << 14 | e), which
    // needs R <= 2^18 (status 32 otherwise: the call raises)
    int P2 = 1;
    while (P2 < E) P2 <<= 1;
    const bool wide = P2 <= 8192;
    if (!wide && R > (1 << 18)) {
      if (tid == 0) ctl[3] |= kStCap;
    }
    unsigned long long* k64 = (unsigned long long*)U;
    unsigned* k32 = (unsigned*)U;
#pragma unroll
    for (int r = 0; r < kPlanPer; r++) {
      const int e = tid + r * T;
      if (e < E) {
        if (wide)
          k64[e] = ((unsigned long long)(unsigned)(kv[r] - kmin) << 32) | (unsigned)e;
        else
          k32[e] = ((unsigned)min(kv[r] - kmin, (1 << 18) - 1) << 14) | (unsigned)e;
      }
    }
    for (int i = E + tid; i < P2; i += T) {
      if (wide)
        k64[i] = ~0ull;
      else
        k32[i] = ~0u;
    }
    __syncthreads();
    for (int size = 2; size <= P2; size <<= 1)
      for (int stride = size >> 1; stride > 0; stride >>= 1) {
        for (int i = tid; i < P2 / 2; i += T) {
          const int lo = 2 * i - (i & (stride - 1));
          const int hi = lo + stride;
          const bool up = ((lo & size) == 0);
          if (wide) {
            const unsigned long long a = k64[lo], b = k64[hi];
            if ((a > b) == up) {
              k64[lo] = b;
              k64[hi] = a;
            }
          } else {
            const unsigned a = k32[lo], b = k32[hi];
            if ((a > b) == up) {
              k32[lo] = b;
              k32[hi] = a;
            }
          }
        }
        __syncthreads();
      }
    for (int p = tid; p < E; p += T) {
      if (wide) {
        spos[p] = (unsigned short)(k64[p] & 0xffffffffull);
        head[p] = (p == 0 || (k64[p] >> 32) != (k64[p - 1] >> 32)) ? 1 : 0;
      } else {
        spos[p] = (unsigned short)(k32[p] & 0x3fffu);
        head[p] = (p == 0 || (k32[p] >> 14) != (k32[p - 1] >> 14)) ? 1 : 0;
      }
    }
  }
  __syncthreads();
  // patch index of every position: exclusive scan of the heads (U is free now)
  int* hd = (int*)U;
  for (int p = tid; p < E; p += T) hd[p] = head[p];
  __syncthreads();
  const int nuniq = fscan(hd, E, scr);   // hd[p] = heads strictly before p
  // patch u starts at the p with hd[p] == u and a head: recompute heads
  for (int p = tid; p < E; p += T) {
    const int u1 = (p + 1 < E) ? hd[p + 1] : nuniq;  // heads up to and including p
    const bool is_head = u1 != hd[p];
    const int u = u1 - 1;                            // patch of position p
    const int e = pos_edge[p];
    plan.epos[p] = e;
    if (is_head) {
      plan.poff[u] = p;
      plan.pkk[u] = (int)min(max(kk[e], (int64_t)0), (int64_t)kmaxc);
    }
  }
  if (tid == 0) plan.poff[nuniq] = E;
  // free-pose masks: OR over the patch's edges (positions are contiguous)
  unsigned* mask = (unsigned*)(U + sizeof(int) * cap);  // [nuniq]
  for (int u = tid; u < nuniq; u += T) mask[u] = 0u;
  __syncthreads();
  for (int p = tid; p < E; p += T) {
    const int u = ((p + 1 < E) ? hd[p + 1] : nuniq) - 1;
    const unsigned c = code[pos_edge[p]];
    const unsigned ci = c & 0xff, cj = c >> 8;
    const unsigned m = (ci != kFix ? 1u << ci : 0u) | (cj != kFix ? 1u << cj : 0u);
    if (m) atomicOr(&mask[u], m);
  }
  __syncthreads();
  for (int u = tid; u < nuniq; u += T) plan.pmask[u] = mask[u];
  if (tid == 0) {
    plan.meta[0] = nuniq;
    plan.meta[1] = ctl[2];
    plan.meta[2] = ctl[3];
    plan.meta[3] = 0;
    if (ctl[3] && plan.sink) atomicOr(plan.sink, ctl[3]);
    *plan.status = 0;  // this call's status word (ORed by the iteration kernel)
  }
}

// ---- the plan over S workgroups (shard s of S) ----
// Every shard makes the pass over the whole edge list (kk / ii / jj of 10k
// edges = 240 KB, L2-resident after the first shard), so kmin / kmax / fmin /
// status and the presence bitmap of patch ids are known everywhere; shard s
// then groups only the edges of ITS bucket range [lo, hi) of kk - kmin:
//   positions  = edges with a smaller kk (counted in the pass) + the local
//                counting sort,
//   patch ids  = present kk values below lo (bitmap popcount) + local index.
// The shards write disjoint ranges of epos / poff / pkk / pmask: no exchange
// between workgroups.  Falls back to plan_block in shard 0 when the kk range
// or the LDS does not fit.
__host__ __device__ constexpr int plan_shards(int E) {
  return E <= 512 ? 1 : ((E + 511) / 512 < kPlanShardMax ? (E + 511) / 512 : kPlanShardMax);
}
template <int kPer>
__device__ __forceinline__ void plan_sharded_k(const int64_t* __restrict__ ii,
                                             const int64_t* __restrict__ jj,
                                               const int64_t* __restrict__ kk, int E, int num_patches,
                                               int num_poses, int t0, int N, const Plan& plan,
                                               char* lds, int cap, size_t lds_bytes, int s, int S) {
  if (S <= 1) {
    if (s == 0) plan_block(ii, jj, kk, E, num_patches, num_poses, t0, N, plan, lds, cap);
    return;
  }
  if (plan.t0d) t0 = *plan.t0d;
  // phase stamps of shard 0 (100 MHz wall clock, 7 stores per launch):
  // meta + 16 as int64 [7], then the shader clock at stamps 0 and 6
  // (scripts/plan_phases.py)
  auto stamp = [&](int q) {
    if (s == 0 && threadIdx.x == 0) {
      reinterpret_cast<int64_t*>(plan.meta + 16)[q] = (int64_t)wall_clock64();
      // shader clock at the first and last stamp: the effective frequency
      if (q == 0 || q == 6) reinterpret_cast<int64_t*>(plan.meta + 16)[7 + (q == 6)] = (int64_t)clock64();
    }
  };
  stamp(0);
  //   [ctl 256 B | code u16[cap] | spos u16[cap] | hf int[R] | pm u32[nl]]
  const int tid = threadIdx.x, lane = tid & 63, T = kPT;
  int* ctl = (int*)lds;  // [0..3] as plan_edges_pass, [4] below, [5] ubelow, [6] nuniq
  int* scr = ctl + 16;
  unsigned short* code = (unsigned short*)(lds + 256);
  unsigned short* spos = code + cap;
  int* hf = reinterpret_cast<int*>(spos + cap);  // histogram of kk - kmin over the FULL range
  int kv[kPer];
  plan_edges_pass<kPer>(ii, jj, kk, E, num_patches, num_poses, t0, N, ctl, code, kv);
  stamp(1);
  const int kmin = ctl[0], R = ctl[1] - kmin + 1;
  const int nlmax = (R + S - 1) / S;
  const bool fits = E > 0 && R <= kHistMax && E < (1 << 14) &&
                    256 + 4 * (size_t)cap + 4 * (size_t)R + 4 * (size_t)nlmax + 4 * kWMaxNB <= lds_bytes;
  if (!fits) {  // shard-uniform (every shard saw the same edges)
    if (s == 0) {
      __syncthreads();  // ctl is re-initialised by plan_block
      plan_block(ii, jj, kk, E, num_patches, num_poses, t0, N, plan, lds, cap);
    }
    return;
  }
  const int lo = (int)((long long)R * s / S), hi = (int)((long long)R * (s + 1) / S), nl = hi - lo;
  unsigned* pm = reinterpret_cast<unsigned*>(hf + R);
  int* wl = reinterpret_cast<int*>(pm + nl);  // [kWMaxNB] block work of this shard's patches
  for (int v = tid; v < R; v += T) hf[v] = 0;
  for (int v = tid; v < nl; v += T) pm[v] = 0u;
  for (int v = tid; v < kWMaxNB; v += T) wl[v] = 0;
  if (tid == 0) {
    ctl[4] = 0;
    ctl[5] = 0;
    ctl[6] = 0;
  }
  __syncthreads();
  // one histogram of the whole kk range: its nonzero buckets below lo number
  // the patches before this shard's, and its [lo, hi) slice is the local
  // counting sort's input (a patch's ~4-10 edges share a bucket; a presence
  // bitmap word took 32 patches' worth of atomics)
  int nb = 0;
#pragma unroll
  for (int r = 0; r < kPer; r++) {
    const int e = tid + r * T;
    if (e >= E) continue;
    const int v = kv[r] - kmin;
    atomicAdd(&hf[v], 1);
    nb += v < lo ? 1 : 0;
  }
  __syncthreads();  // histogram complete
  stamp(2);
  int ub = 0, nu = 0;
  for (int v = tid; v < R; v += T) {
    const int present = hf[v] > 0 ? 1 : 0;
    nu += present;
    ub += v < lo ? present : 0;
  }
  nb = wave_sum_i(nb);
  ub = wave_sum_i(ub);
  nu = wave_sum_i(nu);
  if (lane == 0) {
    atomicAdd(&ctl[4], nb);
    atomicAdd(&ctl[5], ub);
    atomicAdd(&ctl[6], nu);
  }
  int* hist = hf + lo;  // this shard's buckets
  // local counting sort in one packed scan (plan_block's fast path); the
  // scan's barriers also complete the ctl sums above
  fscan(hist, nl, scr, 14);
  stamp(3);
  const int below = ctl[4], ubelow = ctl[5], nuniq = ctl[6];
#pragma unroll
  for (int r = 0; r < kPer; r++) {
    const int e = tid + r * T;
    const int v = kv[r] - kmin - lo;
    if (e >= E || v < 0 || v >= nl) continue;
    const int old = atomicAdd(&hist[v], 1 << 14);
    spos[old >> 14] = (unsigned short)e;
    const unsigned c = code[e], ci = c & 0xff, cj = c >> 8;
    const unsigned m = (ci != kFix ? 1u << ci : 0u) | (cj != kFix ? 1u << cj : 0u);
    if (m) atomicOr(&pm[old & 0x3fff], m);
  }
  __syncthreads();
  stamp(4);
  // block work of the local patches (bucket v: edges end(v) - end(v - 1))
  plan_block_work(nl, [&](int v, int& c, unsigned& m) {
    const int hv = hist[v];
    c = (hv >> 14) - (v == 0 ? 0 : (hist[v - 1] >> 14));
    m = pm[hv & 0x3fff];
  }, wl);
  stamp(5);
#pragma unroll
  for (int r = 0; r < kPer; r++) {
    const int e = tid + r * T;
    const int v = kv[r] - kmin - lo;
    if (e >= E || v < 0 || v >= nl) continue;
    const int hv = hist[v];
    const int b = hv >> 14, a = (v == 0) ? 0 : (hist[v - 1] >> 14);
    const int rank = bucket_rank(spos, a, b, e);
    plan.epos[below + a + rank] = e;
    if (rank == 0) {
      const int u = ubelow + (hv & 0x3fff);
      plan.poff[u] = below + a;
      plan.pkk[u] = kv[r];
      plan.pmask[u] = pm[hv & 0x3fff];
    }
  }
  __syncthreads();  // block work complete (the rank loop above does not touch wl)
  plan_store_work(plan, wl, s, N);
  if (tid == 0 && s == S - 1) plan.poff[nuniq] = E;
  if (tid == 0 && s == 0) {
    plan.meta[0] = nuniq;
    plan.meta[1] = ctl[2];
    plan.meta[2] = ctl[3];
    plan.meta[3] = S;
    if (ctl[3] && plan.sink) atomicOr(plan.sink, ctl[3]);
    *plan.status = 0;
  }
  stamp(6);
}

// The executed code of the plan is what a cold instruction cache pays for
// (the launch follows A-CORR and the BA window, which evict it): graphs of up
// to 4 edges per thread (E <= 2048, cfg2) run a copy unrolled 4 deep instead
// of kPlanPer = 20.
__device__ __forceinline__ void plan_sharded(const int64_t* __restrict__ ii,
                                             const int64_t* __restrict__ jj,
                                             const int64_t* __restrict__ kk, int E, int num_patches,
                                             int num_poses, int t0, int N, const Plan& plan,
                                             char* lds, int cap, size_t lds_bytes, int s, int S) {
  if (E <= 4 * kPT)
    plan_sharded_k<4>(ii, jj, kk, E, num_patches, num_poses, t0, N, plan, lds, cap, lds_bytes, s, S);
  else
    plan_sharded_k<kPlanPer>(ii, jj, kk, E, num_patches, num_poses, t0, N, plan, lds, cap,
                             lds_bytes, s, S);
}

__global__ void __launch_bounds__(kPT) ba_plan_kernel(const int64_t* __restrict__ ii,
                                                      const int64_t* __restrict__ jj,
                                                      const int64_t* __restrict__ kk, int E,
                                                      int num_patches, int num_poses, int t0, int N,
                                                      Plan plan) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  plan_sharded(ii, jj, kk, E, num_patches, num_poses, t0, N, plan, lds, kWMaxE, kWLds, blockIdx.x,
               gridDim.x);
}

// One launch for the start of a DPVO update (dpvo.py:775-824): F-REPROJ of
// every (edge, pixel), the A-CORR edge order and the BA plan.  The plan only
// reads ii / jj / kk, which the update does not change before its BA, so its
// single workgroup (the longest, dispatched first as workgroup 0) runs beside
// the reprojection instead of after A-CORR.
struct RArgs {
  const float* poses;
  const float* patches;
  const float* intrinsics;
  const int64_t* ii;
  const int64_t* jj;
  const int64_t* kk;
  int E, P, num_poses, num_patches, N2, t0, N;
  float* coords;
  int* order;
  int nps;  // plan shards: workgroups [0, nps) plan, nps the edge order, then the reprojection
  int64_t* marks;  // instrumentation (dpvo_ba_set_marks): [2b] / [2b + 1] start / end of workgroup b < 256
};

__global__ void __launch_bounds__(kPT) reproject_plan_kernel(RArgs R, Plan plan) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  if ((int)blockIdx.x < R.nps) {
    plan_sharded(R.ii, R.jj, R.kk, R.E, R.num_patches, R.num_poses, R.t0, R.N, plan, lds, kWMaxE,
                 kWLds, blockIdx.x, R.nps);
    return;
  }
  if ((int)blockIdx.x == R.nps) {
    const OrderIn q{R.poses, R.patches, R.intrinsics, R.ii, R.kk, R.P, R.num_poses, R.num_patches};
    edge_order_block(q, R.jj, R.E, R.N2, R.order, reinterpret_cast<int*>(lds));
    return;
  }
  const int PP = R.P * R.P;
  const int t = (blockIdx.x - R.nps - 1) * kPT + threadIdx.x;
  if (t >= R.E * PP) return;
  reproject_pixel(R.poses, R.patches, R.intrinsics, R.ii, R.jj, R.kk, t / PP, t % PP, R.P,
                  R.num_poses, R.num_patches, R.coords);
}

// The same launch with the insertion of the update's new frame into the
// channels-last pyramid ring (dpvo.py __call__, before update()): its tiles
// (two 256-thread tiles per workgroup) run on the CUs the reprojection and the
// single-workgroup plan leave idle, instead of as their own launch before.
// The insertion writes pyramid slots only, which nothing else in the launch
// reads; outputs are bit-identical to the two separate launches.
struct InsArgs {
  const void* src;
  InsLevels lv;
  int L, C, H, W, gx, gy, ntile;
};

template <typename T>
__device__ __forceinline__ void reproject_plan_insert_body(const RArgs& R, const Plan& plan,
                                                           const InsArgs& I, int nrep, char* lds) {
  const int b = blockIdx.x, b0 = R.nps + 1;  // first reprojection workgroup
  // the plan shards and the edge order are the launch's long chains; the
  // insertion tiles share their CUs: their waves issue first
  if (b <= R.nps) __builtin_amdgcn_s_setprio(3);
  if (b < R.nps) {
    plan_sharded(R.ii, R.jj, R.kk, R.E, R.num_patches, R.num_poses, R.t0, R.N, plan, lds,
                 plan_cap(R.E), plan_lds_bytes(plan_cap(R.E)), b, R.nps);
    return;
  }
  if (b == R.nps) {
    const OrderIn q{R.poses, R.patches, R.intrinsics, R.ii, R.kk, R.P, R.num_poses, R.num_patches};
    edge_order_block(q, R.jj, R.E, R.N2, R.order, reinterpret_cast<int*>(lds));
    return;
  }
  if (b < b0 + nrep) {
    const int PP = R.P * R.P;
    const int t = (b - b0) * kPT + threadIdx.x;
    if (t >= R.E * PP) return;
    reproject_pixel(R.poses, R.patches, R.intrinsics, R.ii, R.jj, R.kk, t / PP, t % PP, R.P,
                    R.num_poses, R.num_patches, R.coords);
    return;
  }
  static_assert(kPT == 512, "two 256-thread insertion tiles per workgroup");
  const int half = threadIdx.x >> 8, t = 2 * (b - b0 - nrep) + half;
  const bool act = t < I.ntile;
  const int tt = act ? t : 0;
  float* tile = reinterpret_cast<float*>(lds) + half * kInsTC * kInsCS;
  ins_tile<T>(static_cast<const T*>(I.src), I.lv, I.L, I.C, I.H, I.W, tt % I.gx,
              (tt / I.gx) % I.gy, tt / (I.gx * I.gy), threadIdx.x & 255, act, tile);
}

template <typename T>
__global__ void __launch_bounds__(kPT) reproject_plan_insert_kernel(RArgs R, Plan plan, InsArgs I,
                                                                    int nrep) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  const bool mk = R.marks && blockIdx.x < 256;
  if (mk && threadIdx.x == 0) R.marks[2 * blockIdx.x] = (int64_t)wall_clock64();
  reproject_plan_insert_body<T>(R, plan, I, nrep, lds);
  if (mk) {
    __syncthreads();
    if (threadIdx.x == 0) R.marks[2 * blockIdx.x + 1] = (int64_t)wall_clock64();
  }
}

// ===========================================================================
// iteration kernel
// ===========================================================================
struct WL {  // LDS layout of one workgroup
  int* ctl;            // [64]
  float* pose;         // [kWSlots][8]
  double* dX;          // [6N]
  unsigned short* tri;  // [NB] block (a, b) of lower-block index (a << 8 | b)
  // relevant patches
  int* roff;           // [nrel + 1] first relevant edge
  float2* nxy;         // [nrel] normalised centre
  float* dep;          // [nrel] inverse depth (current)
  float* dbase;        // [nrel] [2][0][0] of the input (first retraction base)
  double2* qu;         // [nrel] Q, u of the last linearisation
  int* pkx;            // [nrel] patch id, -1 if this workgroup does not write it
  // relevant edges
  unsigned short* ec;  // [nrp] pose slot of ii | slot of jj << 8
  unsigned short* rp;  // [nrp] relevant patch of the edge
  int* eid;            // [nrp] edge index
  float4* tw;          // [nrp] target, weight (LDS), or null: read by edge from the inputs
  float* ej;           // [nrp][12] E entries of the last linearisation (LDS), or null
  char* region;        // union: chunk scratch / reduction table / solver
  // E entries of relevant edge q for iteration parity par: in LDS by q, else in
  // the shared HBM buffer by edge id and parity (write-through sc1 stores and
  // sc1 loads there: see assemble).  Every workgroup holding an
  // edge writes the same bits there (identical poses, depths and order), and
  // parity keeps a workgroup one iteration ahead off the slot a slower one
  // still reads (it can reach iteration it + 2 only after every workgroup
  // has published it + 1, i.e. finished reading iteration it's entries)
  __device__ __forceinline__ void ld_ej(const float* ejg, int E, int q, int par, float4& e0,
                                        float4& e1, float4& e2) const {
    if (ej) {
      const float4* e4 = reinterpret_cast<const float4*>(ej + 12 * (size_t)q);
      e0 = e4[0];
      e1 = e4[1];
      e2 = e4[2];
    } else {  // written sc1 (write-through) by other threads: read past the CU's L1
      const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
          const_cast<float*>(ejg), 0, (int)(sizeof(float) * 24 * (size_t)E), kBufDword3);
      const int o = (int)(sizeof(float) * 12 * ((size_t)par * E + eid[q]));
      e0 = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rs, o, 0, kSc1));
      e1 = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rs, o + 16, 0, kSc1));
      e2 = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rs, o + 32, 0, kSc1));
    }
  }
};

enum { cNrel = 0, cNrp = 1, cFmin = 2, cFail = 3, cTimeout = 4, cCap = 5, cFailAny = 6, cLMulti = 7,
       cScan = 16 };

// E^T dX over relevant edges [q0, q1) (ba_cuda.cu:563), in order (patch_etdx:
// all edges of relevant patch ri).  The E
// entries of kEb edges (HBM sc1 loads on the fallback path) and the dX rows
// they pair with are all read before the first is used, with clamped indices
// and selects instead of guarded reads: one round trip per kEb edges, not one
// per edge (the per-edge loop made the final apply at E = 9850 a chain of
// dependent HBM loads, 12.6 us).  Adding +0.0 for an absent term leaves ex
// unchanged, so the sum is the one of the per-edge loop.
__device__ __forceinline__ double edges_etdx(const WL& L, const WArgs& A, int q0, int q1, int par,
                                             int N) {
  constexpr int kEb = 4;
  double ex = 0.0;
  for (int qb = q0; qb < q1; qb += kEb) {
    float4 e[kEb][3];
    unsigned cc[kEb];
#pragma unroll
    for (int u = 0; u < kEb; u++) {
      const int q = min(qb + u, q1 - 1);
      cc[u] = L.ec[q];
      L.ld_ej(A.ejg, A.E, q, par, e[u][0], e[u][1], e[u][2]);
    }
#pragma unroll
    for (int u = 0; u < kEb; u++) {
      const bool live = qb + u < q1;
      const unsigned si = cc[u] & 0xff, sj = cc[u] >> 8;
      const unsigned nm = (unsigned)max(N - 1, 0);
      const double* dj = L.dX + 6 * min(sj, nm);
      const double* di = L.dX + 6 * min(si, nm);
      const float4 e0 = e[u][0], e1 = e[u][1], e2 = e[u][2];
      const double tj = (double)e0.x * dj[0] + (double)e0.y * dj[1] + (double)e0.z * dj[2] +
                        (double)e0.w * dj[3] + (double)e1.x * dj[4] + (double)e1.y * dj[5];
      const double ti = (double)e1.z * di[0] + (double)e1.w * di[1] + (double)e2.x * di[2] +
                        (double)e2.y * di[3] + (double)e2.z * di[4] + (double)e2.w * di[5];
      ex += (live && sj < (unsigned)N) ? tj : 0.0;
      ex += (live && si < (unsigned)N) ? ti : 0.0;
    }
  }
  return ex;
}
__device__ __forceinline__ double patch_etdx(const WL& L, const WArgs& A, int ri, int par, int N) {
  return edges_etdx(L, A, L.roff[ri], L.roff[ri + 1], par, N);
}

__device__ __forceinline__ unsigned wslot(int gp, int t0, int N, int fmin) {
  if (gp >= t0 && gp < t0 + N) return (unsigned)(gp - t0);
  const int k = gp - fmin;
  return (k >= 0 && k < kWSlots - N) ? (unsigned)(N + k) : kHbm;
}

__device__ __forceinline__ void pose_of(const WArgs& A, const WL& L, unsigned slot, int gp,
                                        float* P) {
  if (slot != kHbm) {
    const float4 a0 = *reinterpret_cast<const float4*>(L.pose + 8 * slot);
    const float4 a1 = *reinterpret_cast<const float4*>(L.pose + 8 * slot + 4);
    P[0] = a0.x; P[1] = a0.y; P[2] = a0.z; P[3] = a0.w; P[4] = a1.x; P[5] = a1.y; P[6] = a1.z;
  } else {
    const float* g = A.poses + 7 * (size_t)gp;
#pragma unroll
    for (int k = 0; k < 7; k++) P[k] = g[k];
  }
}

// nact (out): the threads [0, nact) are the only ones whose acc can be
// nonzero (thread t takes edge q0 + t of a chunk and patch pa + t)
template <int MODE>  // 0: only Q, u (no free pose / N == 0); 1 diagonal block; 2 off-diagonal
__device__ void assemble(const WArgs& A, const WL& L, int nrel, int a, int b, double lam,
                         float fx, float fy, float cx, float cy, int par, double* acc,
                         int& nact) {
  nact = 0;
  constexpr int NA = (MODE == 1) ? 27 : (MODE == 2 ? 36 : 1);
  const int tid = opaque_tid(), N = A.N;
  const unsigned ua = (unsigned)a, ub = (unsigned)b;
  double* pe = reinterpret_cast<double*>(L.region);  // [kChunk][14]: c, u, Ea[6], Eb[6]
#pragma unroll
  for (int k = 0; k < NA; k++) acc[k] = 0.0;
  for (int pa = 0; pa < nrel;) {
    // chunk: whole patches [pa, pb) with at most kChunk edges (one patch may exceed: own chunk)
    int pb = pa + 1;
    {
      int lo = pa + 1, hi = nrel;  // largest pb with roff[pb] - roff[pa] <= kChunk
      const int base = L.roff[pa];
      if (L.roff[nrel] - base <= kChunk) {
        lo = nrel;  // the rest fits (cfg2: every edge in one chunk): no search
      } else {
        while (lo < hi) {
          const int mid = (lo + hi + 1) >> 1;
          if (L.roff[mid] - base <= kChunk) lo = mid; else hi = mid - 1;
        }
      }
      pb = lo;
    }
    const int q0 = L.roff[pa], q1 = L.roff[pb];
    nact = max(nact, min(max(q1 - q0, pb - pa), kWT));
    // pass 1: thread per edge
    for (int q = q0 + tid; q < q1; q += kWT) {
      const unsigned c = L.ec[q];
      const unsigned si = c & 0xff, sj = c >> 8;
      const int e = L.eid[q];
      float Pi[7], Pj[7];
      pose_of(A, L, si, si == kHbm ? (int)A.ii[e] : 0, Pi);
      pose_of(A, L, sj, sj == kHbm ? (int)A.jj[e] : 0, Pj);
      const int ri = L.rp[q];
      float4 tw;
      if (L.tw) {
        tw = L.tw[q];
      } else {
        const float2 tg = reinterpret_cast<const float2*>(A.target)[e];
        const float2 wt = reinterpret_cast<const float2*>(A.weight)[e];
        tw = make_float4(tg.x, tg.y, wt.x, wt.y);
      }
      Lin o;
      lin_edge(Pi, Pj, L.nxy[ri].x, L.nxy[ri].y, L.dep[ri], tw.x, tw.y, tw.z, tw.w, fx, fy, cx,
               cy, o);
      const unsigned ci = si < (unsigned)N ? si : kFix, cj = sj < (unsigned)N ? sj : kFix;
      double cq = 0.0, uq = 0.0, ejv[6] = {0, 0, 0, 0, 0, 0}, eiv[6] = {0, 0, 0, 0, 0, 0};
#pragma unroll
      for (int row = 0; row < 2; row++) {
        const double wr = o.w[row];
        const double wz = wr * (double)o.Jz[row];
#pragma unroll
        for (int k = 0; k < 6; k++) {
          ejv[k] += wz * (double)o.Jj[row][k];
          eiv[k] -= wz * (double)o.Ji[row][k];
        }
        cq += wz * (double)o.Jz[row];
        uq += (wr * (double)o.r[row]) * (double)o.Jz[row];
      }
      // E entries (fp32) for the depth update after the solve
      {
        const float4 e0 = make_float4((float)ejv[0], (float)ejv[1], (float)ejv[2], (float)ejv[3]);
        const float4 e1 = make_float4((float)ejv[4], (float)ejv[5], (float)eiv[0], (float)eiv[1]);
        const float4 e2 = make_float4((float)eiv[2], (float)eiv[3], (float)eiv[4], (float)eiv[5]);
        if (L.ej) {
          float4* eo = reinterpret_cast<float4*>(L.ej + 12 * (size_t)q);
          eo[0] = e0;
          eo[1] = e1;
          eo[2] = e2;
        } else {
          // shared HBM buffer: every workgroup holding the edge writes the same
          // bits; write-through (sc1) stores leave no dirty line in any XCD's
          // L2, so no stale copy of an earlier same-parity iteration can be
          // written back over a newer one (the L2s are not coherent)
          const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
              A.ejg, 0, (int)(sizeof(float) * 24 * (size_t)A.E), kBufDword3);
          const int o = (int)(sizeof(float) * 12 * ((size_t)par * A.E + L.eid[q]));
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4u, e0), rs, o, 0, kSc1);
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4u, e1), rs, o + 16, 0, kSc1);
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4u, e2), rs, o + 32, 0, kSc1);
        }
      }
      double* ps = pe + 14 * (size_t)(q - q0);
      ps[0] = cq;
      ps[1] = uq;
      if (MODE != 0) {
#pragma unroll
        for (int k = 0; k < 6; k++) {
          ps[2 + k] = ((cj == ua) ? ejv[k] : 0.0) + ((ci == ua) ? eiv[k] : 0.0);
          ps[8 + k] = ((cj == ub) ? ejv[k] : 0.0) + ((ci == ub) ? eiv[k] : 0.0);
        }
        // B terms of this block (ba_cuda.cu:339-350), v (:352-370)
        const bool ia = ci == ua, ja = cj == ua, ib = ci == ub, jb = cj == ub;
        const bool hit = (MODE == 1) ? (ia || ja) : ((ia && jb) || (ja && ib));
        if (hit) {
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
      }
    }
    __syncthreads();
    // pass 2a: thread per (patch, component): C, u, E at a / b summed over the
    // patch's edges in edge order, 4 edges' reads in flight (a thread per
    // patch walked ~18 edges one LDS round trip at a time at DPVO sizes,
    // on one partly filled wave); absent terms add +0.0: the sums are the
    // per-patch loop's
    constexpr int NC = (MODE == 2) ? 14 : (MODE == 1 ? 8 : 2);
    // (only for patches with many edges: at ~2 edges per patch, cfg2, the
    // per-patch loop below reads them directly and saves the barrier)
    const bool wide = (q1 - q0) >= 4 * (pb - pa);
    double* psum = pe + 14 * (size_t)kChunk;  // [patch of the chunk][14]
    for (int t = tid; wide && t < (pb - pa) * NC; t += kWT) {
      const int rr = t / NC, c = t - rr * NC;
      const int qa = L.roff[pa + rr], qz = L.roff[pa + rr + 1];
      double sum = 0.0;
      for (int qb = qa; qb < qz; qb += 4) {
        double v[4];
#pragma unroll
        for (int u = 0; u < 4; u++) v[u] = pe[14 * (size_t)(min(qb + u, qz - 1) - q0) + c];
#pragma unroll
        for (int u = 0; u < 4; u++) sum += (qb + u < qz) ? v[u] : 0.0;
      }
      psum[14 * rr + c] = sum;
    }
    if (wide) __syncthreads();
    // pass 2b: thread per patch: Q and the Schur terms (:554-558)
    for (int ri = pa + tid; ri < pb; ri += kWT) {
      double C, U, Ea[6], Eb[6];
      if (wide) {
        const double* ps = psum + 14 * (size_t)(ri - pa);
        C = ps[0];
        U = ps[1];
#pragma unroll
        for (int k = 0; k < 6; k++) {
          Ea[k] = (MODE != 0) ? ps[2 + k] : 0.0;
          Eb[k] = (MODE == 2) ? ps[8 + k] : 0.0;
        }
      } else {  // the patch's edges in order (the same sums)
        C = 0.0;
        U = 0.0;
#pragma unroll
        for (int k = 0; k < 6; k++) Ea[k] = Eb[k] = 0.0;
        for (int q = L.roff[ri]; q < L.roff[ri + 1]; q++) {
          const double* ps = pe + 14 * (size_t)(q - q0);
          C += ps[0];
          U += ps[1];
          if (MODE != 0) {
#pragma unroll
            for (int k = 0; k < 6; k++) {
              Ea[k] += ps[2 + k];
              if (MODE == 2) Eb[k] += ps[8 + k];
            }
          }
        }
      }
      const double Q = 1.0 / (C + lam);  // (:519)
      L.qu[ri] = make_double2(Q, U);
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
    __syncthreads();
    pa = pb;
  }
}

// A published value as one 16-B granule {value, hash, tag}, written by ONE
// 16-B sc1 store: a reader that sees the expected tag and a matching hash has
// the whole value (the granule hand-off of MI355X_MICROARCH.md: no flag, no
// ordering between granules; 16-B sc1 stores observed untorn on gfx950).
// key = (epoch * 64 + iteration + 1) ^ salt: 64 bits, unique per call and
// iteration, and per process (salt: a random 64-bit value drawn once per
// process, so granules another process left in reused memory never carry
// this process's keys).  The tag is key's low word; the hash covers the
// value AND the whole key, so any torn mix of two writes (the tag of one,
// the value and hash of another -- e.g. an internally consistent granule of
// the same parity from iteration it - 2) fails the check, and a granule of
// another call whose key shares the low word fails it through the high word.
__device__ __forceinline__ unsigned gran_hash(unsigned lo, unsigned hi, unsigned long long key) {
  unsigned h = lo ^ 0x5bd1e995u;
  h = (h ^ (h >> 16)) * 0x7feb352du + hi;
  h = (h ^ (h >> 15)) * 0x846ca68bu + (unsigned)key;
  h = (h ^ (h >> 16)) * 0x9E3779B1u + (unsigned)(key >> 32);
  return h ^ (h >> 15);
}
__device__ __forceinline__ v4u granule(double v, unsigned long long key) {
  const unsigned long long b = (unsigned long long)__double_as_longlong(v);
  const unsigned lo = (unsigned)b, hi = (unsigned)(b >> 32);
  v4u r;
  r.x = lo;
  r.y = hi;
  r.z = gran_hash(lo, hi, key);
  r.w = (unsigned)key;
  return r;
}

// fixed-order workgroup reduction of NA accumulators per thread -> out[0..NA)
// (granule mode: gout = this workgroup's granule slot, tag its iteration tag)
template <int NA>
__device__ void reduce_acc(const double* acc, double* red, v4u* gout, unsigned long long tag,
                           int nact) {
  const int tid = opaque_tid();
  // two rounds of 128 columns: red[v][col]; one when only threads below 128
  // hold nonzero sums (nact <= 128: cfg2's workgroups have ~100 relevant
  // edges), saving a barrier and the upper half's stores and adds
  if (nact > 128) {
    if (tid >= 128) {
#pragma unroll
      for (int v = 0; v < NA; v++) red[v * 128 + tid - 128] = acc[v];
    }
    __syncthreads();
    if (tid < 128) {
#pragma unroll
      for (int v = 0; v < NA; v++) red[v * 128 + tid] += acc[v];
    }
  } else if (tid < 128) {
#pragma unroll
    for (int v = 0; v < NA; v++) red[v * 128 + tid] = acc[v];
  }
  __syncthreads();
  // 8 segments of 16 columns per value, 4 independent partial sums each
  double* seg = red + NA * 128;
  for (int t = tid; t < NA * 8; t += kWT) {
    const int v = t >> 3, s = t & 7;
    const double* r = red + v * 128 + 16 * s;
    double p0 = r[0] + r[1], p1 = r[2] + r[3], p2 = r[4] + r[5], p3 = r[6] + r[7];
    p0 += r[8] + r[9];
    p1 += r[10] + r[11];
    p2 += r[12] + r[13];
    p3 += r[14] + r[15];
    seg[t] = (p0 + p1) + (p2 + p3);
  }
  __syncthreads();
  if (tid < NA) {
    const double* s = seg + 8 * tid;
    const double v = ((s[0] + s[1]) + (s[2] + s[3])) + ((s[4] + s[5]) + (s[6] + s[7]));
    const __amdgpu_buffer_rsrc_t rs =
        __builtin_amdgcn_make_buffer_rsrc(gout, 0, 16 * kGranPad, kBufDword3);
    __builtin_amdgcn_raw_buffer_store_b128(granule(v, tag), rs, 16 * tid, 0, kSc1);  // needs no ordering
  }
}

__global__ void __launch_bounds__(kWT) ba_window_kernel(WArgs A) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  const int tid = threadIdx.x, g = blockIdx.x;
  const int N = A.N, P = A.P, PP = P * P, NB = A.NB;
  const float fx = A.intrinsics[0], fy = A.intrinsics[1], cx = A.intrinsics[2],
              cy = A.intrinsics[3];
  const int t0w = A.t0d ? *A.t0d : A.t0;  // first free pose
  // this call's tag: every workgroup reads it at entry; workgroup 0 advances it
  // at its very end, after everyone has read it: each workgroup's read is
  // program-ordered before its RELEASED iteration-0 flag, which workgroup 0
  // acquires before the advance.  Across calls the kernel boundary orders the
  // advance before the next call's reads (a relaxed agent-scope load reads
  // the coherent value), so neither side needs its own fence.
  const long long epoch =
      __hip_atomic_load(&A.flags[kEpochWord], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1;
  mark(A, 0);

  WL L;
  L.ctl = (int*)lds;
  int* ctl = L.ctl;
  int* scr = ctl + cScan;
  L.pose = (float*)(lds + 256);
  L.dX = (double*)(lds + 256 + sizeof(float) * 8 * kWSlots);
  L.tri = (unsigned short*)(lds + 256 + sizeof(float) * 8 * kWSlots + sizeof(double) * 6 * kWMaxN);
  size_t off = al16(256 + sizeof(float) * 8 * kWSlots + sizeof(double) * 6 * kWMaxN +
                    sizeof(unsigned short) * (kWMaxN * (kWMaxN + 1) / 2));
  for (int t = tid; t < NB; t += kWT) {
    int ta, tb;
    tri_of(t, ta, tb);
    L.tri[t] = (unsigned short)((ta << 8) | tb);
  }
  // The first batch of plan entries (below) does not depend on the block: it
  // is issued before the block-work loads so both share one round trip.
  constexpr int kB = 8;
  unsigned m0[kB];
  int pa0[kB], pb0[kB], kx0[kB];
#pragma unroll
  for (int r = 0; r < kB; r++) {
    const int u = min(tid + r * kWT, A.E - 1);
    m0[r] = A.plan.pmask[u];
    pa0[r] = A.plan.poff[u];
    pb0[r] = A.plan.poff[u + 1];
    kx0[r] = A.plan.pkk[u];
  }
  const int nuniq = A.plan.meta[0], fmin = A.plan.meta[1];
  // ---------------- workgroups -> lower blocks ----------------
  // Blocks in the order diagonal (j < N: (j, j)) then strictly lower
  // row-major (j = N + o, o = a (a - 1) / 2 + b); block j gets workgroups
  // [bstart[j], bstart[j + 1]).  Diagonal blocks: the host's Sd each.  Lower
  // blocks: when the host grid has shares to give out (So > 1), one each plus
  // the rest in proportion to their work from the plan (edges of the patches
  // whose free poses hold both poses: the block's re-linearisation count), so
  // that the blocks of the oldest window frames, which most patches see, get
  // more shares (E = 3940: kernel 63.8 -> 54.0 us); otherwise So each.
  // Every wave computes the split in registers (lane l: lower blocks 2l and
  // 2l + 1, one DPP scan, a ballot finds this workgroup's block): no LDS
  // round trip and no barrier; wave 0 leaves bstart in LDS for the gather,
  // ordered before its readers by the setup's barriers.
  int* bstart = reinterpret_cast<int*>(lds + off);  // [NB + 1]
  off = al16(off + sizeof(int) * (kWMaxNB + 1));
  // gather destination of each slot: 36 lblk(a, b) (its block's place in S)
  // for a lower block with one share, whose partial IS the block; -1 for the
  // slots whose block sums several shares (diagonal blocks, split lower blocks)
  int* sdst = reinterpret_cast<int*>(lds + off);  // [G]
  off = al16(off + sizeof(int) * kWMaxG);
  // the split lower blocks (o | lblk << 16), ctl[cLMulti] of them
  int* mlist = reinterpret_cast<int*>(lds + off);  // [NB - N]
  off = al16(off + sizeof(int) * kWMaxNB);
  for (int sl = tid; sl < A.G; sl += kWT) sdst[sl] = -1;
  const int gd = N * A.Sd, nlow = NB - N;
  const int gx = A.G - gd - nlow;  // shares beyond Sd per diagonal and one per lower block
  int blk = 0, sub = 0, S = 1;
  if (NB > 0 && g < gd) {
    blk = g / A.Sd;
    sub = g - blk * A.Sd;
    S = A.Sd;
  }
  if (gx > 0 && nlow > 0) {
    const int lane = tid & 63;
    const int nsh = A.plan.meta[3];
    int w2[2];
#pragma unroll
    for (int h = 0; h < 2; h++) {
      const int o = min(2 * lane + h, nlow - 1);  // clamped: loads stay unconditional
      int ja = 1;
      while ((ja + 1) * ja / 2 <= o) ja++;
      const int4* src = reinterpret_cast<const int4*>(
          A.plan.meta + kMetaWork + (o + ja) * kPlanShardMax);  // lblk(ja, jb) = o + ja
      int wq[kPlanShardMax];
#pragma unroll
      for (int q4 = 0; q4 < kPlanShardMax / 4; q4++) {
        const int4 v = src[q4];
        wq[4 * q4] = v.x;
        wq[4 * q4 + 1] = v.y;
        wq[4 * q4 + 2] = v.z;
        wq[4 * q4 + 3] = v.w;
      }
      int w = 0;
#pragma unroll
      for (int q = 0; q < kPlanShardMax; q++) w += q < nsh ? wq[q] : 0;
      w2[h] = (2 * lane + h < nlow) ? w : 0;
    }
    const int incl = wave_incl_sum(w2[0] + w2[1]);
    const int woff = __builtin_amdgcn_readlane(incl, 63);
    const bool prop = nsh > 0 && woff > 0;  // else the host's So each
    auto share0 = [&](int o, int cum) {
      return gd + (prop ? o + (int)((long long)gx * cum / woff) : o * A.So);
    };
    const int ex = incl - w2[0] - w2[1];
    const int st0 = share0(2 * lane, ex), st1 = share0(2 * lane + 1, ex + w2[0]);
    if (tid < 64) {
      if (2 * lane < nlow) bstart[N + 2 * lane] = st0;
      if (2 * lane + 1 < nlow) bstart[N + 2 * lane + 1] = st1;
    }
    if (g >= gd) {
      const unsigned long long b0 = __ballot(2 * lane < nlow && st0 <= g);
      const unsigned long long b1 = __ballot(2 * lane + 1 < nlow && st1 <= g);
      const int o = __popcll(b0) + __popcll(b1) - 1;  // st(0) = gd <= g
      const int s_o = __builtin_amdgcn_readlane((o & 1) ? st1 : st0, o >> 1);
      const int s_n = (o + 1 >= nlow) ? A.G
                                      : __builtin_amdgcn_readlane(((o + 1) & 1) ? st1 : st0,
                                                                  (o + 1) >> 1);
      blk = N + o;
      sub = g - s_o;
      S = s_n - s_o;
    }
  } else {
    if (tid > N && tid < NB) bstart[tid] = gd + (tid - N) * A.So;
    if (NB > 0 && g >= gd) {
      const int o = (g - gd) / A.So;
      blk = N + o;
      sub = g - gd - o * A.So;
      S = A.So;
    }
  }
  if (tid <= N) bstart[tid] = tid * A.Sd;
  if (tid == 0) bstart[NB] = A.G;
  int a = 0, b = 0;
  if (NB == 0) {
  } else if (blk < N) {
    a = b = blk;
  } else {
    const int o = blk - N;
    a = 1;
    while ((a + 1) * a / 2 <= o) a++;
    b = o - a * (a - 1) / 2;
  }
  const bool diag = (a == b);
  auto diag_shares = [&](int p) { return bstart[p + 1] - bstart[p]; };
  // ---------------- setup: relevant patches of this workgroup ----------------
  // rel(u): mask holds a and b and u % S == sub; workgroup 0 also takes the
  // patches without a free pose (their dZ = Q u).  One scan packs
  // (#patches << 16 | #edges) (E <= 4096 keeps both below 2^16).
  // Global round trips are the setup's cost (~1 us each on a cold L2): the
  // plan meta and the first kB * 256 patches' plan entries are loaded in ONE
  // batch (speculatively, indices clamped to the E-sized arrays), then the
  // patch values, the edge ids and the pose table in a second, then the
  // per-edge inputs in a third.
  const unsigned need = (NB > 0) ? ((1u << a) | (1u << b)) : 0u;
  if (tid == 0) {
    ctl[cFail] = 0;
    ctl[cFailAny] = 0;
    ctl[cTimeout] = 0;
    ctl[cCap] = 0;
    ctl[cLMulti] = 0;
  }
  int* cnt = (int*)(lds + off);  // [nuniq] scan input / prefix (kept until the records are built)
  auto relevant = [&](unsigned m, int u) {
    return (NB == 0) ? true : (((m & need) == need && (u % S) == sub) || (g == 0 && m == 0));
  };
#pragma unroll
  for (int r = 0; r < kB; r++) {
    const int u = tid + r * kWT;
    if (u < nuniq) cnt[u] = relevant(m0[r], u) ? ((1 << 16) | (pb0[r] - pa0[r])) : 0;
  }
  // patches past the first batch (nuniq > kB * 256): loaded here, kB per thread
  // per round trip (loads unconditional: index clamped, value selected after)
  for (int u0 = tid + kB * kWT; u0 < nuniq; u0 += kB * kWT) {
    unsigned m[kB];
    int p0[kB], p1[kB];
#pragma unroll
    for (int r = 0; r < kB; r++) {
      const int u = min(u0 + r * kWT, nuniq - 1);
      m[r] = A.plan.pmask[u];
      p0[r] = A.plan.poff[u];
      p1[r] = A.plan.poff[u + 1];
    }
#pragma unroll
    for (int r = 0; r < kB; r++) {
      const int u = u0 + r * kWT;
      if (u < nuniq) cnt[u] = relevant(m[r], u) ? ((1 << 16) | (p1[r] - p0[r])) : 0;
    }
  }
  mark(A, 40);
  __syncthreads();
  for (int o = tid; o < NB - N; o += kWT) {  // bstart complete after the barrier above
    const int s0 = bstart[N + o], s1 = bstart[N + o + 1];
    int aa = 1;
    while ((aa + 1) * aa / 2 <= o) aa++;  // lblk(aa, o - aa (aa - 1) / 2) = o + aa
    if (s1 - s0 == 1)
      sdst[s0] = 36 * (o + aa);
    else if (s1 - s0 > 1)
      mlist[atomicAdd(&ctl[cLMulti], 1)] = o | ((o + aa) << 16);  // any order: sums are per block
  }
  const int tot = fscan(cnt, nuniq, scr);
  mark(A, 41);
  int nrel = tot >> 16, nrp = tot & 0xffff;
  // LDS plan: [head | cnt | patch records | edge records | region | tw | ej]
  const size_t chunk_b = sizeof(double) * 2 * 14 * kChunk;  // edge records + per-patch sums
  const size_t red_b = sizeof(double) * (36 * 128 + 36 * 8);
  const size_t NN = N > 0 ? N : 1;
  const size_t solve_b =
      sizeof(double) * (36 * (NN * (NN + 1) / 2) + 6 * NN) + wsolve_bytes((int)NN) + 64;
  // gather: S, y and a copy of every published partial (read with one wave of loads)
  const size_t gather_b = sizeof(double) * (36 * (NN * (NN + 1) / 2) + 6 * NN + (size_t)kPartPad * A.G);
  size_t region_b = chunk_b > red_b ? chunk_b : red_b;
  region_b = region_b > solve_b ? region_b : solve_b;
  region_b = region_b > gather_b ? region_b : gather_b;
  const size_t rec0 = al16(off + sizeof(int) * (nuniq + 1));
  auto rec_bytes = [&](int nr, int ne) {
    return al16(sizeof(int) * (nr + 1)) + al16(sizeof(float2) * (nr + 1)) +
           2 * al16(sizeof(float) * (nr + 1)) + al16(sizeof(double2) * (nr + 1)) +
           al16(sizeof(int) * (nr + 1)) + 2 * al16(sizeof(unsigned short) * (ne + 1)) +
           al16(sizeof(int) * (ne + 1));
  };
  bool fits = rec0 + rec_bytes(nrel, nrp) + region_b <= (size_t)kWLds;
  if (!fits) {  // contributes nothing; the call reports status 32 (raised by the extension)
    if (tid == 0) ctl[cCap] = 1;
    nrel = nrp = 0;
  }
  size_t o2 = rec0;
  auto take = [&](size_t bytes) {
    char* p = lds + o2;
    o2 = al16(o2 + bytes);
    return p;
  };
  L.roff = (int*)take(sizeof(int) * (nrel + 1));
  L.nxy = (float2*)take(sizeof(float2) * (nrel + 1));
  L.dep = (float*)take(sizeof(float) * (nrel + 1));
  L.dbase = (float*)take(sizeof(float) * (nrel + 1));
  L.qu = (double2*)take(sizeof(double2) * (nrel + 1));
  L.pkx = (int*)take(sizeof(int) * (nrel + 1));
  L.ec = (unsigned short*)take(sizeof(unsigned short) * (nrp + 1));
  L.rp = (unsigned short*)take(sizeof(unsigned short) * (nrp + 1));
  L.eid = (int*)take(sizeof(int) * (nrp + 1));
  L.region = take(region_b);
  // target/weight and E entries in LDS when they fit; else E entries in the
  // shared HBM buffer (WL::ld_ej) and target/weight read from the inputs
  const size_t tw_b = sizeof(float4) * (nrp + 1), ej_b = sizeof(float) * 12 * (nrp + 1);
  L.tw = nullptr;
  L.ej = nullptr;
  if (o2 + tw_b + ej_b <= (size_t)kWLds) {
    L.tw = (float4*)take(tw_b);
    L.ej = (float*)take(ej_b);
  } else if (o2 + tw_b <= (size_t)kWLds) {
    L.tw = (float4*)take(tw_b);
  }
  // pass A1, thread per relevant patch, no global loads: record offsets, the
  // patch of every position, the final-depth writer
  int* rpo = reinterpret_cast<int*>(L.qu);  // first sorted position (until the first linearisation)
  auto record = [&](int u, int kx, int po, unsigned m, int c0, int c1) {
    const int ri = c0 >> 16, q0 = c0 & 0xffff, ne = (c1 - c0) & 0xffff;
    L.roff[ri] = q0;
    rpo[ri] = po;
    for (int t = 0; t < ne; t++) L.rp[q0 + t] = (unsigned short)ri;
    if (ne > kChunk) ctl[cCap] = 1;
    // writer of the final depth: the diagonal workgroup of one of the
    // patch's free poses (the ((u / 4) mod popc(m))-th, so that the oldest
    // window frames, which most patches see, do not own nearly all of them)
    // with share u % (its shares) -- that workgroup linearised every edge of
    // the patch;
    // workgroup 0 for patches without a free pose
    bool own;
    if (NB == 0) own = true;
    else if (m == 0) own = (g == 0);
    else {
      unsigned mm = m;
      // (the owner's diagonal block is split in diag_shares(p) shares, p its pose)
      for (int t = (u >> 2) % __popc(m); t > 0; t--) mm &= mm - 1;
      const int po = __builtin_ctz(mm);
      own = diag && po == a && (u % diag_shares(po)) == sub;
    }
    L.pkx[ri] = own ? kx : -1;
    return ri;
  };
  // (1) the prefix entries of the thread's patches are read in one batch (a
  // live test per patch between the record stores waited for its own reads)
  // and each live patch leaves (u | mask << 16, kx, first position) at its
  // record index; (2) after a barrier, a thread per record builds it.  A
  // workgroup's few relevant patches are scattered over the kB slots of all
  // threads, so record() run per slot issued its ~200 instructions kB times
  // per wave; per record index it runs once.
  auto cnt_at = [&](int u) { return (u < nuniq) ? cnt[u] : tot; };
  static_assert(kWMaxE <= 65536 && kWMaxN <= 16, "patch index and pose mask packed in 16 bits each");
  int* dl = rpo + (nrel + 1);  // [nrel][3] scratch in qu's space past rpo (qu: 4 ints per record)
  bool lv0[kB];
  {
    int c0[kB], c1[kB];
#pragma unroll
    for (int r = 0; r < kB; r++) {
      const int u = min(tid + r * kWT, nuniq - 1);
      c0[r] = cnt[u];
      c1[r] = cnt_at(u + 1);
    }
#pragma unroll
    for (int r = 0; r < kB; r++) {
      const int u = tid + r * kWT;
      lv0[r] = nrel > 0 && u < nuniq && c0[r] != c1[r];
      if (lv0[r]) {
        int* d = dl + 3 * (c0[r] >> 16);
        d[0] = (int)((unsigned)u | (m0[r] << 16));
        d[1] = kx0[r];
        d[2] = pa0[r];
      }
    }
  }
  for (int u0 = tid + kB * kWT; u0 < nuniq && nrel > 0; u0 += kB * kWT) {
    int kx[kB], po[kB];
    unsigned msk[kB];
#pragma unroll
    for (int r = 0; r < kB; r++) {
      const int uc = min(u0 + r * kWT, nuniq - 1);
      kx[r] = A.plan.pkk[uc];
      po[r] = A.plan.poff[uc];
      msk[r] = A.plan.pmask[uc];
    }
    int c0[kB], c1[kB];
#pragma unroll
    for (int r = 0; r < kB; r++) {
      const int uc = min(u0 + r * kWT, nuniq - 1);
      c0[r] = cnt[uc];
      c1[r] = cnt_at(uc + 1);
    }
#pragma unroll
    for (int r = 0; r < kB; r++) {
      const int u = u0 + r * kWT;
      if (u < nuniq && c0[r] != c1[r]) {
        int* d = dl + 3 * (c0[r] >> 16);
        d[0] = (int)((unsigned)u | (msk[r] << 16));
        d[1] = kx[r];
        d[2] = po[r];
      }
    }
  }
  __syncthreads();
  // the record's patch values [0][1][1], [1][1][1], [2][1][1], [2][0][0]
  // (ba_cuda.cu:282-285, :225) are loaded first: their round trip overlaps
  // the record's LDS work
  const int c11 = P + 1;
  for (int t = tid; t < nrel; t += kWT) {
    const int* d = dl + 3 * t;
    const unsigned um = (unsigned)d[0];
    const int u = (int)(um & 0xffffu), kx = d[1];
    const float* pk = A.patches + (size_t)kx * 3 * PP;
    const float v0 = pk[c11], v1 = pk[PP + c11], v2 = pk[2 * PP + c11], v3 = pk[2 * PP];
    record(u, kx, d[2], um >> 16, cnt[u], cnt_at(u + 1));
    L.nxy[t] = make_float2((v0 - cx) / fx, (v1 - cy) / fy);
    L.dep[t] = v2;
    L.dbase[t] = v3;  // patch_retr_kernel reads [2][0][0] (:225)
  }
  if (tid == 0) L.roff[nrel] = nrp;
  __syncthreads();
  mark(A, 42);
  // pass B, second round trip: the edge ids of this thread's first kB
  // relevant edges and the pose table, all issued before any is used
  int ev0[kB];
#pragma unroll
  for (int r = 0; r < kB; r++) {
    const int q = min(tid + r * kWT, max(nrp - 1, 0));
    const int ri = nrp > 0 ? L.rp[q] : 0;
    const int p = nrp > 0 ? rpo[ri] + (q - L.roff[ri]) : 0;
    ev0[r] = A.plan.epos[min(max(p, 0), A.E - 1)];
  }
  // pose table: free poses t0.., then fixed ones from fmin
  constexpr int kPr = kWSlots * 8 / kWT;
  float pv[kPr];
#pragma unroll
  for (int r = 0; r < kPr; r++) {
    const int k = tid + r * kWT, sl = k >> 3, c = k & 7;
    const int gp = (sl < N) ? t0w + sl : fmin + (sl - N);
    pv[r] = A.poses[7 * (size_t)min(max(gp, 0), A.num_poses - 1) + min(c, 6)];
  }
#pragma unroll
  for (int r = 0; r < kPr; r++) {
    const int k = tid + r * kWT, sl = k >> 3, c = k & 7;
    const int gp = (sl < N) ? t0w + sl : fmin + (sl - N);
    const bool ok = c < 7 && gp >= 0 && gp < A.num_poses && (sl < N || fmin != 0x7fffffff);
    L.pose[k] = ok ? pv[r] : ((c == 6) ? 1.0f : 0.0f);
  }
  mark(A, 43);
  // pass B, thread per relevant edge: slots, edge index, target/weight (the
  // third round trip; further batches of kB edges per thread each need two)
  for (int q0 = tid; q0 < nrp; q0 += kB * kWT) {
    int ev[kB];
    if (q0 == tid) {
#pragma unroll
      for (int r = 0; r < kB; r++) ev[r] = ev0[r];
    } else {
#pragma unroll
      for (int r = 0; r < kB; r++) {  // unconditional loads (see above)
        const int q = min(q0 + r * kWT, nrp - 1);
        const int ri = L.rp[q];
        ev[r] = A.plan.epos[rpo[ri] + (q - L.roff[ri])];
      }
    }
    int64_t gi[kB], gj[kB];
    float2 tg[kB], wt[kB];
#pragma unroll
    for (int r = 0; r < kB; r++) {
      const int e = ev[r];
      gi[r] = A.ii[e];
      gj[r] = A.jj[e];
      tg[r] = reinterpret_cast<const float2*>(A.target)[e];
      wt[r] = reinterpret_cast<const float2*>(A.weight)[e];
    }
#pragma unroll
    for (int r = 0; r < kB; r++) {
      const int q = q0 + r * kWT;
      if (q >= nrp) continue;
      const unsigned si = wslot((int)gi[r], t0w, N, fmin), sj = wslot((int)gj[r], t0w, N, fmin);
      L.ec[q] = (unsigned short)(si | (sj << 8));
      L.eid[q] = ev[r];
      if (L.tw) L.tw[q] = make_float4(tg[r].x, tg[r].y, wt[r].x, wt[r].y);
    }
  }
  __syncthreads();
  mark(A, 1);
  if (A.marks && tid == 0 && g < 256) A.marks[1152 + g] = (int64_t)wall_clock64();  // setup done
  const int nrel_e = nrel;

  // ---------------- iterations ----------------
  const double lam = (double)A.lmbda[0];
  for (int it = 0; it < A.iters; it++) {
    const int tid = opaque_tid();  // (shadows the kernel's: see opaque_tid)
    const int mb = 2 + 8 * it;
    if (it > 0) {
      // ---- apply dX of iteration it-1: poses, then inverse depths ----
      for (int i = tid; i < N; i += kWT) {  // pose_retr_kernel (:178-206)
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
      for (int ri = tid; ri < nrel_e; ri += kWT) {  // dZ = Q (u - E^T dX) (:563), patch_retr (:209-229)
        const double ex = patch_etdx(L, A, ri, (it - 1) & 1, N);
        const double2 qu = L.qu[ri];
        const float dz = (float)(qu.x * (qu.y - ex));
        const float base = (it == 1) ? L.dbase[ri] : L.dep[ri];
        float d = base + dz;
        d = (d > 20.0f) ? 1.0f : d;
        L.dep[ri] = (float)fmax((double)d, 1e-4);
      }
      __syncthreads();
    }
    // ---- linearise + assemble this workgroup's block ----
    double acc[36];
    int nact = kWT;  // threads that can hold nonzero acc (assemble)
    // partials double-buffered by iteration parity: a workgroup can only reach
    // buffer it & 1 again (iteration it + 2) after every workgroup has published
    // iteration it + 1, i.e. after each finished reading iteration it's slots
    double* red = reinterpret_cast<double*>(L.region);
    const unsigned long long gkey = (unsigned long long)(epoch * 64 + it + 1) ^ A.salt;
    const unsigned gtag = (unsigned)gkey;
    v4u* const gbuf = A.gran + (size_t)(it & 1) * A.G * kGranPad;
    v4u* const gslot = gbuf + (size_t)g * kGranPad;
    if (NB == 0) {
      assemble<0>(A, L, nrel_e, a, b, lam, fx, fy, cx, cy, it & 1, acc, nact);
    } else if (diag) {
      assemble<1>(A, L, nrel_e, a, b, lam, fx, fy, cx, cy, it & 1, acc, nact);
      mark(A, mb + 4);
      if (A.marks && tid == 0 && it == 0 && g < 256) A.marks[1408 + g] = (int64_t)wall_clock64();
      reduce_acc<27>(acc, red, gslot, gkey, nact);
    } else {
      assemble<2>(A, L, nrel_e, a, b, lam, fx, fy, cx, cy, it & 1, acc, nact);
      if (A.marks && tid == 0 && it == 0 && g < 256) A.marks[1408 + g] = (int64_t)wall_clock64();
      reduce_acc<36>(acc, red, gslot, gkey, nact);
    }
    mark(A, mb + 0);
    if (A.marks && tid == 0 && it < 2 && g < 256)  // per-workgroup stamps (instrumentation)
      A.marks[128 + 256 * it + g] = (int64_t)wall_clock64();
    if (NB == 0) continue;  // structure only: dZ = Q u, applied after the loop
    const int NNb = N;
    double* Sd = reinterpret_cast<double*>(L.region);
    double* yd = Sd + 36 * NB;
    double* pc = yd + 6 * N;  // [G][kPartPad] copy of the partials
    // the reduction scratch (red, seg) and pc share L.region: no thread may
    // write pc before the publishing threads have read their sums
    __syncthreads();
    // ---- granule hand-off: every thread polls the granules it gathers ----
    // No flag and no barrier between "published" and "loaded": a granule is
    // consumed as soon as its tag (this call's epoch, this iteration) and
    // hash check out, so the gather overlaps the wait for the slowest
    // workgroup and the tail after it is one load round trip.
    {
      const int ndg = bstart[NNb];  // diagonal blocks' workgroups first: 27 granules, the others 36
      const int T = ndg * 27 + (A.G - ndg) * 36;
      const int pcoff = (int)(pc - Sd);
      const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
          gbuf, 0, (int)(16 * kGranPad * (size_t)A.G), kBufDword3);
      constexpr int kIn = 16;
      const long long tw0 = (long long)wall_clock64();
      bool late = false;
      for (int t0_ = tid; t0_ < T; t0_ += kIn * kWT) {
        int off[kIn], pos[kIn];
        unsigned pend = 0;
#pragma unroll
        for (int r = 0; r < kIn; r++) {
          const int t = min(t0_ + r * kWT, T - 1);
          int sl, k;
          if (t < ndg * 27) {
            sl = t / 27;
            k = t - 27 * sl;
          } else {
            const int u = t - ndg * 27;
            sl = ndg + u / 36;
            k = u - 36 * (u / 36);
          }
          off[r] = 16 * (sl * kGranPad + k);
          // its place: in S for a one-share lower block, else in the partials copy
          const int sd = sdst[sl];
          pos[r] = sd >= 0 ? sd + k : pcoff + sl * kPartPad + k;
          pend |= (t0_ + r * kWT < T) ? (1u << r) : 0u;
        }
        while (pend) {
          v4u v[kIn];
#pragma unroll
          for (int r = 0; r < kIn; r++)  // all kIn in flight (unconditional loads)
            v[r] = __builtin_bit_cast(v4u, __builtin_amdgcn_raw_buffer_load_b128(rs, off[r], 0, kSc1));
#pragma unroll
          for (int r = 0; r < kIn; r++) {
            const bool ok = ((pend >> r) & 1u) && v[r].w == gtag && v[r].z == gran_hash(v[r].x, v[r].y, gkey);
            if (ok) {
              Sd[pos[r]] = __longlong_as_double((long long)(((unsigned long long)v[r].y << 32) | v[r].x));
              pend &= ~(1u << r);
            }
          }
          if (!pend) break;
          if ((long long)wall_clock64() - tw0 > kSpin) {
            late = true;
            break;
          }
          __builtin_amdgcn_s_sleep(1);
        }
      }
      if (late) ctl[cTimeout] = 1;
    }
    mark(A, mb + 1);
    if (A.marks && tid == 0 && it < 2 && g < 256) A.marks[640 + 256 * it + g] = (int64_t)wall_clock64();
    __syncthreads();
    mark(A, mb + 5);  // every thread's granules in LDS
    {
      // The blocks that sum several shares, in share order: every diagonal
      // block (21 stored entries mirrored to 36, and its 6 y entries) and the
      // split lower blocks, if any; a one-share lower block is already in S.
      // (One wave per SIMD: the cost here is instruction issue, so the work is
      // only what needs summing -- summing all 36 NB + 6 N entries from the
      // partials copy was 3.3 us per iteration.)
      for (int t = tid; t < 42 * N; t += kWT) {
        const int p = t / 42, e = t - 42 * p;
        const int x = e / 6, z = e - 6 * x;  // e >= 36: y entry z (x == 6)
        const int xx = max(x, z), zz = min(x, z);
        const int idx = (x == 6) ? 21 + z : xx * (xx + 1) / 2 + zz;
        const int s0 = bstart[p], s1 = bstart[p + 1];
        double sv = 0.0;
        for (int sb = s0; sb < s1; sb++) sv += pc[sb * kPartPad + idx];
        if (x == 6) {
          yd[6 * p + z] = sv;
        } else {
          if (x == z) sv += 1e-4 * sv + 1.0;  // S += I (1e-4 S + 1) (ba_cuda.cu:560)
          Sd[36 * lblk(p, p) + e] = sv;
        }
      }
      for (int t = tid; t < 36 * ctl[cLMulti]; t += kWT) {
        const int q = t / 36, k = t - 36 * q, ol = mlist[q], o = ol & 0xffff;
        const int s0 = bstart[N + o], s1 = bstart[N + o + 1];
        double sv = 0.0;
        for (int sb = s0; sb < s1; sb++) sv += pc[sb * kPartPad + k];
        Sd[36 * (ol >> 16) + k] = sv;
      }
    }
    __syncthreads();
    mark(A, mb + 2);
    // ---- dense solve, redundantly in every workgroup (identical bits) ----
    WSolve sv;
    sv.S = Sd;
    sv.y = yd;
    sv.x = yd + 6 * N;
    sv.r = sv.x + 6 * N;
    sv.A = reinterpret_cast<float*>(sv.r + 6 * N);
    sv.Z = sv.A + 36 * NB;
    sv.v0 = sv.Z + 36 * NB;
    sv.v1 = sv.v0 + 6 * N;
    const bool ok = wsolve(sv, N, kRefine, &ctl[cFail]);
    const bool zero = !ok || ctl[cTimeout] != 0;
    for (int k = tid; k < 6 * N; k += kWT) {
      const double v = zero ? 0.0 : sv.x[k];  // (dpvo/ba.py:17-21)
      L.dX[k] = v;
      if (g == 0 && A.dxo) A.dxo[k] = v;
    }
    if (!ok && tid == 0) ctl[cFailAny] = 1;
    __syncthreads();
    mark(A, mb + 3);
  }

  // ---------------- final apply + write-back ----------------
  if (A.iters > 0) {
    const int it = A.iters;
    for (int i = tid; i < N; i += kWT) {
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
    mark(A, 48);  // final-apply sub-phases (instrumentation): poses retracted
    if (A.marks && g == 0 && tid == 0) {
      A.marks[52] = nrp;
      A.marks[53] = (L.ej ? 2 : 1);  // E entries in LDS, else in the HBM buffer
    }
    mark(A, 49);
    {
      // the depths this workgroup writes (owned patches); with the E entries
      // in HBM, kTP threads per patch: each sums E^T dX over a contiguous
      // part of the patch's edges
      // (patch_etdx's per-edge order inside the part), the parts are added in
      // part order -- one HBM round trip of E entries instead of one per 4
      // edges of a ~18-edge patch on a single thread
      constexpr int kTP = 8;
      // region: olist [nrel + 1] (owned flags -> prefix), oidx [nrel], opart [owned][kTP]
      int* olist = reinterpret_cast<int*>(L.region);
      double* opart = reinterpret_cast<double*>(L.region + al16(sizeof(int) * (2 * (size_t)nrel_e + 1)));
      if (L.ej ||
          al16(sizeof(int) * (2 * (size_t)nrel_e + 1)) + sizeof(double) * kTP * (size_t)nrel_e > region_b) {
        // E entries in LDS (short patches, cfg2-like windows), or more relevant
        // patches than the region holds parts for: one thread per patch
        for (int ri = tid; ri < nrel_e; ri += kWT) {
          if (L.pkx[ri] < 0) continue;
          const double ex = patch_etdx(L, A, ri, (it - 1) & 1, N);
          const double2 qu = L.qu[ri];
          const float dz = (float)(qu.x * (qu.y - ex));
          const float base = (it == 1) ? L.dbase[ri] : L.dep[ri];
          float d = base + dz;
          d = (d > 20.0f) ? 1.0f : d;
          L.dep[ri] = (float)fmax((double)d, 1e-4);
        }
        olist = nullptr;
      }
      if (olist) {
      for (int ri = tid; ri < nrel_e; ri += kWT) olist[ri] = L.pkx[ri] >= 0 ? 1 : 0;
      __syncthreads();
      const int nown = fscan(olist, nrel_e, ctl + cScan);  // olist[ri] = owned patches before ri
      // compact: owned patch k -> relevant index (stored after the prefix array)
      int* oidx = olist + nrel_e + 1;
      for (int ri = tid; ri < nrel_e; ri += kWT)
        if (L.pkx[ri] >= 0) oidx[olist[ri]] = ri;
      __syncthreads();
      for (int t = tid; t < nown * kTP; t += kWT) {
        const int k = t / kTP, part = t % kTP, ri = oidx[k];
        const int qa = L.roff[ri], qz = L.roff[ri + 1], len = (qz - qa + kTP - 1) / kTP;
        const int q0 = min(qa + part * len, qz), q1 = min(q0 + len, qz);
        opart[t] = edges_etdx(L, A, q0, q1, (it - 1) & 1, N);
      }
      __syncthreads();
      for (int k = tid; k < nown; k += kWT) {
        const int ri = oidx[k];
        double ex = 0.0;
#pragma unroll
        for (int part = 0; part < kTP; part++) ex += opart[k * kTP + part];
        const double2 qu = L.qu[ri];
        const float dz = (float)(qu.x * (qu.y - ex));
        const float base = (it == 1) ? L.dbase[ri] : L.dep[ri];
        float d = base + dz;
        d = (d > 20.0f) ? 1.0f : d;
        L.dep[ri] = (float)fmax((double)d, 1e-4);
      }
      }
    }
    __syncthreads();
    mark(A, 50);  // depths updated
    for (int k = tid; k < nrel_e * PP; k += kWT) {
      const int ri = k / PP, c = k % PP;
      const int kx = L.pkx[ri];
      if (kx >= 0) A.patches[(size_t)kx * 3 * PP + 2 * PP + c] = L.dep[ri];
    }
    if (g == 0)
      for (int i = tid; i < N; i += kWT) {
        const int gp = t0w + i;
        if (gp >= 0 && gp < A.num_poses)
          for (int c = 0; c < 7; c++) A.poses[7 * (size_t)gp + c] = L.pose[8 * i + c];
      }
  }
  if (tid == 0) {
    int st = 0;
    if (ctl[cTimeout]) st |= kStTimeout;
    if (g == 0) st |= A.plan.meta[2];  // kk clamp from the plan
    if (ctl[cCap]) st |= kStCap;
    if (g == 0 && ctl[cFailAny]) st |= kStChol;
    if (st) {
      atomicOr(A.status, st);
      if (A.sink) atomicOr(A.sink, st);
    }
    if (g == 0) {
      __hip_atomic_store(&A.flags[kEpochWord], epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      mark(A, 63);
    }
    if (A.marks && g < 256) A.marks[2176 + g] = (int64_t)wall_clock64();  // workgroup end
  }
}

}  // namespace

// ---------------------------------------------------------------- host side
static size_t al256w(size_t v) { return (v + 255) / 256 * 256; }

struct WGrid {
  int NB, Sd, So, G;
};
static WGrid window_grid(int E, int N) {
  WGrid w;
  w.NB = N * (N + 1) / 2;
  if (N <= 0) {
    w.Sd = w.So = 1;
    w.G = 1;
    return w;
  }
  // shares per block: sparse graphs (cfg2: ~1.8 edges per patch) load the
  // diagonal blocks most; DPVO windows (a patch sees ~10 free poses) load
  // every block alike, so large windows split all blocks evenly
  w.So = E > 2048 ? 4 : 1;
  w.Sd = 4;
  auto G = [&]() { return N * w.Sd + (w.NB - N) * w.So; };
  while (G() > kWMaxG && w.Sd > 1) {
    if (w.Sd > w.So) w.Sd--;
    else if (w.So > 1) w.So--;
    else w.Sd--;
  }
  w.G = G();
  return w;
}

// Workgroups of ba_window_kernel the current device can hold at once (its
// grid exchange needs every workgroup resident): CUs x blocks per CU, asked
// once per device.  0 if the runtime cannot say (then nothing is supported).
static int window_coresident() {
  static std::mutex mu;
  static std::map<int, int> cache;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return 0;
  std::lock_guard<std::mutex> lk(mu);
  auto it = cache.find(dev);
  if (it != cache.end()) return it->second;
  int cus = 0, per = 0;
  (void)hipFuncSetAttribute((const void*)ba_window_kernel,
                            hipFuncAttributeMaxDynamicSharedMemorySize, kWLds);
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
      hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, (const void*)ba_window_kernel, kWT,
                                                   kWLds) != hipSuccess) {
    (void)hipGetLastError();
    cus = per = 0;
  }
  cache[dev] = cus * per;
  return cache[dev];
}

// per-process granule-key salt (granule()): drawn once from the OS entropy
// source, mixed with the clock and the pid in case the source is weak
static unsigned long long granule_salt() {
  static const unsigned long long salt = [] {
    unsigned long long v = 0;
    try {
      std::random_device rd;
      v = ((unsigned long long)rd() << 32) ^ rd();
    } catch (...) {
    }
    v ^= (unsigned long long)std::chrono::steady_clock::now().time_since_epoch().count() *
         0x9E3779B97F4A7C15ull;
    v ^= (unsigned long long)getpid() << 17;
    return v;
  }();
  return salt;
}

bool ba_window_supported(int E, int N, int P) {
  if (E <= 0 || E > kWMaxE || N < 0 || N > kWMaxN || P < 2 || P * P > 64) return false;
  const int G = window_grid(E, N).G;
  return G <= kWMaxG && G <= window_coresident();
}

// granules of one grid: [2][G][kGranPad]
static size_t gran_count(const WGrid& w) { return (size_t)2 * kGranPad * w.G; }

size_t ba_window_scratch_bytes(int E, int N) {
  const WGrid w = window_grid(E, N);
  return al256w(sizeof(int) * (size_t)E) + al256w(sizeof(int) * (size_t)(E + 1)) +
         al256w(sizeof(unsigned) * (size_t)E) + al256w(sizeof(int) * (size_t)E) +
         al256w(kMetaBytes) + al256w(sizeof(double) * 2 * kPartPad * (size_t)w.G) +
         al256w((size_t)16 * gran_count(w)) + al256w(sizeof(float) * 24 * (size_t)E);
}

namespace {
std::mutex g_wflag_mu;
std::map<int, long long*> g_wflags;  // per device; BA calls on one device must not overlap
long long* wflag_slot(hipStream_t st) {
  int dev = 0;
  (void)hipGetDevice(&dev);
  std::lock_guard<std::mutex> lk(g_wflag_mu);
  auto it = g_wflags.find(dev);
  if (it != g_wflags.end()) return it->second;
  long long* p = nullptr;
  if (hipMalloc(&p, sizeof(long long) * kFlagWords) != hipSuccess) return nullptr;
  if (hipMemsetAsync(p, 0, sizeof(long long) * kFlagWords, st) != hipSuccess) return nullptr;
  g_wflags[dev] = p;
  return p;
}
}  // namespace

namespace {
std::mutex g_sink_mu;
std::map<int, int*> g_sink;  // per device: caller's sticky status word
int* sink_for_device() {
  int dev = 0;
  (void)hipGetDevice(&dev);
  std::lock_guard<std::mutex> lk(g_sink_mu);
  auto it = g_sink.find(dev);
  return it == g_sink.end() ? nullptr : it->second;
}
}  // namespace

void ba_set_status_sink(int* sink) {
  int dev = 0;
  (void)hipGetDevice(&dev);
  std::lock_guard<std::mutex> lk(g_sink_mu);
  g_sink[dev] = sink;
}

// byte offsets of the plan arrays inside the window scratch (tests, tools)
void ba_window_plan_offsets(int E, int64_t* out) {
  out[0] = 0;                                                  // epos [E]
  out[1] = out[0] + (int64_t)al256w(sizeof(int) * (size_t)E);  // poff [E + 1]
  out[2] = out[1] + (int64_t)al256w(sizeof(int) * (size_t)(E + 1));  // pmask [E]
  out[3] = out[2] + (int64_t)al256w(sizeof(unsigned) * (size_t)E);  // pkk [E]
  out[4] = out[3] + (int64_t)al256w(sizeof(int) * (size_t)E);  // meta [8]: nuniq, fmin, status;
                                                               // [16, 28): int64 phase stamps
}

static Plan plan_view(char* scratch, int E, int* status) {
  Plan p;
  char* s = scratch;
  p.epos = (int*)s;
  s += al256w(sizeof(int) * (size_t)E);
  p.poff = (int*)s;
  s += al256w(sizeof(int) * (size_t)(E + 1));
  p.pmask = (unsigned*)s;
  s += al256w(sizeof(unsigned) * (size_t)E);
  p.pkk = (int*)s;
  s += al256w(sizeof(int) * (size_t)E);
  p.meta = (int*)s;
  p.status = status;
  p.sink = sink_for_device();
  p.t0d = nullptr;
  return p;
}

static void set_attrs() {
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)ba_window_kernel,
                              hipFuncAttributeMaxDynamicSharedMemorySize, kWLds);
    (void)hipFuncSetAttribute((const void*)ba_plan_kernel,
                              hipFuncAttributeMaxDynamicSharedMemorySize, kWLds);
    (void)hipFuncSetAttribute((const void*)reproject_plan_kernel,
                              hipFuncAttributeMaxDynamicSharedMemorySize, kWLds);
    (void)hipFuncSetAttribute((const void*)reproject_plan_insert_kernel<float>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, kWLds);
    (void)hipFuncSetAttribute((const void*)reproject_plan_insert_kernel<__half>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, kWLds);
    attr = true;
  }
}

// edge grouping only (reads ii / jj / kk): may run on another stream than
// the iterations, e.g. concurrently with A-CORR
int ba_window_plan(const int64_t* ii, const int64_t* jj, const int64_t* kk, int E, int num_patches,
                   int num_poses, int t0, int t1, char* scratch, int* status, void* stream,
                   const int* t0d) {
  set_attrs();
  Plan plan = plan_view(scratch, E, status);
  plan.t0d = t0d;
  hipLaunchKernelGGL(ba_plan_kernel, dim3(plan_shards(E)), dim3(kPT), kWLds, as_stream(stream), ii, jj, kk, E,
                     num_patches, num_poses, t0, t1 - t0, plan);
  return launch_status();
}

// reprojection + A-CORR edge order + edge grouping in one launch (shapes
// validated by the caller, dpvo_reproject_ordered_plan)
int ba_window_reproject_plan(const float* poses, const float* patches, const float* intrinsics,
                             const int64_t* ii, const int64_t* jj, const int64_t* kk, int E, int P,
                             int num_poses, int num_patches, int N2, float* coords, int* order,
                             int t0, int t1, char* scratch, int* status, void* stream,
                             const int* t0d) {
  set_attrs();
  Plan plan = plan_view(scratch, E, status);
  plan.t0d = t0d;
  RArgs r;
  r.marks = nullptr;
  r.poses = poses;
  r.patches = patches;
  r.intrinsics = intrinsics;
  r.ii = ii;
  r.jj = jj;
  r.kk = kk;
  r.E = E;
  r.P = P;
  r.num_poses = num_poses;
  r.num_patches = num_patches;
  r.N2 = N2;
  r.t0 = t0;
  r.N = t1 - t0;
  r.coords = coords;
  r.order = order;
  r.nps = plan_shards(E);
  const int total = E * P * P;
  hipLaunchKernelGGL(reproject_plan_kernel, dim3(r.nps + 1 + (total + kPT - 1) / kPT), dim3(kPT), kWLds,
                     as_stream(stream), r, plan);
  return launch_status();
}

// reproject + order + plan + frame insertion (src [C, H, W] NCHW fp32 / fp16,
// dst[l] the channels-last slot of level l, scale[l] in {1, 2, 4, 8})
int ba_window_reproject_plan_insert(const float* poses, const float* patches,
                                    const float* intrinsics, const int64_t* ii, const int64_t* jj,
                                    const int64_t* kk, int E, int P, int num_poses,
                                    int num_patches, int N2, float* coords, int* order, int t0,
                                    int t1, char* scratch, int* status, const void* src,
                                    void* const* dst, const int* scale, int L, int C, int H, int W,
                                    int half, int64_t* marks, void* stream) {
  set_attrs();
  Plan plan = plan_view(scratch, E, status);
  plan.t0d = nullptr;
  RArgs r;
  r.marks = marks;
  r.poses = poses;
  r.patches = patches;
  r.intrinsics = intrinsics;
  r.ii = ii;
  r.jj = jj;
  r.kk = kk;
  r.E = E;
  r.P = P;
  r.num_poses = num_poses;
  r.num_patches = num_patches;
  r.N2 = N2;
  r.t0 = t0;
  r.N = t1 - t0;
  r.coords = coords;
  r.order = order;
  r.nps = plan_shards(E);
  InsArgs I = {};
  I.src = src;
  I.L = L;
  I.C = C;
  I.H = H;
  I.W = W;
  I.lv.mem = 1;
  for (int l = 0; l < L; l++) {
    I.lv.dst[l] = dst[l];
    I.lv.s[l] = scale[l];
  }
  I.gx = (W + kInsTX - 1) / kInsTX;
  I.gy = (H + kInsTY - 1) / kInsTY;
  I.ntile = I.gx * I.gy * ((C + kInsTC - 1) / kInsTC);
  const int nrep = (E * P * P + kPT - 1) / kPT;
  const dim3 grid(r.nps + 1 + nrep + (I.ntile + 1) / 2);
  // LDS sized for this E (the plan's need), not the kWMaxE maximum: the
  // insertion tiles then run several workgroups per CU beside the plan
  size_t lds = plan_lds_bytes(plan_cap(E));
  lds = std::max(lds, sizeof(float) * 2 * kInsTC * kInsCS);
  lds = std::max(lds, sizeof(int) * (size_t)(kOrderBins + 2));
  if (half)
    hipLaunchKernelGGL(reproject_plan_insert_kernel<__half>, grid, dim3(kPT), lds,
                       as_stream(stream), r, plan, I, nrep);
  else
    hipLaunchKernelGGL(reproject_plan_insert_kernel<float>, grid, dim3(kPT), lds,
                       as_stream(stream), r, plan, I, nrep);
  return launch_status();
}

int ba_window_run(float* poses, float* patches, const float* intrinsics, const float* target,
                  const float* weight, const float* lmbda, const int64_t* ii, const int64_t* jj,
                  const int64_t* kk, int E, int P, int num_poses, int num_patches, int t0, int t1,
                  int iterations, char* scratch, int* status, int64_t* marks, double* dxo,
                  void* stream, const int* t0d = nullptr);

int ba_window_launch(float* poses, float* patches, const float* intrinsics, const float* target,
                     const float* weight, const float* lmbda, const int64_t* ii, const int64_t* jj,
                     const int64_t* kk, int E, int P, int num_poses, int num_patches, int t0, int t1,
                     int iterations, char* scratch, int* status, int64_t* marks, double* dxo,
                     void* stream) {
  const int rc = ba_window_plan(ii, jj, kk, E, num_patches, num_poses, t0, t1, scratch, status,
                                stream, nullptr);
  if (rc) return rc;
  return ba_window_run(poses, patches, intrinsics, target, weight, lmbda, ii, jj, kk, E, P,
                       num_poses, num_patches, t0, t1, iterations, scratch, status, marks, dxo,
                       stream);
}

int ba_window_run(float* poses, float* patches, const float* intrinsics, const float* target,
                  const float* weight, const float* lmbda, const int64_t* ii, const int64_t* jj,
                  const int64_t* kk, int E, int P, int num_poses, int num_patches, int t0, int t1,
                  int iterations, char* scratch, int* status, int64_t* marks, double* dxo,
                  void* stream, const int* t0d) {
  set_attrs();
  if (iterations > 63) return DPVO_ERR_UNSUPPORTED;  // 6-bit iteration tag per epoch
  const int N = t1 - t0;
  const WGrid w = window_grid(E, N);
  hipStream_t st = as_stream(stream);
  WArgs a;
  a.flags = wflag_slot(st);
  if (!a.flags) return DPVO_ERR_LAUNCH;
  a.plan = plan_view(scratch, E, status);
  char* s = scratch + al256w(sizeof(int) * (size_t)E) + al256w(sizeof(int) * (size_t)(E + 1)) +
            al256w(sizeof(unsigned) * (size_t)E) + al256w(sizeof(int) * (size_t)E) +
            al256w(kMetaBytes);
  a.part = (double*)s;
  s += al256w(sizeof(double) * 2 * kPartPad * (size_t)w.G);
  a.gran = (v4u*)s;
  s += al256w((size_t)16 * gran_count(w));
  a.ejg = (float*)s;
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
  a.t0d = t0d;
  a.N = N;
  a.iters = iterations;
  a.NB = w.NB;
  a.Sd = w.Sd;
  a.So = w.So;
  a.G = w.G;
  a.status = status;
  a.sink = a.plan.sink;
  a.marks = marks;
  a.dxo = dxo;
  a.salt = granule_salt();
  hipLaunchKernelGGL(ba_window_kernel, dim3(w.G), dim3(kWT), kWLds, st, a);
  return launch_status();
}

}  // namespace dpvo
