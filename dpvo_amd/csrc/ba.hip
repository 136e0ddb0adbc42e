// ba.hip -- fastba on gfx950: F-BA (Schur bundle adjustment), F-REPROJ, F-NBR.
//
// Reference semantics: dpvo/fastba/ba_cuda.cu + block_e.cu + ba.cpp
// (cuteboyqq/DPVO).  One F-BA iteration (ba_cuda.cu:482-579):
//   per edge: residual + Jacobians (fp32, :265-333); B, E, C, v, u sums
//   Q = 1/(C+lmbda); S = B - E Q E^T; y = v - E Q u; S += I*(1e-4 S + 1)
//   dX = chol_solve(S, y); dZ = Q (u - E^T dX); pose / patch retraction.
//
// MI355X design (DESIGN.md "F-BA"): no float atomics anywhere.
//   setup  (1 WG, once per call): sort kk in LDS (bitonic), unique/inverse,
//          group edges by patch, build each patch's sorted free-pose list.
//   linearize (thread per patch): the fp32 edge math of the reference, patch
//          sums C,u and the patch's E column blocks c_{u,p} (fp64, private).
//   schur  (one WG per lower 6x6 block of S): B and E Q E^T terms reduced in
//          registers + LDS in a fixed order -> deterministic fp64 S, y.
//   solve  (1 WG): damping, fp64 Cholesky in LDS (L kept in the upper
//          triangle, one barrier per column), triangular solves in one wave,
//          pose retraction, dZ and patch retraction.
// The split (build_schur -> all-reduce(S,y) -> solve_update) is the
// edge-sharded multi-GPU form.
#include "common.hpp"

namespace dpvo {

constexpr int kSetupThreads = 1024;
constexpr int kMaxSetupE = 16384;  // LDS: 16384 x 8 B keys = 128 KiB
constexpr int kMaxFree = 20;       // 6N <= 120: fp64 S in LDS = 116 KiB (and <= 32 for masks)
constexpr int kSchurThreads = 256;
constexpr int kSolveThreads = 1024;
constexpr int kJStride = 32;       // floats per edge: w r Jz Ji[2][6] Jj[2][6]

struct BaWs {
  int32_t* ku;      // [E]   inverse index into unique patches
  int32_t* pedge;   // [E]   edges grouped by patch (ascending edge id)
  int32_t* poff;    // [E+1] patch -> edge range
  int32_t* boff;    // [E+1] patch -> pose-block range
  int32_t* bpose;   // [2E]  free pose of each block (ascending per patch)
  int32_t* eslot;   // [2E]  block slot of (ii, jj) of each edge, -1 = fixed pose
  int32_t* meta;    // [4]   nuniq, status, nblocks, num_patches
  int64_t* kx;      // [E]   unique patch ids (ascending)
  int64_t* skey;    // [E]   sorted kk (scratch)
  float* J;         // [E][32]
  double* Q;        // [E]
  double* U;        // [E]
  double* cb;       // [2E][6]
  double* S;        // [NL][36]
  double* y;        // [6N]
  double* dX;       // [6N]
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
  t.ku = (int32_t*)take(sizeof(int32_t) * E);
  t.pedge = (int32_t*)take(sizeof(int32_t) * E);
  t.poff = (int32_t*)take(sizeof(int32_t) * (E + 1));
  t.boff = (int32_t*)take(sizeof(int32_t) * (E + 1));
  t.bpose = (int32_t*)take(sizeof(int32_t) * 2 * E);
  t.eslot = (int32_t*)take(sizeof(int32_t) * 2 * E);
  t.meta = (int32_t*)take(sizeof(int32_t) * 4);
  t.kx = (int64_t*)take(sizeof(int64_t) * E);
  t.skey = (int64_t*)take(sizeof(int64_t) * E);
  t.J = (float*)take(sizeof(float) * kJStride * E);
  t.Q = (double*)take(sizeof(double) * E);
  t.U = (double*)take(sizeof(double) * E);
  t.cb = (double*)take(sizeof(double) * 12 * E);
  t.S = (double*)take(sizeof(double) * 36 * (NL ? NL : 1));
  t.y = (double*)take(sizeof(double) * 6 * (N ? N : 1));
  t.dX = (double*)take(sizeof(double) * 6 * (N ? N : 1));
  if (w) *w = t;
  return off;
}

// ---------------------------------------------------------------------------
// block-wide exclusive scan of data[0..n) in LDS (int), returns the total.
// scratch: >= kSetupThreads/64 + 1 ints of LDS.
// ---------------------------------------------------------------------------
__device__ int block_exclusive_scan(int* data, int n, int* scratch) {
  const int tid = threadIdx.x, nt = blockDim.x;
  const int per = (n + nt - 1) / nt;
  const int lo = min(tid * per, n), hi = min(lo + per, n);
  int s = 0;
  for (int i = lo; i < hi; i++) s += data[i];
  // inclusive wave scan of s
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
  int run = scratch[wid] + v - s;  // exclusive prefix of this thread's chunk
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
// setup: unique/inverse of kk (torch::_unique(kk, sorted, inverse),
// ba_cuda.cu:447), edges grouped by patch, per-patch free-pose block lists.
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(kSetupThreads)
    ba_setup_kernel(const int64_t* __restrict__ ii, const int64_t* __restrict__ jj,
                    const int64_t* __restrict__ kk, int E, int num_patches, int t0, int N,
                    int P2, BaWs w) {
  extern __shared__ __attribute__((aligned(16))) unsigned long long keys[];
  const int tid = threadIdx.x, nt = blockDim.x;
  int* scratch = reinterpret_cast<int*>(keys + P2);  // kSetupThreads/64 + 1 ints
  int& bad = scratch[kSetupThreads / 64 + 1];
  if (tid == 0) bad = 0;
  __syncthreads();
  for (int i = tid; i < P2; i += nt) {
    unsigned long long k = ~0ull;
    if (i < E) {
      int64_t v = kk[i];
      if (v < 0 || v >= num_patches) {
        bad = 1;
        v = v < 0 ? 0 : num_patches - 1;
      }
      k = ((unsigned long long)v << 32) | (unsigned)i;
    }
    keys[i] = k;
  }
  __syncthreads();
  // bitonic sort (ascending) of P2 keys
  for (int size = 2; size <= P2; size <<= 1) {
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      for (int i = tid; i < P2 / 2; i += nt) {
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
  for (int i = tid; i < E; i += nt) {
    w.pedge[i] = (int)(keys[i] & 0xffffffffu);
    w.skey[i] = (int64_t)(keys[i] >> 32);
  }
  __syncthreads();
  int* flag = reinterpret_cast<int*>(keys);  // keys no longer needed
  for (int i = tid; i < E; i += nt) flag[i] = (i == 0 || w.skey[i] != w.skey[i - 1]) ? 1 : 0;
  __syncthreads();
  // heads must be read before the scan overwrites them: keep a copy in poff
  for (int i = tid; i < E; i += nt) w.poff[i] = flag[i];
  __syncthreads();
  const int nuniq = block_exclusive_scan(flag, E, scratch);
  for (int i = tid; i < E; i += nt) {
    const int r = flag[i] + w.poff[i] - 1;  // rank of this sorted position
    w.ku[w.pedge[i]] = r;
    flag[i] = r;
  }
  __syncthreads();
  for (int i = tid; i < E; i += nt) {
    if (i == 0 || flag[i] != flag[i - 1]) {
      w.kx[flag[i]] = w.skey[i];
      w.poff[flag[i]] = i;
    }
  }
  __syncthreads();
  if (tid == 0) {
    w.poff[nuniq] = E;
    w.meta[0] = nuniq;
    w.meta[1] = bad ? 2 : 0;
    w.meta[3] = num_patches;
  }
  __syncthreads();
  // ---- per-patch free-pose lists (N <= 32: one bit per free pose) ----
  int* cnt = flag;
  for (int u = tid; u < nuniq; u += nt) {
    unsigned mask = 0;
    for (int t = w.poff[u]; t < w.poff[u + 1]; t++) {
      const int e = w.pedge[t];
      const int64_t pi = ii[e] - t0, pj = jj[e] - t0;
      if (pi >= 0 && pi < N) mask |= 1u << pi;
      if (pj >= 0 && pj < N) mask |= 1u << pj;
    }
    cnt[u] = __popc(mask);
  }
  __syncthreads();
  const int nblocks = block_exclusive_scan(cnt, nuniq, scratch);
  for (int u = tid; u < nuniq; u += nt) w.boff[u] = cnt[u];
  if (tid == 0) {
    w.boff[nuniq] = nblocks;
    w.meta[2] = nblocks;
  }
  __syncthreads();
  // slot(p) = number of distinct free poses < p in the patch (ascending list)
  for (int u = tid; u < nuniq; u += nt) {
    unsigned mask = 0;
    const int a = w.poff[u], b = w.poff[u + 1];
    for (int t = a; t < b; t++) {
      const int e = w.pedge[t];
      const int64_t pi = ii[e] - t0, pj = jj[e] - t0;
      if (pi >= 0 && pi < N) mask |= 1u << pi;
      if (pj >= 0 && pj < N) mask |= 1u << pj;
    }
    const int base = w.boff[u];
    for (unsigned m = mask; m; m &= m - 1) {
      const int p = __ffs(m) - 1;
      w.bpose[base + __popc(mask & ((1u << p) - 1u))] = p;
    }
    for (int t = a; t < b; t++) {
      const int e = w.pedge[t];
      const int64_t pi = ii[e] - t0, pj = jj[e] - t0;
      w.eslot[2 * e + 0] = (pi >= 0 && pi < N) ? __popc(mask & ((1u << pi) - 1u)) : -1;
      w.eslot[2 * e + 1] = (pj >= 0 && pj < N) ? __popc(mask & ((1u << pj) - 1u)) : -1;
    }
  }
}

// ---------------------------------------------------------------------------
// linearize: one thread per unique patch.  fp32 edge math exactly as
// reprojection_residuals_and_hessian (ba_cuda.cu:265-333); patch sums in fp64.
// ---------------------------------------------------------------------------
__device__ __forceinline__ void edge_linearize(const float* __restrict__ poses,
                                               const float* __restrict__ patches, int P, float fx,
                                               float fy, float cx, float cy, float tx, float ty,
                                               float wx, float wy, int ix, int jx, int64_t kx,
                                               float* __restrict__ o) {
  const float* pi = poses + 7 * (size_t)ix;
  const float* pj = poses + 7 * (size_t)jx;
  const float* pk = patches + (size_t)kx * 3 * P * P;
  const int c11 = P + 1;  // patches[kx][*][1][1]  (ba_cuda.cu:282-285)
  float ti[3] = {pi[0], pi[1], pi[2]}, qi[4] = {pi[3], pi[4], pi[5], pi[6]};
  float tj[3] = {pj[0], pj[1], pj[2]}, qj[4] = {pj[3], pj[4], pj[5], pj[6]};
  float Xi[4], Xj[4];
  Xi[0] = (pk[c11] - cx) / fx;
  Xi[1] = (pk[P * P + c11] - cy) / fy;
  Xi[2] = 1.0f;
  Xi[3] = pk[2 * P * P + c11];
  float tij[3], qij[4];
  relSE3(ti, qi, tj, qj, tij, qij);
  actSE3(tij, qij, Xi, Xj);
  const float X = Xj[0], Y = Xj[1], Z = Xj[2], W = Xj[3];
  const float d = ((double)Z >= 0.2) ? 1.0f / Z : 0.0f;  // ba_cuda.cu:296
  const float d2 = d * d;
  const float x1 = fx * (X / Z) + cx;
  const float y1 = fy * (Y / Z) + cy;
  const float rx = tx - x1, ry = ty - y1;
  const bool in_bounds = (sqrtf(rx * rx + ry * ry) < 128.0f) && ((double)Z > 0.2) &&
                         (x1 > -64.0f) && (y1 > -64.0f) && (x1 < 2.0f * cx + 64.0f) &&
                         (y1 < 2.0f * cy + 64.0f);  // :305-306
  const float mask = in_bounds ? 1.0f : 0.0f;
  float Jj0[6] = {fx * W * d, 0.0f, fx * -X * W * d2, fx * -X * Y * d2, fx * (1 + X * X * d2),
                  fx * -Y * d};
  float Jj1[6] = {0.0f, fy * W * d, fy * -Y * W * d2, fy * (-1 - Y * Y * d2), fy * (X * Y * d2),
                  fy * X * d};
  float Ji0[6], Ji1[6];
  adjSE3(tij, qij, Jj0, Ji0);
  adjSE3(tij, qij, Jj1, Ji1);
  o[0] = mask * wx;
  o[1] = mask * wy;
  o[2] = tx - x1;
  o[3] = ty - y1;
  o[4] = fx * (tij[0] * d - tij[2] * (X * d2));
  o[5] = fy * (tij[1] * d - tij[2] * (Y * d2));
#pragma unroll
  for (int a = 0; a < 6; a++) {
    o[6 + a] = Ji0[a];
    o[12 + a] = Ji1[a];
    o[18 + a] = Jj0[a];
    o[24 + a] = Jj1[a];
  }
}

__global__ void __launch_bounds__(256)
    ba_linearize_kernel(const float* __restrict__ poses, const float* __restrict__ patches,
                        const float* __restrict__ intrinsics, const float* __restrict__ target,
                        const float* __restrict__ weight, const float* __restrict__ lmbda,
                        const int64_t* __restrict__ ii, const int64_t* __restrict__ jj,
                        const int64_t* __restrict__ kk, int P, int num_poses, BaWs w) {
  const int u = blockIdx.x * blockDim.x + threadIdx.x;
  const int nuniq = w.meta[0];
  if (u >= nuniq) return;
  const float fx = intrinsics[0], fy = intrinsics[1], cx = intrinsics[2], cy = intrinsics[3];
  const double lam = (double)lmbda[0];
  const int a = w.poff[u], b = w.poff[u + 1];
  const int b0 = w.boff[u], nb = w.boff[u + 1] - b0;
  double* cbp = w.cb + 6 * (size_t)b0;
  for (int i = 0; i < 6 * nb; i++) cbp[i] = 0.0;
  double C = 0.0, Uu = 0.0;
  for (int t = a; t < b; t++) {
    const int e = w.pedge[t];
    int ix = (int)ii[e], jx = (int)jj[e];
    ix = min(max(ix, 0), num_poses - 1);  // memory guard (reference: unchecked)
    jx = min(max(jx, 0), num_poses - 1);
    float* o = w.J + (size_t)kJStride * e;
    const int64_t kx = min(max(kk[e], (int64_t)0), (int64_t)w.meta[3] - 1);
    edge_linearize(poses, patches, P, fx, fy, cx, cy, target[2 * e], target[2 * e + 1],
                   weight[2 * e], weight[2 * e + 1], ix, jx, kx, o);
    const int si = w.eslot[2 * e], sj = w.eslot[2 * e + 1];
    for (int row = 0; row < 2; row++) {
      const double wr = o[row];
      const float r = o[2 + row], Jz = o[4 + row];
      const float* Ji = o + 6 + 6 * row;
      const float* Jj = o + 18 + 6 * row;
      for (int k = 0; k < 6; k++) {  // E blocks (ba_cuda.cu:352-363)
        if (si >= 0) cbp[6 * si + k] -= wr * Jz * Ji[k];
        if (sj >= 0) cbp[6 * sj + k] += wr * Jz * Jj[k];
      }
      C += wr * Jz * Jz;  // :372-373
      Uu += wr * r * Jz;
    }
  }
  w.Q[u] = 1.0 / (C + lam);  // :519
  w.U[u] = Uu;
}

// ---------------------------------------------------------------------------
// schur: one workgroup per lower 6x6 block (a, b), a >= b, of
//   S = B - E Q E^T  and (diagonal blocks) y = v - E Q u.
// ---------------------------------------------------------------------------
__device__ __forceinline__ void tri_decode(int t, int* a, int* b) {
  int r = (int)((sqrtf(8.0f * t + 1.0f) - 1.0f) * 0.5f);
  while (r * (r + 1) / 2 > t) r--;
  while ((r + 1) * (r + 2) / 2 <= t) r++;
  *a = r;
  *b = t - r * (r + 1) / 2;
}

__global__ void __launch_bounds__(kSchurThreads)
    ba_schur_kernel(const int64_t* __restrict__ ii, const int64_t* __restrict__ jj, int E, int t0,
                    int N, BaWs w, double* __restrict__ S_out, double* __restrict__ y_out) {
  __shared__ double red[42][kSchurThreads / 64];
  int pa, pb;
  tri_decode(blockIdx.x, &pa, &pb);
  const bool diag = pa == pb;
  const int tid = threadIdx.x;
  double acc[36], yacc[6];
#pragma unroll
  for (int i = 0; i < 36; i++) acc[i] = 0.0;
#pragma unroll
  for (int i = 0; i < 6; i++) yacc[i] = 0.0;

  // ---- B and v terms (ba_cuda.cu:339-370) ----
  for (int e = tid; e < E; e += kSchurThreads) {
    const int64_t pi = ii[e] - t0, pj = jj[e] - t0;
    const bool fi = pi >= 0 && pi < N, fj = pj >= 0 && pj < N;
    int mode = 0;  // bit0: +JiJi^T, bit1: +JjJj^T, bit2: -(JiJj^T+JjJi^T), bit3: -JiJj^T, bit4: -JjJi^T
    if (diag) {
      if (fi && pi == pa) mode |= 1;
      if (fj && pj == pa) mode |= 2;
      if (fi && fj && pi == pa && pj == pa) mode |= 4;
    } else {
      if (fi && fj && pi == pa && pj == pb) mode |= 8;
      if (fi && fj && pj == pa && pi == pb) mode |= 16;
    }
    if (!mode) continue;
    const float* o = w.J + (size_t)kJStride * e;
    for (int row = 0; row < 2; row++) {
      const double wr = o[row];
      const float r = o[2 + row];
      const float* Ji = o + 6 + 6 * row;
      const float* Jj = o + 18 + 6 * row;
      float ji[6], jv[6];
#pragma unroll
      for (int k = 0; k < 6; k++) { ji[k] = Ji[k]; jv[k] = Jj[k]; }
#pragma unroll
      for (int x = 0; x < 6; x++)
#pragma unroll
        for (int z = 0; z < 6; z++) {
          double s = 0.0;
          if (mode & 1) s += wr * ji[x] * ji[z];
          if (mode & 2) s += wr * jv[x] * jv[z];
          if (mode & 4) s -= wr * ji[x] * jv[z] + wr * jv[x] * ji[z];
          if (mode & 8) s -= wr * ji[x] * jv[z];
          if (mode & 16) s -= wr * jv[x] * ji[z];
          acc[x * 6 + z] += s;
        }
      if (diag) {
#pragma unroll
        for (int x = 0; x < 6; x++) {
          if (mode & 1) yacc[x] -= wr * r * ji[x];
          if (mode & 2) yacc[x] += wr * r * jv[x];
        }
      }
    }
  }
  // ---- E Q E^T and E Q u terms (ba_cuda.cu:554-558) ----
  const int nuniq = w.meta[0];
  for (int u = tid; u < nuniq; u += kSchurThreads) {
    const int b0 = w.boff[u], b1 = w.boff[u + 1];
    int sa = -1, sb = -1;
    for (int s = b0; s < b1; s++) {
      const int p = w.bpose[s];
      if (p == pa) sa = s;
      if (p == pb) sb = s;
    }
    if (sa < 0 || sb < 0) continue;
    const double q = w.Q[u];
    const double* ca = w.cb + 6 * (size_t)sa;
    const double* cbb = w.cb + 6 * (size_t)sb;
    double va[6], vb[6];
#pragma unroll
    for (int k = 0; k < 6; k++) { va[k] = ca[k]; vb[k] = cbb[k]; }
#pragma unroll
    for (int x = 0; x < 6; x++)
#pragma unroll
      for (int z = 0; z < 6; z++) acc[x * 6 + z] -= va[x] * q * vb[z];
    if (diag) {
      const double qu = q * w.U[u];
#pragma unroll
      for (int x = 0; x < 6; x++) yacc[x] -= va[x] * qu;
    }
  }
  // ---- fixed-order reduction: wave shuffles, then across waves ----
  const int lane = tid & 63, wid = tid >> 6;
#pragma unroll
  for (int i = 0; i < 42; i++) {
    double v = i < 36 ? acc[i] : yacc[i - 36];
    v = wave_sum(v);
    if (lane == 0) red[i][wid] = v;
  }
  __syncthreads();
  if (tid < 42) {
    double s = 0.0;
    for (int k = 0; k < kSchurThreads / 64; k++) s += red[tid][k];
    if (tid < 36)
      S_out[(size_t)blockIdx.x * 36 + tid] = s;
    else if (diag)
      y_out[6 * pa + (tid - 36)] = s;
  }
}

// ---------------------------------------------------------------------------
// solve + update (single workgroup).
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(kSolveThreads)
    ba_solve_kernel(float* __restrict__ poses, float* __restrict__ patches, int P, int num_poses,
                    int t0, int N, const double* __restrict__ S_in, const double* __restrict__ y_in,
                    BaWs w, double* __restrict__ dX_out) {
  extern __shared__ __attribute__((aligned(16))) double sm[];
  const int n = 6 * N;
  const int ld = n + 1;  // padded row stride (banks)
  double* S = sm;                        // [n][ld]
  double* diagL = S + (size_t)n * ld;    // [n]
  double* x = diagL + n;                 // [n]
  int& fail = *reinterpret_cast<int*>(x + n);
  const int tid = threadIdx.x, nt = blockDim.x;
  if (tid == 0) fail = 0;
  if (n > 0) {
    // lower blocks -> dense lower triangle; damping S += I * (1e-4 S + 1) (ba_cuda.cu:560)
    const int NL = N * (N + 1) / 2;
    for (int t = tid; t < NL * 36; t += nt) {
      const int blk = t / 36, e = t % 36;
      int a, b;
      tri_decode(blk, &a, &b);
      const int r = 6 * a + e / 6, c = 6 * b + e % 6;
      double v = S_in[t];
      if (r == c) v += 1e-4 * v + 1.0;
      if (c <= r) S[r * ld + c] = v;
    }
    for (int i = tid; i < n; i += nt) x[i] = y_in[i];
    __syncthreads();
    // Cholesky, right-looking; L(r,j) stored at S[j][r] (upper triangle)
    for (int j = 0; j < n; j++) {
      const double d = S[j * ld + j];
      if (!(d > 0.0)) {  // uniform: every thread reads the same value
        if (tid == 0) fail = 1;
        break;
      }
      const double sd = sqrt(d), inv_d = 1.0 / d;
      const int m = n - j - 1;
      for (int t = tid; t < m * m; t += nt) {
        const int r = j + 1 + t / m, c = j + 1 + t % m;
        if (c <= r) S[r * ld + c] -= S[r * ld + j] * S[c * ld + j] * inv_d;
      }
      for (int r = j + 1 + tid; r < n; r += nt) S[j * ld + r] = S[r * ld + j] / sd;
      if (tid == 0) diagL[j] = sd;
      __syncthreads();
    }
    __syncthreads();
    if (fail) {
      for (int i = tid; i < n; i += nt) x[i] = 0.0;  // dX = 0 (dpvo/ba.py:17-21)
    } else if (tid < 64) {
      // forward L z = y, backward L^T x = z, one wave (wave-synchronous LDS)
      for (int j = 0; j < n; j++) {
        const double z = x[j] / diagL[j];
        wave_lds_sync();
        for (int r = j + 1 + tid; r < n; r += 64) x[r] -= S[j * ld + r] * z;
        if (tid == 0) x[j] = z;
        wave_lds_sync();
      }
      for (int j = n - 1; j >= 0; j--) {
        const double v = x[j] / diagL[j];
        wave_lds_sync();
        for (int r = tid; r < j; r += 64) x[r] -= S[r * ld + j] * v;
        if (tid == 0) x[j] = v;
        wave_lds_sync();
      }
    }
    __syncthreads();
    for (int i = tid; i < n; i += nt) {
      w.dX[i] = x[i];
      if (dX_out) dX_out[i] = x[i];
    }
    // pose retraction poses[t0+i] <- Exp(dX_i) poses[t0+i] (pose_retr_kernel :178-206)
    for (int i = tid; i < N; i += nt) {
      const int t = t0 + i;
      if (t < 0 || t >= num_poses) continue;
      float* pt = poses + 7 * (size_t)t;
      float xi[6], t1[3], q1[4];
      for (int k = 0; k < 6; k++) xi[k] = (float)x[6 * i + k];
      float tt[3] = {pt[0], pt[1], pt[2]}, qq[4] = {pt[3], pt[4], pt[5], pt[6]};
      retrSE3(xi, tt, qq, t1, q1);
      pt[0] = t1[0]; pt[1] = t1[1]; pt[2] = t1[2];
      pt[3] = q1[0]; pt[4] = q1[1]; pt[5] = q1[2]; pt[6] = q1[3];
    }
  }
  if (tid == 0) w.meta[1] = (w.meta[1] & ~1) | (fail ? 1 : 0);
  // dZ = Q (u - E^T dX) and patch retraction (patch_retr_kernel :209-229)
  const int nuniq = w.meta[0];
  for (int u = tid; u < nuniq; u += nt) {
    double s = w.U[u];
    if (n > 0) {
      for (int b = w.boff[u]; b < w.boff[u + 1]; b++) {
        const int p = w.bpose[b];
        const double* c = w.cb + 6 * (size_t)b;
        for (int k = 0; k < 6; k++) s -= c[k] * x[6 * p + k];
      }
    }
    const float dz = (float)(w.Q[u] * s);
    float* pk = patches + (size_t)w.kx[u] * 3 * P * P + 2 * P * P;
    float d = pk[0] + dz;
    d = (d > 20.0f) ? 1.0f : d;
    d = (float)fmax((double)d, 1e-4);
    for (int k = 0; k < P * P; k++) pk[k] = d;
  }
}

static size_t solve_smem(int N) {
  const int n = 6 * N;
  return sizeof(double) * ((size_t)n * (n + 1) + 2 * (size_t)n + 2);  // + fail flag
}

// ---------------------------------------------------------------------------
// F-REPROJ (ba_cuda.cu:379-429): one thread per (edge, patch pixel).
// ---------------------------------------------------------------------------
__global__ void reproject_kernel(const float* __restrict__ poses, const float* __restrict__ patches,
                                 const float* __restrict__ intrinsics,
                                 const int64_t* __restrict__ ii, const int64_t* __restrict__ jj,
                                 const int64_t* __restrict__ kk, int E, int P, int num_poses,
                                 int num_patches, float* __restrict__ coords) {
  const int PP = P * P;
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= E * PP) return;
  const int n = t / PP, pix = t % PP;
  const float fx = intrinsics[0], fy = intrinsics[1], cx = intrinsics[2], cy = intrinsics[3];
  const int ix = (int)min(max(ii[n], (int64_t)0), (int64_t)num_poses - 1);
  const int jx = (int)min(max(jj[n], (int64_t)0), (int64_t)num_poses - 1);
  const int64_t kx = min(max(kk[n], (int64_t)0), (int64_t)num_patches - 1);
  const float* pi = poses + 7 * (size_t)ix;
  const float* pj = poses + 7 * (size_t)jx;
  float ti[3] = {pi[0], pi[1], pi[2]}, qi[4] = {pi[3], pi[4], pi[5], pi[6]};
  float tj[3] = {pj[0], pj[1], pj[2]}, qj[4] = {pj[3], pj[4], pj[5], pj[6]};
  float tij[3], qij[4];
  relSE3(ti, qi, tj, qj, tij, qij);
  const float* pk = patches + (size_t)kx * 3 * PP;
  float Xi[4], Xj[4];
  Xi[0] = (pk[pix] - cx) / fx;
  Xi[1] = (pk[PP + pix] - cy) / fy;
  Xi[2] = 1.0f;
  Xi[3] = pk[2 * PP + pix];
  actSE3(tij, qij, Xi, Xj);
  coords[((size_t)n * 2 + 0) * PP + pix] = fx * (Xj[0] / Xj[2]) + cx;
  coords[((size_t)n * 2 + 1) * PP + pix] = fy * (Xj[1] / Xj[2]) + cy;
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

}  // namespace dpvo

using namespace dpvo;

static size_t setup_smem(int P2) {
  return sizeof(unsigned long long) * P2 + sizeof(int) * (kSetupThreads / 64 + 4);
}

// Kernels whose LDS exceeds the 64 KiB default opt in to the 160 KiB of a CU.
static void ensure_lds_limits() {
  static bool done = false;
  if (done) return;
  (void)hipFuncSetAttribute((const void*)ba_setup_kernel,
                            hipFuncAttributeMaxDynamicSharedMemorySize,
                            (int)setup_smem(kMaxSetupE));
  (void)hipFuncSetAttribute((const void*)ba_solve_kernel,
                            hipFuncAttributeMaxDynamicSharedMemorySize, (int)solve_smem(kMaxFree));
  done = true;
}

static int pow2_at_least(int v) {
  int p = 1;
  while (p < v) p <<= 1;
  return p;
}

DPVO_EXPORT size_t dpvo_ba_workspace_bytes(int E, int t0, int t1) {
  const int N = t1 > t0 ? t1 - t0 : 0;
  return ba_layout(E > 0 ? E : 1, N, nullptr, nullptr);
}

DPVO_EXPORT int dpvo_ba_max_free_poses(void) { return kMaxFree; }

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
  const int P2 = pow2_at_least(E < 2 ? 2 : E);
  hipLaunchKernelGGL(ba_setup_kernel, dim3(1), dim3(kSetupThreads), setup_smem(P2),
                     as_stream(stream), ii, jj, kk, E, num_patches, t0, N, P2, w);
  return launch_status();
}

DPVO_EXPORT int dpvo_ba_build_schur(const float* poses, const float* patches,
                                    const float* intrinsics, const float* target,
                                    const float* weight, const float* lmbda, const int64_t* ii,
                                    const int64_t* jj, const int64_t* kk, int E, int P,
                                    int num_poses, int t0, int t1, void* workspace,
                                    double* S_lower, double* y, void* stream) {
  if (E <= 0) return DPVO_OK;
  if (P < 2 || num_poses <= 0 || t1 < t0) return DPVO_ERR_INVALID;
  const int N = t1 - t0;
  if (N > kMaxFree || E > kMaxSetupE) return DPVO_ERR_UNSUPPORTED;
  BaWs w;
  ba_layout(E, N, (char*)workspace, &w);
  hipStream_t s = as_stream(stream);
  hipLaunchKernelGGL(ba_linearize_kernel, dim3((E + 255) / 256), dim3(256), 0, s, poses, patches,
                     intrinsics, target, weight, lmbda, ii, jj, kk, P, num_poses, w);
  int st = launch_status();
  if (st || N == 0) return st;
  const int NL = N * (N + 1) / 2;
  hipLaunchKernelGGL(ba_schur_kernel, dim3(NL), dim3(kSchurThreads), 0, s, ii, jj, E, t0, N, w,
                     S_lower ? S_lower : w.S, y ? y : w.y);
  return launch_status();
}

DPVO_EXPORT int dpvo_ba_solve_update(float* poses, float* patches, const double* S_lower,
                                     const double* y, int E, int P, int num_poses, int t0, int t1,
                                     void* workspace, double* dX_out, void* stream) {
  if (E <= 0) return DPVO_OK;
  if (P < 2 || t1 < t0) return DPVO_ERR_INVALID;
  const int N = t1 - t0;
  if (N > kMaxFree) return DPVO_ERR_UNSUPPORTED;
  BaWs w;
  ba_layout(E, N, (char*)workspace, &w);
  ensure_lds_limits();
  hipLaunchKernelGGL(ba_solve_kernel, dim3(1), dim3(kSolveThreads), solve_smem(N),
                     as_stream(stream), poses, patches, P, num_poses, t0, N,
                     S_lower ? S_lower : w.S, y ? y : w.y, w, dX_out);
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

DPVO_EXPORT int dpvo_ba_forward(float* poses, float* patches, const float* intrinsics,
                                const float* target, const float* weight, const float* lmbda,
                                const int64_t* ii, const int64_t* jj, const int64_t* kk, int E,
                                int P, int num_poses, int num_patches, int PPF, int t0, int t1,
                                int iterations, int eff_impl, void* workspace,
                                size_t workspace_bytes, void* stream) {
  (void)PPF;
  (void)eff_impl;  // one block-sparse implementation serves both reference paths
  if (E <= 0 || iterations <= 0) return DPVO_OK;
  int st = dpvo_ba_setup(ii, jj, kk, E, num_patches, t0, t1, workspace, workspace_bytes, stream);
  if (st) return st;
  for (int it = 0; it < iterations; it++) {
    st = dpvo_ba_build_schur(poses, patches, intrinsics, target, weight, lmbda, ii, jj, kk, E, P,
                             num_poses, t0, t1, workspace, nullptr, nullptr, stream);
    if (st) return st;
    st = dpvo_ba_solve_update(poses, patches, nullptr, nullptr, E, P, num_poses, t0, t1,
                              workspace, nullptr, stream);
    if (st) return st;
  }
  return DPVO_OK;
}

DPVO_EXPORT int dpvo_reproject(const float* poses, const float* patches, const float* intrinsics,
                               const int64_t* ii, const int64_t* jj, const int64_t* kk, int E,
                               int P, int num_poses, int num_patches, float* coords, void* stream) {
  if (E <= 0) return DPVO_OK;
  if (P <= 0 || num_poses <= 0 || num_patches <= 0) return DPVO_ERR_INVALID;
  const int total = E * P * P;
  hipLaunchKernelGGL(reproject_kernel, dim3((total + 255) / 256), dim3(256), 0,
                     as_stream(stream), poses, patches, intrinsics, ii, jj, kk, E, P, num_poses,
                     num_patches, coords);
  return launch_status();
}

DPVO_EXPORT int dpvo_neighbors_max_edges(void) { return 1 << 30; }

DPVO_EXPORT int dpvo_neighbors(const int64_t* ii, const int64_t* jj, int E, int64_t* ix,
                               int64_t* jx, void* stream) {
  if (E <= 0) return DPVO_OK;
  hipLaunchKernelGGL(neighbors_kernel, dim3((E + 255) / 256), dim3(256), 0, as_stream(stream), ii,
                     jj, E, ix, jx);
  return launch_status();
}
