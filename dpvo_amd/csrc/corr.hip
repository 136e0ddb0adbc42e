// corr.hip -- altcorr on gfx950: A-CORR, A-CORR-BWD, A-PATCH, A-PATCH-BWD.
//
// Reference semantics: dpvo/altcorr/correlation_kernel.cu (cuteboyqq/DPVO).
//   raw[b,m,yy,xx,i0,j0] = sum_c fmap1[b,ii[m],c,i0,j0] * fmap2[b,jj[m],c,y0+yy-R,x0+xx-R]
//   (0 outside the map), y0 = floor(y), x0 = floor(x)                  (:82-175)
//   out = bilinear(raw, frac(x), frac(y)) permuted to [b,m,xx,yy,i0,j0] (:232-272)
//
// MI355X design (DESIGN.md "A-CORR"): one 64-lane wave per edge.  The p*p
// windows of one edge overlap, so instead of 576 independent 128-long dot
// products (the reference's one-thread-per-output, every fmap2 value read
// p*p times) the wave treats the edge as a tiny GEMM
//     G[k][px] = sum_c f1[c][k] * f2[c][px]   over the UNION bounding box of
// the windows (<= 128 pixels, two per lane): every fmap2 value of the edge is
// loaded once, f1 (4.6 KB, wave-uniform) comes through the scalar cache into
// SGPR operands of v_fma, and the bilinear + permute is fused into the store
// phase, which gathers raw values from G in LDS.  No intermediate volume is
// written to HBM.
#include "common.hpp"

namespace dpvo {

// corr_nchw.hip: the matrix-core forward for NCHW fp16 / fp32 levels (returns
// DPVO_ERR_UNSUPPORTED outside its shape; the VALU kernels below take those)
int corr_nchw_mma(const void* fmap1, const void* const* fmap2, const int* H2, const int* W2,
                  const float* scale, int L, bool use_scale, const float* coords,
                  const int64_t* ii, const int64_t* jj, int B, int M, int C, int np, int N1,
                  int N2, int R, int dtype, void* out_t, float* out_f, hipStream_t s);

constexpr int kCorrWaves = 4;       // waves (edges) per workgroup
constexpr int kBoxPx = 2 * kWave;   // bounding-box pixels per wave (2 per lane)

struct CorrLevel {
  const void* f2;
  int H2, W2;
  float scale;
};
struct CorrLevels {
  CorrLevel lv[8];
};

// Per-wave scratch in LDS: slab (G or raw) + per-patch-pixel geometry.
template <int NPT>
struct CorrGeom {
  int x0[NPT], y0[NPT];
  float dx[NPT], dy[NPT];
};

// Compute one edge's correlation (one level) and write the bilinear,
// permuted output.  `out_stride`/`out_off` let the fused multi-level kernel
// interleave levels on the last axis (DPVO's torch.stack(..., -1)).
template <typename T, int NPT>
__device__ __forceinline__ void corr_edge(const T* __restrict__ fmap1, const T* __restrict__ fmap2,
                          const float* __restrict__ coords, int b, int m, int ix, int jx, int M,
                          int C, int np, int N1, int N2, int H2, int W2, int R, float scale,
                          bool use_scale, typename Acc<T>::type* slab, CorrGeom<NPT>* geo,
                          T* __restrict__ out_t, float* __restrict__ out_f, int out_stride,
                          int out_off) {
  using A = typename Acc<T>::type;
  const int lane = threadIdx.x & (kWave - 1);
  const int D = 2 * R + 2, Dp = D - 1;

  // ---- geometry: coords [B,M,2,np] -> floor / frac per patch pixel ----
  float cv = 0.f;
  if (lane < 2 * np) {
    cv = coords[((size_t)b * M + m) * 2 * np + lane];
    if (use_scale) cv = cv / scale;  // reference: coords / scale (dpvo.py:462-463)
  }
  int xlo = 0x7fffffff, xhi = -0x7fffffff, ylo = 0x7fffffff, yhi = -0x7fffffff;
#pragma unroll
  for (int k = 0; k < NPT; k++) {
    if (k < np) {
      const float x = __shfl(cv, k, kWave);
      const float y = __shfl(cv, np + k, kWave);
      const int xf = ifloor_safe(x), yf = ifloor_safe(y);
      xlo = min(xlo, xf);
      xhi = max(xhi, xf);
      ylo = min(ylo, yf);
      yhi = max(yhi, yf);
      if (lane == 0) {
        geo->x0[k] = xf;
        geo->y0[k] = yf;
        geo->dx[k] = x - floorf(x);  // correlation_kernel.cu:262
        geo->dy[k] = y - floorf(y);
      }
    }
  }
  wave_lds_sync();
  // union bounding box of all windows, clipped to the map (wave-uniform values:
  // readfirstlane makes the channel loop below scalar-controlled)
  xlo = wave_uniform(max(xlo - R, 0));
  ylo = wave_uniform(max(ylo - R, 0));
  xhi = wave_uniform(min(xhi + R + 1, W2 - 1));
  yhi = wave_uniform(min(yhi + R + 1, H2 - 1));
  const bool idx_ok = ix >= 0 && ix < N1 && jx >= 0 && jx < N2;
  int bw = xhi - xlo + 1, bh = yhi - ylo + 1;
  if (bw <= 0 || bh <= 0 || !idx_ok) bw = bh = 0;
  const int npx = bw * bh;
  const bool fast = npx <= kBoxPx && np == NPT;

  const size_t HW2 = (size_t)H2 * W2;
  const T* f1 = fmap1 + ((size_t)b * N1 + (idx_ok ? ix : 0)) * C * np;
  const T* f2 = fmap2 + ((size_t)b * N2 + (idx_ok ? jx : 0)) * C * HW2;

  if (fast) {
    // ---- G[k][p] = sum_c f1[c][k] f2[c][p], lane owns p = lane, lane + 64 ----
    // Branch-free: every lane loads from a valid address and masks the value;
    // f1 rows are wave-uniform (scalar loads into SGPR operands of v_fma);
    // the next 4-channel chunk of f2 is in flight while this one is consumed.
    const int p0 = lane, p1 = lane + kWave;
    const bool v0 = p0 < npx, v1 = p1 < npx;
    const int r0 = v0 ? p0 / bw : 0, r1 = v1 ? p1 / bw : 0;
    const size_t o0 = v0 ? (size_t)(ylo + r0) * W2 + xlo + (p0 - r0 * bw) : 0;
    const size_t o1 = v1 ? (size_t)(ylo + r1) * W2 + xlo + (p1 - r1 * bw) : 0;
    const T* fa = f2 + o0;
    const T* fb = f2 + o1;
    A acc0[NPT], acc1[NPT];
#pragma unroll
    for (int k = 0; k < NPT; k++) acc0[k] = acc1[k] = A(0);
    constexpr int CH = 4;
    const int Cv = npx > 0 ? (C / CH) * CH : 0;
    A na[CH], nb[CH];
    if (Cv > 0) {
#pragma unroll
      for (int j = 0; j < CH; j++) {
        na[j] = to_acc(fa[j * HW2]);
        nb[j] = to_acc(fb[j * HW2]);
      }
    }
    for (int c0 = 0; c0 < Cv; c0 += CH) {
      A a[CH], bq[CH];
#pragma unroll
      for (int j = 0; j < CH; j++) {
        a[j] = v0 ? na[j] : A(0);
        bq[j] = v1 ? nb[j] : A(0);
      }
      if (c0 + CH < Cv) {
#pragma unroll
        for (int j = 0; j < CH; j++) {
          na[j] = to_acc(fa[(c0 + CH + j) * HW2]);
          nb[j] = to_acc(fb[(c0 + CH + j) * HW2]);
        }
      }
      const T* w = f1 + (size_t)c0 * NPT;
#pragma unroll
      for (int j = 0; j < CH; j++)
#pragma unroll
        for (int k = 0; k < NPT; k++) {
          const A wk = to_acc(w[j * NPT + k]);
          acc0[k] += wk * a[j];
          acc1[k] += wk * bq[j];
        }
    }
    for (int c = Cv; npx > 0 && c < C; c++) {  // channel tail (C % 4)
      const A a = v0 ? to_acc(fa[c * HW2]) : A(0);
      const A bq = v1 ? to_acc(fb[c * HW2]) : A(0);
#pragma unroll
      for (int k = 0; k < NPT; k++) {
        const A wk = to_acc(f1[(size_t)c * NPT + k]);
        acc0[k] += wk * a;
        acc1[k] += wk * bq;
      }
    }
#pragma unroll
    for (int k = 0; k < NPT; k++) {
      slab[k * kBoxPx + p0] = acc0[k];
      slab[k * kBoxPx + p1] = acc1[k];
    }
  } else {
    // ---- rare: windows too spread for the box; raw[k][yy][xx] directly ----
    const int nraw = np * D * D;
    for (int e = lane; e < nraw; e += kWave) {
      const int k = e / (D * D), t = e % (D * D), yy = t / D, xx = t % D;
      const int i1 = geo->y0[k] + yy - R, j1 = geo->x0[k] + xx - R;
      A s = A(0);
      if (idx_ok && i1 >= 0 && i1 < H2 && j1 >= 0 && j1 < W2) {
        for (int c = 0; c < C; c++)
          s += to_acc(f1[c * np + k]) * to_acc(f2[c * HW2 + (size_t)i1 * W2 + j1]);
      }
      slab[e] = s;
    }
  }
  wave_lds_sync();

  // ---- bilinear + permute, fused into the store (correlation_kernel.cu:260-271) ----
  const int total = Dp * Dp * np;
  const size_t ebase = ((size_t)b * M + m) * total;
  for (int o = lane; o < total; o += kWave) {
    const int k = o % np, t = o / np, yy = t % Dp, xx = t / Dp;
    A r00, r01, r10, r11;
    if (fast) {
      const int gy = geo->y0[k] + yy - R - ylo, gx = geo->x0[k] + xx - R - xlo;
      const A* g = slab + k * kBoxPx;
      auto at = [&](int y, int x) -> A {
        return (y >= 0 && y < bh && x >= 0 && x < bw) ? g[y * bw + x] : A(0);
      };
      r00 = at(gy, gx);
      r01 = at(gy, gx + 1);
      r10 = at(gy + 1, gx);
      r11 = at(gy + 1, gx + 1);
    } else {
      const A* g = slab + k * D * D;
      r00 = g[yy * D + xx];
      r01 = g[yy * D + xx + 1];
      r10 = g[(yy + 1) * D + xx];
      r11 = g[(yy + 1) * D + xx + 1];
    }
    const A dx = geo->dx[k], dy = geo->dy[k];  // dx.to(fmap dtype) (cu:262-263)
    A v = ((A(1) - dx) * (A(1) - dy)) * r00;
    v = v + (dx * (A(1) - dy)) * r01;
    v = v + ((A(1) - dx) * dy) * r10;
    v = v + (dx * dy) * r11;
    if (out_t)
      out_t[ebase + o] = (T)v;
    else
      out_f[(ebase + o) * out_stride + out_off] = (float)v;
  }
  wave_lds_sync();  // slab is reused by this wave only; keep reads before any later reuse
}

template <typename T, int NPT>
__global__ void __launch_bounds__(kCorrWaves* kWave)
    corr_fwd_kernel(const T* __restrict__ fmap1, const T* __restrict__ fmap2,
                    const float* __restrict__ coords, const int64_t* __restrict__ ii,
                    const int64_t* __restrict__ jj, int B, int M, int C, int np, int N1, int N2,
                    int H2, int W2, int R, T* __restrict__ out) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int D = 2 * R + 2;
  const int slab_floats = max(NPT * kBoxPx, NPT * D * D);
  const int wid = wave_uniform(threadIdx.x / kWave);
  using A = typename Acc<T>::type;
  A* slab = reinterpret_cast<A*>(smem) + wid * slab_floats;
  CorrGeom<NPT>* geo =
      reinterpret_cast<CorrGeom<NPT>*>(reinterpret_cast<A*>(smem) + kCorrWaves * slab_floats) + wid;
  const int unit = blockIdx.x * kCorrWaves + wid;
  if (unit >= B * M) return;  // waves are independent: no block barrier in corr_edge
  const int b = unit / M, m = unit % M;
  const int ix = wave_uniform((int)ii[m]), jx = wave_uniform((int)jj[m]);
  corr_edge<T, NPT>(fmap1, fmap2, coords, b, m, ix, jx, M, C, np, N1, N2, H2, W2, R, 1.f, false,
                    slab, geo, out, nullptr, 1, 0);
}

template <typename T, int NPT>
__global__ void __launch_bounds__(kCorrWaves* kWave)
    corr_fwd_levels_kernel(const T* __restrict__ fmap1, CorrLevels lv, int L,
                           const float* __restrict__ coords, const int64_t* __restrict__ ii,
                           const int64_t* __restrict__ jj, int B, int M, int C, int np, int N1,
                           int N2, int R, float* __restrict__ out) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int D = 2 * R + 2;
  const int slab_floats = max(NPT * kBoxPx, NPT * D * D);
  const int wid = wave_uniform(threadIdx.x / kWave);
  using A = typename Acc<T>::type;
  A* slab = reinterpret_cast<A*>(smem) + wid * slab_floats;
  CorrGeom<NPT>* geo =
      reinterpret_cast<CorrGeom<NPT>*>(reinterpret_cast<A*>(smem) + kCorrWaves * slab_floats) + wid;
  const int l = blockIdx.y;
  const int unit = blockIdx.x * kCorrWaves + wid;
  if (unit >= B * M) return;
  const int b = unit / M, m = unit % M;
  const int ix = wave_uniform((int)ii[m]), jx = wave_uniform((int)jj[m]);
  const CorrLevel& c = lv.lv[l];
  corr_edge<T, NPT>(fmap1, reinterpret_cast<const T*>(c.f2), coords, b, m, ix, jx, M, C, np, N1,
                    N2, c.H2, c.W2, R, c.scale, true, slab, geo, nullptr, out, L, l);
}

template <int NPT, typename A = float>
static size_t corr_smem_bytes(int R) {
  const int D = 2 * R + 2;
  const int slab = NPT * kBoxPx > NPT * D * D ? NPT * kBoxPx : NPT * D * D;
  return sizeof(A) * kCorrWaves * slab + sizeof(CorrGeom<NPT>) * kCorrWaves;
}

template <typename T>
static int launch_corr_fwd(const void* fmap1, const void* fmap2, const float* coords,
                           const int64_t* ii, const int64_t* jj, int B, int M, int C, int np,
                           int N1, int N2, int H2, int W2, int R, void* out, hipStream_t s) {
  const dim3 grid((B * M + kCorrWaves - 1) / kCorrWaves), block(kCorrWaves * kWave);
#define DPVO_CORR_CASE(NPT)                                                                    \
  if (np <= NPT) {                                                                             \
    hipLaunchKernelGGL((corr_fwd_kernel<T, NPT>), grid, block,                                 \
                       (corr_smem_bytes<NPT, typename Acc<T>::type>(R)), s,                    \
                       (const T*)fmap1, (const T*)fmap2, coords, ii, jj, B, M, C, np, N1, N2,  \
                       H2, W2, R, (T*)out);                                                    \
    return launch_status();                                                                    \
  }
  DPVO_CORR_CASE(1)
  DPVO_CORR_CASE(4)
  DPVO_CORR_CASE(9)
  DPVO_CORR_CASE(16)
#undef DPVO_CORR_CASE
  return DPVO_ERR_UNSUPPORTED;
}

template <typename T>
static int launch_corr_fwd_levels(const void* fmap1, const CorrLevels& lv, int L,
                                  const float* coords, const int64_t* ii, const int64_t* jj,
                                  int B, int M, int C, int np, int N1, int N2, int R, float* out,
                                  hipStream_t s) {
  const dim3 grid((B * M + kCorrWaves - 1) / kCorrWaves, L), block(kCorrWaves * kWave);
#define DPVO_CORR_CASE(NPT)                                                                       \
  if (np <= NPT) {                                                                                \
    hipLaunchKernelGGL((corr_fwd_levels_kernel<T, NPT>), grid, block,                            \
                       (corr_smem_bytes<NPT, typename Acc<T>::type>(R)), s,                       \
                       (const T*)fmap1, lv, L, coords, ii, jj, B, M, C, np, N1, N2, R, out);      \
    return launch_status();                                                                       \
  }
  DPVO_CORR_CASE(1)
  DPVO_CORR_CASE(4)
  DPVO_CORR_CASE(9)
  DPVO_CORR_CASE(16)
#undef DPVO_CORR_CASE
  return DPVO_ERR_UNSUPPORTED;
}

// ---------------------------------------------------------------------------
// A-CORR-BWD (correlation_kernel.cu:178-229, 275-325).  One wave per edge:
// the bilinear transpose of grad is scattered into the edge's bounding box
// Gb[k][px] in LDS; fmap2_grad gets one atomic per (channel, box pixel)
// (pre-summed over the p*p patch pixels), fmap1_grad one per (channel, k)
// after a wave reduction.  Windows too spread for the box fall back to the
// reference's per-entry atomics.
// ---------------------------------------------------------------------------
template <typename T, int NPT>
__global__ void __launch_bounds__(kCorrWaves* kWave)
    corr_bwd_kernel(const T* __restrict__ fmap1, const T* __restrict__ fmap2,
                    const float* __restrict__ coords, const int64_t* __restrict__ ii,
                    const int64_t* __restrict__ jj, const float* __restrict__ grad, int B, int M,
                    int C, int np, int N1, int N2, int H2, int W2, int R, float* __restrict__ g1,
                    float* __restrict__ g2) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int D = 2 * R + 2, Dp = D - 1;
  const int slab_floats = max(NPT * kBoxPx, NPT * D * D);
  const int wid = wave_uniform(threadIdx.x / kWave);
  const int lane = threadIdx.x & (kWave - 1);
  float* slab = smem + wid * slab_floats;
  CorrGeom<NPT>* geo =
      reinterpret_cast<CorrGeom<NPT>*>(smem + kCorrWaves * slab_floats) + wid;
  const int unit = blockIdx.x * kCorrWaves + wid;
  if (unit >= B * M) return;  // no block-level barrier below
  const int b = unit / M, m = unit % M;
  const int ix = wave_uniform((int)ii[m]), jx = wave_uniform((int)jj[m]);
  if (ix < 0 || ix >= N1 || jx < 0 || jx >= N2) return;

  float cv = lane < 2 * np ? coords[((size_t)b * M + m) * 2 * np + lane] : 0.f;
  int xlo = 0x7fffffff, xhi = -0x7fffffff, ylo = 0x7fffffff, yhi = -0x7fffffff;
#pragma unroll
  for (int k = 0; k < NPT; k++) {
    if (k < np) {
      const float x = __shfl(cv, k, kWave), y = __shfl(cv, np + k, kWave);
      const int xf = ifloor_safe(x), yf = ifloor_safe(y);
      xlo = min(xlo, xf); xhi = max(xhi, xf); ylo = min(ylo, yf); yhi = max(yhi, yf);
      if (lane == 0) {
        geo->x0[k] = xf; geo->y0[k] = yf;
        geo->dx[k] = x - floorf(x); geo->dy[k] = y - floorf(y);
      }
    }
  }
  xlo = max(xlo - R, 0); ylo = max(ylo - R, 0);
  xhi = min(xhi + R + 1, W2 - 1); yhi = min(yhi + R + 1, H2 - 1);
  int bw = xhi - xlo + 1, bh = yhi - ylo + 1;
  if (bw <= 0 || bh <= 0) return;  // every window outside the map: no gradient
  const int npx = bw * bh;
  const size_t HW2 = (size_t)H2 * W2;
  const T* f1 = fmap1 + ((size_t)b * N1 + ix) * C * np;
  const T* f2 = fmap2 + ((size_t)b * N2 + jx) * C * HW2;
  float* G1 = g1 + ((size_t)b * N1 + ix) * C * np;
  float* G2 = g2 + ((size_t)b * N2 + jx) * C * HW2;
  const float* gr = grad + ((size_t)b * M + m) * Dp * Dp * np;  // [xx][yy][k]
  wave_lds_sync();

  // corr_grad[k][yy][xx] = g1 + g2 + g3 + g4 (correlation_kernel.cu:303-308)
  auto cg_at = [&](int k, int yy, int xx) -> float {
    const float dx = geo->dx[k], dy = geo->dy[k];
    auto G = [&](int a, int c) { return gr[(c * Dp + a) * np + k]; };
    float t1 = 0.f, t2 = 0.f, t3 = 0.f, t4 = 0.f;
    if (yy < Dp && xx < Dp) t1 = ((1.0f - dx) * (1.0f - dy)) * G(yy, xx);
    if (yy < Dp && xx >= 1) t2 = (dx * (1.0f - dy)) * G(yy, xx - 1);
    if (yy >= 1 && xx < Dp) t3 = ((1.0f - dx) * dy) * G(yy - 1, xx);
    if (yy >= 1 && xx >= 1) t4 = (dx * dy) * G(yy - 1, xx - 1);
    return ((t1 + t2) + t3) + t4;
  };

  if (npx <= kBoxPx) {
    for (int e = lane; e < NPT * kBoxPx; e += kWave) slab[e] = 0.f;
    wave_lds_sync();
    for (int e = lane; e < np * D * D; e += kWave) {
      const int k = e / (D * D), t = e % (D * D), yy = t / D, xx = t % D;
      const int gy = geo->y0[k] + yy - R - ylo, gx = geo->x0[k] + xx - R - xlo;
      if (gy >= 0 && gy < bh && gx >= 0 && gx < bw) slab[k * kBoxPx + gy * bw + gx] = cg_at(k, yy, xx);
    }
    wave_lds_sync();
    const int p0 = lane, p1 = lane + kWave;
    const bool v0 = p0 < npx, v1 = p1 < npx;
    const int r0 = v0 ? p0 / bw : 0, r1 = v1 ? p1 / bw : 0;
    const size_t o0 = (size_t)(ylo + r0) * W2 + xlo + (p0 - r0 * bw);
    const size_t o1 = (size_t)(ylo + r1) * W2 + xlo + (p1 - r1 * bw);
    float q0[NPT], q1[NPT];
    bool any0 = false, any1 = false;
#pragma unroll
    for (int k = 0; k < NPT; k++) {
      q0[k] = k < np ? slab[k * kBoxPx + p0] : 0.f;
      q1[k] = k < np ? slab[k * kBoxPx + p1] : 0.f;
      any0 |= q0[k] != 0.f;
      any1 |= q1[k] != 0.f;
    }
    for (int c = 0; c < C; c++) {
      float s0 = 0.f, s1 = 0.f;
#pragma unroll
      for (int k = 0; k < NPT; k++) {
        if (k < np) {
          const float w = to_acc(f1[c * np + k]);
          s0 += q0[k] * w;
          s1 += q1[k] * w;
        }
      }
      if (v0 && any0) atomicAdd(G2 + c * HW2 + o0, s0);
      if (v1 && any1) atomicAdd(G2 + c * HW2 + o1, s1);
      const float a0 = v0 ? to_acc(f2[c * HW2 + o0]) : 0.f;
      const float a1 = v1 ? to_acc(f2[c * HW2 + o1]) : 0.f;
#pragma unroll
      for (int k = 0; k < NPT; k++) {
        if (k < np) {
          const float t = wave_sum(q0[k] * a0 + q1[k] * a1);
          if (lane == 0) atomicAdd(G1 + c * np + k, t);
        }
      }
    }
  } else {
    for (int e = lane; e < np * D * D; e += kWave) {
      const int k = e / (D * D), t = e % (D * D), yy = t / D, xx = t % D;
      const int i1 = geo->y0[k] + yy - R, j1 = geo->x0[k] + xx - R;
      if (i1 < 0 || i1 >= H2 || j1 < 0 || j1 >= W2) continue;
      const float g = cg_at(k, yy, xx);
      for (int c = 0; c < C; c++) {
        atomicAdd(G1 + c * np + k, g * to_acc(f2[c * HW2 + (size_t)i1 * W2 + j1]));
        atomicAdd(G2 + c * HW2 + (size_t)i1 * W2 + j1, g * to_acc(f1[c * np + k]));
      }
    }
  }
}

template <typename T>
__global__ void cast_from_f32_kernel(const float* __restrict__ in, T* __restrict__ out, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n;
       i += (size_t)gridDim.x * blockDim.x)
    out[i] = from_acc<T>(in[i]);
}

// ---------------------------------------------------------------------------
// A-PATCH / A-PATCH-BWD (correlation_kernel.cu:16-80): gather / scatter of a
// (2R+2)^2 window per patch centre; one thread per output element, stores
// in output order (coalesced).
// ---------------------------------------------------------------------------
template <typename T>
__global__ void patchify_fwd_kernel(const T* __restrict__ net, const float* __restrict__ coords,
                                    int B, int C, int H, int W, int M, int R, int clamp,
                                    T* __restrict__ out) {
  const int D = 2 * R + 2;
  const size_t total = (size_t)B * M * C * D * D;
  for (size_t n = blockIdx.x * (size_t)blockDim.x + threadIdx.x; n < total;
       n += (size_t)gridDim.x * blockDim.x) {
    size_t t = n;
    const int xx = t % D; t /= D;
    const int yy = t % D; t /= D;
    const int c = t % C; t /= C;
    const int m = t % M;
    const int b = t / M;
    const float x = coords[((size_t)b * M + m) * 2 + 0];
    const float y = coords[((size_t)b * M + m) * 2 + 1];
    int i = ifloor_safe(y) + (yy - R), j = ifloor_safe(x) + (xx - R);
    T v = from_acc<T>(0.f);
    if (clamp) {
      i = min(max(i, 0), H - 1);
      j = min(max(j, 0), W - 1);
      v = net[(((size_t)b * C + c) * H + i) * W + j];
    } else if (i >= 0 && i < H && j >= 0 && j < W) {
      v = net[(((size_t)b * C + c) * H + i) * W + j];
    }
    out[n] = v;
  }
}

template <typename T>
__global__ void patchify_bwd_kernel(const T* __restrict__ grad, const float* __restrict__ coords,
                                    int B, int C, int H, int W, int M, int R, int clamp,
                                    float* __restrict__ net_grad) {
  const int D = 2 * R + 2;
  const size_t total = (size_t)B * M * C * D * D;
  for (size_t n = blockIdx.x * (size_t)blockDim.x + threadIdx.x; n < total;
       n += (size_t)gridDim.x * blockDim.x) {
    size_t t = n;
    const int xx = t % D; t /= D;
    const int yy = t % D; t /= D;
    const int c = t % C; t /= C;
    const int m = t % M;
    const int b = t / M;
    const float x = coords[((size_t)b * M + m) * 2 + 0];
    const float y = coords[((size_t)b * M + m) * 2 + 1];
    int i = ifloor_safe(y) + (yy - R), j = ifloor_safe(x) + (xx - R);
    if (clamp) {
      i = min(max(i, 0), H - 1);
      j = min(max(j, 0), W - 1);
    } else if (!(i >= 0 && i < H && j >= 0 && j < W)) {
      continue;
    }
    atomicAdd(net_grad + (((size_t)b * C + c) * H + i) * W + j, to_acc(grad[n]));
  }
}

static inline unsigned grid_for(size_t n, int block = 256) {
  size_t g = (n + block - 1) / block;
  if (g > 65536) g = 65536;
  return (unsigned)(g ? g : 1);
}

}  // namespace dpvo

using namespace dpvo;

DPVO_EXPORT int dpvo_corr_forward(const void* fmap1, const void* fmap2, const float* coords,
                                  const int64_t* ii, const int64_t* jj, int B, int M, int C, int H,
                                  int W, int N1, int N2, int H2, int W2, int radius, int dtype,
                                  void* out, void* stream) {
  if (B < 0 || M < 0 || C <= 0 || H <= 0 || W <= 0 || radius < 0 || radius > 7 || H2 <= 0 ||
      W2 <= 0)
    return DPVO_ERR_INVALID;
  if (H * W > 16) return DPVO_ERR_UNSUPPORTED;
  if (B * M == 0) return DPVO_OK;
  if (!fmap1 || !fmap2 || !coords || !ii || !jj || !out) return DPVO_ERR_INVALID;
  hipStream_t s = as_stream(stream);
  const int np = H * W;
  if (dtype == DPVO_F16 || dtype == DPVO_F32) {
    const int st = corr_nchw_mma(fmap1, &fmap2, &H2, &W2, nullptr, 1, false, coords, ii, jj, B,
                                 M, C, np, N1, N2, radius, dtype, out, nullptr, s);
    if (st != DPVO_ERR_UNSUPPORTED) return st;
  }
  switch (dtype) {
    case DPVO_F32:
      return launch_corr_fwd<float>(fmap1, fmap2, coords, ii, jj, B, M, C, np, N1, N2, H2, W2,
                                    radius, out, s);
    case DPVO_F16:
      return launch_corr_fwd<__half>(fmap1, fmap2, coords, ii, jj, B, M, C, np, N1, N2, H2, W2,
                                     radius, out, s);
    case DPVO_F64:
      return launch_corr_fwd<double>(fmap1, fmap2, coords, ii, jj, B, M, C, np, N1, N2, H2, W2,
                                     radius, out, s);
  }
  return DPVO_ERR_INVALID;
}

DPVO_EXPORT int dpvo_corr_forward_levels(const void* fmap1, const void* const* fmap2,
                                         const int* H2, const int* W2, const float* scale, int L,
                                         const float* coords, const int64_t* ii,
                                         const int64_t* jj, int B, int M, int C, int H, int W,
                                         int N1, int N2, int radius, int dtype, float* out,
                                         void* stream) {
  if (L <= 0 || L > 8 || radius < 0 || radius > 7 || C <= 0 || H <= 0 || W <= 0)
    return DPVO_ERR_INVALID;
  if (H * W > 16) return DPVO_ERR_UNSUPPORTED;
  if (B * M == 0) return DPVO_OK;
  CorrLevels lv = {};
  for (int l = 0; l < L; l++) {
    if (!fmap2[l] || H2[l] <= 0 || W2[l] <= 0 || !(scale[l] > 0.f)) return DPVO_ERR_INVALID;
    lv.lv[l] = CorrLevel{fmap2[l], H2[l], W2[l], scale[l]};
  }
  hipStream_t s = as_stream(stream);
  const int np = H * W;
  if (dtype == DPVO_F16 || dtype == DPVO_F32) {
    const int st = corr_nchw_mma(fmap1, fmap2, H2, W2, scale, L, true, coords, ii, jj, B, M, C,
                                 np, N1, N2, radius, dtype, nullptr, out, s);
    if (st != DPVO_ERR_UNSUPPORTED) return st;
  }
  switch (dtype) {
    case DPVO_F32:
      return launch_corr_fwd_levels<float>(fmap1, lv, L, coords, ii, jj, B, M, C, np, N1, N2,
                                           radius, out, s);
    case DPVO_F16:
      return launch_corr_fwd_levels<__half>(fmap1, lv, L, coords, ii, jj, B, M, C, np, N1, N2,
                                            radius, out, s);
  }
  return DPVO_ERR_UNSUPPORTED;
}

DPVO_EXPORT int dpvo_corr_backward(const void* fmap1, const void* fmap2, const float* coords,
                                   const int64_t* ii, const int64_t* jj, const float* grad, int B,
                                   int M, int C, int H, int W, int N1, int N2, int H2, int W2,
                                   int radius, int dtype, void* fmap1_grad, void* fmap2_grad,
                                   void* stream) {
  if (B < 0 || M < 0 || C <= 0 || H <= 0 || W <= 0 || radius < 0 || radius > 7)
    return DPVO_ERR_INVALID;
  if (H * W > 16) return DPVO_ERR_UNSUPPORTED;
  if (dtype != DPVO_F32) return DPVO_ERR_UNSUPPORTED;  // fp32 atomics (training path)
  hipStream_t s = as_stream(stream);
  const size_t n1 = (size_t)B * N1 * C * H * W, n2 = (size_t)B * N2 * C * H2 * W2;
  if (hipMemsetAsync(fmap1_grad, 0, n1 * sizeof(float), s) != hipSuccess ||
      hipMemsetAsync(fmap2_grad, 0, n2 * sizeof(float), s) != hipSuccess)
    return DPVO_ERR_LAUNCH;
  if (B * M == 0) return DPVO_OK;
  const int np = H * W;
  const dim3 grid((B * M + kCorrWaves - 1) / kCorrWaves), block(kCorrWaves * kWave);
#define DPVO_BWD_CASE(NPT)                                                                     \
  if (np <= NPT) {                                                                             \
    hipLaunchKernelGGL((corr_bwd_kernel<float, NPT>), grid, block, corr_smem_bytes<NPT>(radius), \
                       s, (const float*)fmap1, (const float*)fmap2, coords, ii, jj, grad, B, M, C, \
                       np, N1, N2, H2, W2, radius, (float*)fmap1_grad, (float*)fmap2_grad);    \
    return launch_status();                                                                    \
  }
  DPVO_BWD_CASE(1)
  DPVO_BWD_CASE(4)
  DPVO_BWD_CASE(9)
  DPVO_BWD_CASE(16)
#undef DPVO_BWD_CASE
  return DPVO_ERR_UNSUPPORTED;
}

DPVO_EXPORT int dpvo_patchify_forward(const void* net, const float* coords, int B, int C, int H,
                                      int W, int M, int radius, int clamp, int dtype, void* out,
                                      void* stream) {
  if (B < 0 || M < 0 || C <= 0 || H <= 0 || W <= 0 || radius < 0) return DPVO_ERR_INVALID;
  const int D = 2 * radius + 2;
  const size_t total = (size_t)B * M * C * D * D;
  if (total == 0) return DPVO_OK;
  hipStream_t s = as_stream(stream);
  switch (dtype) {
    case DPVO_F32:
      hipLaunchKernelGGL(patchify_fwd_kernel<float>, dim3(grid_for(total)), dim3(256), 0, s,
                         (const float*)net, coords, B, C, H, W, M, radius, clamp, (float*)out);
      return launch_status();
    case DPVO_F16:
      hipLaunchKernelGGL(patchify_fwd_kernel<__half>, dim3(grid_for(total)), dim3(256), 0, s,
                         (const __half*)net, coords, B, C, H, W, M, radius, clamp, (__half*)out);
      return launch_status();
    case DPVO_F64:
      hipLaunchKernelGGL(patchify_fwd_kernel<double>, dim3(grid_for(total)), dim3(256), 0, s,
                         (const double*)net, coords, B, C, H, W, M, radius, clamp, (double*)out);
      return launch_status();
  }
  return DPVO_ERR_INVALID;
}

DPVO_EXPORT int dpvo_patchify_backward(const void* grad, const float* coords, int B, int C, int H,
                                       int W, int M, int radius, int clamp, int dtype,
                                       void* net_grad, void* stream) {
  if (B < 0 || M < 0 || C <= 0 || H <= 0 || W <= 0 || radius < 0) return DPVO_ERR_INVALID;
  if (dtype != DPVO_F32) return DPVO_ERR_UNSUPPORTED;
  hipStream_t s = as_stream(stream);
  if (hipMemsetAsync(net_grad, 0, (size_t)B * C * H * W * sizeof(float), s) != hipSuccess)
    return DPVO_ERR_LAUNCH;
  const int D = 2 * radius + 2;
  const size_t total = (size_t)B * M * C * D * D;
  if (total == 0) return DPVO_OK;
  hipLaunchKernelGGL(patchify_bwd_kernel<float>, dim3(grid_for(total)), dim3(256), 0, s,
                     (const float*)grad, coords, B, C, H, W, M, radius, clamp, (float*)net_grad);
  return launch_status();
}
