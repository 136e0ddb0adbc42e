// corr_nhwc.hip -- A-CORR on gfx950 for channels-last feature pyramids.
//
// Same semantics as corr.hip / correlation_kernel.cu:82-175 + 232-272
// (raw window dot products over C channels, 0 outside the map, bilinear with
// frac(x), frac(y), output permuted to [b, m, xx, yy, i0, j0] and the levels
// stacked on the last axis, dpvo.py:462-465), for fmap2 levels stored
// [B, N2, H, W, C] (channels-last; DESIGN.md "A-CORR: layout").
//
// Why: with channel-major planes a window row is ~10 contiguous floats, so
// every fmap2 load touches a partial 128-B line; channels-last makes each
// window row one contiguous run of (width x C x 4) bytes.  The per-edge GEMM
//     G[k][px] = sum_c f1[c][k] * f2[px][c]     (k < p*p, px in the union
// bounding box of the edge's windows) runs on the matrix cores, then the
// bilinear + permute reads the windows out of G.  One kernel,
// corr_nhwc_lvl_kernel: one wave per (edge, level) unit, whole-line tile
// loads through an LDS stage; fp32 features with exact fp32 products
// (v_mfma_f32_16x16x4_f32), fp16 features (the fork's MIXED_PRECISION rings)
// on v_mfma_f32_16x16x32_f16, fp32 accumulation in both.
#include <type_traits>

#include "common.hpp"
#include "pyr_insert.hpp"


namespace dpvo {

constexpr int kNhwcC = 128;     // channels (DPVO gmap / fmap width)
constexpr int kMaxL = 4;        // levels per launch
constexpr int kOutPerLane = 8;  // (2R+1)^2 * p*p <= 512 outputs per level
constexpr int kNpMax = 16;      // p*p <= 16 (one MFMA row tile)

struct NhwcLevels {
  const void* f2[kMaxL];  // float or __half, [B, N2, H, W, C]
  int H2[kMaxL], W2[kMaxL];
  float scale[kMaxL];
};

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
// 16-B tile vector (a native vector: a uint4 struct copy is a memcpy that
// keeps the ring in scratch)
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
// global-address-space view of a tile vector: a generic pointer would make
// every tile load a flat load, which counts in both vmcnt and lgkmcnt and
// makes the wait before each tile drain the whole ring
typedef const __attribute__((address_space(1))) u32x4 gu32x4;

// wave-uniform per-level parameter without a dynamic index into the kernel
// argument struct (that would route every access through scratch / flat
// loads, which count in vmcnt and force full drains in the tile loop)
template <typename X>
__device__ __forceinline__ X sel4(int l, X a, X b, X c, X d) {
  return l == 0 ? a : l == 1 ? b : l == 2 ? c : d;
}
#define LV_SEL(field, l) sel4((l), lv.field[0], lv.field[1], lv.field[2], lv.field[3])

// ---------------------------------------------------------------------------
// corr_nhwc_lvl_kernel: one wave per (edge, pyramid level) unit; fp32
// features with exact fp32 products (v_mfma_f32_16x16x4_f32), fp16 features
// on v_mfma_f32_16x16x32_f16 (a tile line is 64 channels: 2 MFMAs).
//
// What bounds A-CORR is the vector-memory path, not the matrix cores: the
// loads alone of round 5's per-edge kernel's B layout (16 box pixels x 64 B per
// global_load_dwordx4 = 16 half-used 128-B lines per KiB) take 46.6 us at
// cfg2, the same bytes as whole lines (8 pixels x 128 B per instruction)
// 28.0 us (scripts/micro/load_pattern.hip).  So the box tiles are loaded as
// whole lines and turned into the MFMA B layout through a 2-KiB LDS stage per
// wave (one 128-B line of the tile's 16 pixels at a time, XOR-swizzled
// so both the stage writes and the B-fragment reads are conflict-free).
// Units: one wave per (edge, level) (8192 at cfg2) puts 4 waves on a SIMD
// instead of the per-edge kernel's 2; every wave runs TWO units, level l of
// edge A and level L-1-l of edge B (the fine and the coarse levels pair up:
// 7 + 4 and 6 + 5 tiles at cfg2), so the whole grid is resident at once
// (4096 waves on 1024 SIMDs) with no second-round tail.  The waves are
// independent (no barrier); each builds its unit's A fragments (the gmap
// patch, 32 registers) and writes its level's slice of the edge's [nout][L]
// output block.
// ---------------------------------------------------------------------------
constexpr int kLvlMaxTiles = 10;                   // box up to 160 pixels on the matrix path
constexpr int kLvlBoxStride = 16 * kLvlMaxTiles + 4;
constexpr int kLvlStage = 16 * 128;                // bytes: 16 pixels x one 128-B line

struct LvlGeom {
  int x0[kNpMax], y0[kNpMax];
  float dx[kNpMax], dy[kNpMax];
};
// per wave: G [np][kLvlBoxStride] floats, the stage, the geometry, the
// first unit's output slice (nout floats; the second unit's stays in the stage)
__host__ __device__ inline int corr_lvl_out_bytes(int np, int R) {
  return ((2 * R + 1) * (2 * R + 1) * np * (int)sizeof(float) + 15) & ~15;
}
// edge positions per workgroup: its npos x L waves hold the (edge, level)
// units, one or two per wave (pairs: L >= 3, where one unit per wave would
// not leave the whole grid resident at DPVO sizes)
__host__ __device__ inline bool corr_lvl_paired(int L) { return L >= 3; }
__host__ __device__ inline int corr_lvl_npos(int L) { return L >= 3 ? 1 : kMaxL / L; }
__host__ __device__ inline int corr_lvl_wave_bytes(int np, int R) {
  return (int)(sizeof(float) * np * kLvlBoxStride + kLvlStage + sizeof(LvlGeom)) +
         corr_lvl_out_bytes(np, R);
}

// RAW9: p = 3, R = 3 (DPVO) as compile-time constants; otherwise run-time np, R
// T = float: exact fp32 products (v_mfma_f32_16x16x4_f32); T = __half (the
// fork's MIXED_PRECISION rings): f16 x f16 on v_mfma_f32_16x16x32_f16, fp32
// accumulation (documented deviation: the reference accumulates in fp16)
template <typename T, int RING, bool RAW9, bool PAIRED>
__global__ void __launch_bounds__(kMaxL* kWave) __attribute__((amdgpu_waves_per_eu(RING > 2 ? 3 : 4)))
    corr_nhwc_lvl_kernel(const T* __restrict__ fmap1, NhwcLevels lv, int L,
                         const float* __restrict__ coords, const int64_t* __restrict__ ii,
                         const int64_t* __restrict__ jj, int B, int M, int np_, int N1, int N2,
                         int R_, const int* __restrict__ order, float* __restrict__ out) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int np = RAW9 ? 9 : np_, R = RAW9 ? 3 : R_;
  const int w = wave_uniform(threadIdx.x / kWave), lane = threadIdx.x & (kWave - 1);
  const int C = kNhwcC, D = 2 * R + 2, Dp = D - 1, nout = Dp * Dp * np;
  const int wbytes = corr_lvl_wave_bytes(np, R);
  char* wl = reinterpret_cast<char*>(smem) + (size_t)w * wbytes;
  float* G = reinterpret_cast<float*>(wl);
  char* stage = wl + sizeof(float) * np * kLvlBoxStride;
  LvlGeom* geo = reinterpret_cast<LvlGeom*>(stage + kLvlStage);
  // output slices: unit 0 (level w of edge A) in its own region, unit 1
  // (level L-1-w of edge B) in the stage, stored by the workgroup at the end
  float* outA = reinterpret_cast<float*>(geo + 1);
  const int ai = lane & 15, aq = lane >> 4;

  // edge positions of this workgroup: with an order (B == 1, XCD-aware) XCD
  // x = blockIdx % 8 takes the x-th eighth of the edges grouped by target
  // frame, a workgroup two positions of it half an eighth apart
  const int nE = B * M;
  // paired: a wave runs level l of position q and level L-1-l of position
  // q + half (fine and coarse levels together); otherwise one unit per wave
  constexpr bool paired = PAIRED;  // = corr_lvl_paired(L)
  const int per = order ? (M + 7) / 8 : nE, half = paired ? (per + 1) / 2 : per;
  const int x8 = order ? (int)(blockIdx.x % 8) : 0, j8 = order ? (int)(blockIdx.x / 8) : (int)blockIdx.x;
  const int npair = PAIRED ? 1 : corr_lvl_npos(L);
  if (j8 * npair >= half) return;

  // ---- one (edge position p, level lev) unit
  auto run_unit = [&](int p, int lev, float* so) __attribute__((always_inline)) {
    const int edge = order ? wave_uniform(order[p]) : p;
    const int b = edge / M, m = edge % M;
    const int ix = wave_uniform((int)ii[m]), jx = wave_uniform((int)jj[m]);
    const bool idx_ok = ix >= 0 && ix < N1 && jx >= 0 && jx < N2;

    // the gmap patch [C][np] (whole lines, 16 B per lane), staged through G
    // once the first box tiles are in flight
    constexpr int kE16 = 16 / sizeof(T);  // elements per 16 B
    constexpr int kPA = (kNhwcC * (RAW9 ? 9 : kNpMax) / kE16 + kWave - 1) / kWave;
    const int n16 = C * np / kE16;
    u32x4 pa[kPA];
    {
      const T* f1 = fmap1 + ((size_t)b * N1 + (idx_ok ? ix : 0)) * C * np;
#pragma unroll
      for (int r = 0; r < kPA; r++)
        pa[r] = reinterpret_cast<const u32x4*>(f1)[min(lane + kWave * r, n16 - 1)];
    }
    __builtin_amdgcn_sched_barrier(0);  // the geometry waits for the coordinates only

    // the edge's coordinates: RAW9 by scalar loads (uniform address: the
    // scalar cache, not the vector-memory queue the tile loads keep full)
    float cx = 0.f, cy = 0.f;  // lane k < np: patch pixel k (level-1 pixels)
    if constexpr (RAW9) {
      const float* cp = coords + ((size_t)b * M + m) * 18;
      float c[18];
#pragma unroll
      for (int j = 0; j < 18; j++) c[j] = cp[j];
#pragma unroll
      for (int j = 0; j < 9; j++) {
        cx = (lane == j) ? c[j] : cx;
        cy = (lane == j) ? c[9 + j] : cy;
      }
    } else {
      const float cv = (lane < 2 * np) ? coords[((size_t)b * M + m) * 2 * np + lane] : 0.f;
      cx = __shfl(cv, min(ai, np - 1), kWave);
      cy = __shfl(cv, np + min(ai, np - 1), kWave);
    }

    // geometry of the level: lane k < np takes patch pixel k (floor / frac),
    // row (16-lane) min / max scans by DPP give the box
    const int H2 = LV_SEL(H2, lev), W2 = LV_SEL(W2, lev);
    int xlo, ylo, bw, bh;
    bool inner;  // box not clamped to the map: every tap of every window is in it
    int kb[9];   // RAW9, per patch pixel k (wave-uniform): window origin in G ...
    float w00[9], w01[9], w10[9], w11[9];  // ... and the bilinear weights
    {
      const bool act = lane < np;
      const float sc = LV_SEL(scale, lev);
      const bool pow2 = (__float_as_uint(sc) & 0x7fffffu) == 0u;  // x / 2^k == x * 2^-k
      const float rs = 1.0f / sc;
      const float x = pow2 ? cx * rs : cx / sc, y = pow2 ? cy * rs : cy / sc;
      const int xf = ifloor_safe(x), yf = ifloor_safe(y);
      const float dx = x - floorf(x), dy = y - floorf(y);  // correlation_kernel.cu:262
      if (act) {
        geo->x0[ai] = xf;
        geo->y0[ai] = yf;
        geo->dx[ai] = dx;
        geo->dy[ai] = dy;
      }
      auto rmin = [](int v) {
        v = min(v, __builtin_amdgcn_update_dpp(0x7fffffff, v, 0x111, 0xf, 0xf, false));
        v = min(v, __builtin_amdgcn_update_dpp(0x7fffffff, v, 0x112, 0xf, 0xf, false));
        v = min(v, __builtin_amdgcn_update_dpp(0x7fffffff, v, 0x114, 0xf, 0xf, false));
        v = min(v, __builtin_amdgcn_update_dpp(0x7fffffff, v, 0x118, 0xf, 0xf, false));
        return __builtin_amdgcn_readlane(v, 15);
      };
      const int lo_x = rmin(act ? xf : 0x7fffffff), lo_y = rmin(act ? yf : 0x7fffffff);
      const int hi_x = -rmin(act ? -xf : 0x7fffffff), hi_y = -rmin(act ? -yf : 0x7fffffff);
      xlo = wave_uniform(max(lo_x - R, 0));
      ylo = wave_uniform(max(lo_y - R, 0));
      const int xhi = min(hi_x + R + 1, W2 - 1), yhi = min(hi_y + R + 1, H2 - 1);
      bw = wave_uniform(xhi - xlo + 1);
      bh = wave_uniform(yhi - ylo + 1);
      if (bw <= 0 || bh <= 0 || !idx_ok) bw = bh = 0;
      inner = bw > 0 && lo_x - R >= 0 && lo_y - R >= 0 && hi_x + R + 1 <= W2 - 1 &&
              hi_y + R + 1 <= H2 - 1;
      if constexpr (RAW9) {
        const int kbv = (yf - R - ylo) * bw + (xf - R - xlo);
        const float a00 = (1.f - dx) * (1.f - dy), a01 = dx * (1.f - dy), a10 = (1.f - dx) * dy,
                    a11 = dx * dy;
#pragma unroll
        for (int k = 0; k < 9; k++) {
          kb[k] = __builtin_amdgcn_readlane(kbv, k);
          w00[k] = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(a00), k));
          w01[k] = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(a01), k));
          w10[k] = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(a10), k));
          w11[k] = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(a11), k));
        }
      }
    }
    const int ntile = (bw * bh + 15) >> 4;
    const bool fast = ntile <= kLvlMaxTiles;

    // bilinear + permute from G (correlation_kernel.cu:260-271) into this
    // level's output slice so[nout] in LDS (output order)
    auto tap4 = [&](int k, int yy, int xx, bool mat, float& r00, float& r01, float& r10,
                    float& r11) __attribute__((always_inline)) {
      if (mat) {  // clamped (valid) LDS addresses, zeroed by a select
        const int cap = max(bw * bh - 1, 0);
        const int gy = geo->y0[k] + yy - R - ylo, gx = geo->x0[k] + xx - R - xlo;
        const float* g = G + k * kLvlBoxStride;
        const bool y0i = gy >= 0 && gy < bh, y1i = gy + 1 >= 0 && gy + 1 < bh;
        const bool x0i = gx >= 0 && gx < bw, x1i = gx + 1 >= 0 && gx + 1 < bw;
        const float a00 = g[min(max(gy * bw + gx, 0), cap)];
        const float a01 = g[min(max(gy * bw + gx + 1, 0), cap)];
        const float a10 = g[min(max((gy + 1) * bw + gx, 0), cap)];
        const float a11 = g[min(max((gy + 1) * bw + gx + 1, 0), cap)];
        r00 = (y0i && x0i) ? a00 : 0.f;
        r01 = (y0i && x1i) ? a01 : 0.f;
        r10 = (y1i && x0i) ? a10 : 0.f;
        r11 = (y1i && x1i) ? a11 : 0.f;
      } else {
        const float* g = G + k * D * D;
        r00 = g[yy * D + xx];
        r01 = g[yy * D + xx + 1];
        r10 = g[(yy + 1) * D + xx];
        r11 = g[(yy + 1) * D + xx + 1];
      }
    };
    auto bil = [&](int k, float r00, float r01, float r10, float r11) __attribute__((always_inline)) {
      const float dx = geo->dx[k], dy = geo->dy[k];
      float v = ((1.f - dx) * (1.f - dy)) * r00;
      v = v + (dx * (1.f - dy)) * r01;
      v = v + ((1.f - dx) * dy) * r10;
      v = v + (dx * dy) * r11;
      return v;
    };
    auto bilinear_store = [&](bool mat) __attribute__((always_inline)) {
      if constexpr (RAW9) {
        // lane = output point (xx = lane >> 3, yy = lane & 7), every k: uniform
        // weights, no index division; through the stage into output order
        const int xx = min(lane >> 3, Dp - 1), yy = min(lane & 7, Dp - 1);
        const bool on = (lane >> 3) < Dp && (lane & 7) < Dp;
        float v[9];
        if (mat && inner) {  // every tap in the box: 4 reads at fixed offsets
          const int loff = yy * bw + xx;
#pragma unroll
          for (int k = 0; k < 9; k++) {
            const float* g = G + k * kLvlBoxStride + kb[k] + loff;
            const float r00 = g[0], r01 = g[1], r10 = g[bw], r11 = g[bw + 1];
            float t = w00[k] * r00;
            t = t + w01[k] * r01;
            t = t + w10[k] * r10;
            t = t + w11[k] * r11;
            v[k] = t;
          }
        } else {
#pragma unroll
          for (int k = 0; k < 9; k++) {
            float r00, r01, r10, r11;
            tap4(k, yy, xx, mat, r00, r01, r10, r11);
            v[k] = bil(k, r00, r01, r10, r11);
          }
        }
        if (on) {
#pragma unroll
          for (int k = 0; k < 9; k++) so[(xx * Dp + yy) * 9 + k] = v[k];
        }
      } else {
#pragma unroll
        for (int u = 0; u < kOutPerLane; u++) {
          const int o = lane + kWave * u;
          const int k = min(o % np, np - 1), t = o / np, yy = min(t % Dp, Dp - 1),
                    xx = min(t / Dp, Dp - 1);
          float r00, r01, r10, r11;
          tap4(k, yy, xx, mat, r00, r01, r10, r11);
          const float v = bil(k, r00, r01, r10, r11);
          if (o < nout) so[o] = v;
        }
      }
    };
    wave_lds_sync();  // geo visible
    if (!fast) {
      // windows too spread for the matrix path: raw[k][yy][xx] as fp32 dot
      // products straight from HBM into G, then the bilinear
      const T* f2 = static_cast<const T*>(LV_SEL(f2, lev)) +
                    ((size_t)b * N2 + (idx_ok ? jx : 0)) * H2 * W2 * C;
      const T* f1 = fmap1 + ((size_t)b * N1 + (idx_ok ? ix : 0)) * C * np;
      for (int e = lane; e < np * D * D; e += kWave) {
        const int k = e / (D * D), t = e % (D * D), yy = t / D, xx = t % D;
        const int i1 = geo->y0[k] + yy - R, j1 = geo->x0[k] + xx - R;
        float sacc = 0.f;
        if (idx_ok && i1 >= 0 && i1 < H2 && j1 >= 0 && j1 < W2) {
          const T* px = f2 + ((size_t)i1 * W2 + j1) * C;
          for (int c = 0; c < C; c++) sacc += to_acc(f1[(size_t)c * np + k]) * to_acc(px[c]);
        }
        G[e] = sacc;
      }
      wave_lds_sync();
      bilinear_store(false);
      wave_lds_sync();  // G free
      return;
    }

    // box tiles as whole lines: instruction h of tile t covers pixels
    // 16 t + 8 (h & 1) + (lane >> 3), 128-B line h >> 1, 16 B (lane & 7) each
    const int npx = max(bw * bh, 1), bw1 = max(bw, 1);
    const T* base = static_cast<const T*>(LV_SEL(f2, lev)) +
                        (((size_t)b * N2 + (idx_ok ? jx : 0)) * H2 * W2 +
                         (ntile > 0 ? (size_t)ylo * W2 + xlo : 0)) * C +
                        kE16 * (lane & 7);
    const int rowe = W2 * C;
    const float rbw = 1.0f / (float)bw1;
    // 16-B loads per lane per tile: a tile is 16 pixels x C channels, an
    // instruction 8 pixels x one 128-B line
    constexpr int V = (int)(kNhwcC * sizeof(T)) / 64;
    const T* base0 = static_cast<const T*>(LV_SEL(f2, lev));
    auto load_tile = [&](u32x4 (&d)[V], int t) __attribute__((always_inline)) {
      // past the end (ring refills, never used): every lane reads the same 16 B,
      // one line request per instruction instead of eight
      const bool past = t >= ntile;
      const T* s[2];
#pragma unroll
      for (int ph = 0; ph < 2; ph++) {
        const int px = min(16 * t + 8 * ph + (lane >> 3), npx - 1);  // pad lanes: pixel npx - 1
        const int r = (int)(((float)px + 0.5f) * rbw), cc = px - r * bw1;
        s[ph] = past ? base0 : base + r * rowe + cc * C;
      }
#pragma unroll
      for (int h = 0; h < V; h++)
        d[h] = *reinterpret_cast<const gu32x4*>(
            reinterpret_cast<uintptr_t>(s[h & 1] + (128 / sizeof(T)) * (h >> 1)));
    };
    u32x4 ring[RING][V];
    // unconditional preload (an empty box reads the frame's first pixel): the
    // waits below then count exactly
#pragma unroll
    for (int k = 0; k < RING; k++) {
      load_tile(ring[k], k);
      __builtin_amdgcn_sched_barrier(0);
    }

    // A fragments: lane (i = lane & 15, q = lane >> 4) holds patch row i
    // (zero for rows i >= np); fp32: channels 16 h + 4 q + s at a[4 h + s],
    // fp16: channels 32 t + 8 q + j at ah[t][j]
    constexpr bool kF16 = std::is_same<T, __half>::value;
    float a[kF16 ? 1 : 32];
    f16x8 ah[kF16 ? 4 : 1];
    {
#pragma unroll
      for (int r = 0; r < kPA; r++) reinterpret_cast<u32x4*>(G)[min(lane + kWave * r, n16 - 1)] = pa[r];
      wave_lds_sync();
      const bool arow = idx_ok && ai < np;
      const int fi = min(ai, np - 1);
      if constexpr (kF16) {
        const _Float16* Gh = reinterpret_cast<const _Float16*>(G);
#pragma unroll
        for (int t = 0; t < 4; t++)
#pragma unroll
          for (int j = 0; j < 8; j++) {
            const _Float16 v = Gh[(32 * t + 8 * aq + j) * np + fi];
            ah[t][j] = arow ? v : (_Float16)0.0f;
          }
      } else {
#pragma unroll
        for (int h = 0; h < 8; h++)
#pragma unroll
          for (int s = 0; s < 4; s++) {
            const float v = G[(16 * h + 4 * aq + s) * np + fi];
            a[4 * h + s] = arow ? v : 0.0f;
          }
      }
      wave_lds_sync();  // G free again
    }

    // stage addresses: a lane writes its 16 B of pixel pt = 8 ph + (lane >> 3),
    // chunk c = lane & 7 at pt * 128 + ((c ^ (pt & 7)) * 16); B fragment of
    // lane (n, q), half j of the quarter: chunk 4 j + q of pixel n
    const int wr0 = (lane >> 3) * 128 + (((lane & 7) ^ (lane >> 3)) << 4);
    const int rd0 = ai * 128 + ((aq ^ (ai & 7)) << 4), rd1 = ai * 128 + (((4 + aq) ^ (ai & 7)) << 4);
    auto step = [&](u32x4 (&cur)[V], int t) __attribute__((always_inline)) {
      const bool live = t < ntile;
      f32x4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
      if (live) {
        // one 128-B line of the tile's 16 pixels per stage round: fp32 32
        // channels (8 MFMAs of K = 4), fp16 64 channels (2 MFMAs of K = 32)
#pragma unroll
        for (int qt = 0; qt < V / 2; qt++) {
          *reinterpret_cast<u32x4*>(stage + wr0) = cur[2 * qt];
          *reinterpret_cast<u32x4*>(stage + 1024 + wr0) = cur[2 * qt + 1];
          const u32x4 b0 = *reinterpret_cast<const u32x4*>(stage + rd0);
          const u32x4 b1 = *reinterpret_cast<const u32x4*>(stage + rd1);
          if constexpr (kF16) {
            acc0 = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah[2 * qt], __builtin_bit_cast(f16x8, b0),
                                                          acc0, 0, 0, 0);
            acc1 = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah[2 * qt + 1],
                                                          __builtin_bit_cast(f16x8, b1), acc1, 0, 0, 0);
          } else {
            const float4 f0 = __builtin_bit_cast(float4, b0), f1v = __builtin_bit_cast(float4, b1);
            const float bb[8] = {f0.x, f0.y, f0.z, f0.w, f1v.x, f1v.y, f1v.z, f1v.w};
#pragma unroll
            for (int j = 0; j < 2; j++)
#pragma unroll
              for (int s = 0; s < 4; s++) {
                const float av = a[4 * (2 * qt + j) + s], bv = bb[4 * j + s];
                if (s & 1) acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(av, bv, acc1, 0, 0, 0);
                else acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(av, bv, acc0, 0, 0, 0);
              }
          }
        }
      }
      // refill this slot with tile t + RING (unconditional: every path into
      // the next group has the same load order, the wait before a tile
      // drains only that tile's loads)
      load_tile(cur, t + RING);
      if (live) {
        // D: lane holds rows 4q + r (patch pixels), column lane & 15 (box pixel)
#pragma unroll
        for (int r = 0; r < 4; r++) {
          const int row = 4 * aq + r;
          if (row < np) G[row * kLvlBoxStride + 16 * t + ai] = acc0[r] + acc1[r];
        }
      }
    };
    for (int t = 0; t < ntile; t += RING) {
#pragma unroll
      for (int k = 0; k < RING; k++) step(ring[k], t + k);
    }
    wave_lds_sync();
    bilinear_store(true);
    wave_lds_sync();  // G, stage and geo free for the next unit
  };

  // wave w: pair sp = w / L, level lw = w % L of its first edge, L-1-lw of its second
  const int lim = order ? min(per * (x8 + 1), M) : nE;
  auto pair_ok = [&](int q, int u) {
    const int pa = x8 * per + q;
    return q < half && (u == 0 ? pa < lim
                               : (paired && pa + half < lim && pa + half < x8 * per + per));
  };
  {
    const int sp = PAIRED ? 0 : w / L, lw = w - sp * L, q = j8 * npair + sp;
    const int pA = x8 * per + q;
    if (pair_ok(q, 0)) run_unit(pA, lw, outA);
    if (pair_ok(q, 1)) run_unit(pA + half, L - 1 - lw, reinterpret_cast<float*>(stage));
  }

  // the edges' [nout][L] blocks from the waves' slices: whole lines, 16 B per
  // lane when the block is a whole number of 16-B pieces
  __syncthreads();
  const int nl = nout * L, tid = threadIdx.x, nth = npair * L * kWave;
#pragma unroll
  for (int u2 = 0; u2 < (PAIRED ? 2 : 2 * kMaxL); u2++) {
    const int sp = u2 >> 1, u = u2 & 1, q = j8 * npair + sp;
    if (sp >= npair) break;
    if (!pair_ok(q, u)) continue;
    const int pos = x8 * per + q + (u ? half : 0);
    const int edge = order ? wave_uniform(order[pos]) : pos;
    float* dst = out + (size_t)edge * nl;
    // level l of the pair's first edge is in wave sp L + l's own region, of
    // its second edge in wave sp L + L-1-l's stage
    const int off = u == 0 ? (int)(reinterpret_cast<char*>(outA) - wl) : (int)(stage - wl);
    auto slice = [&](int l) -> const float* {
      const int wv = sp * L + (u == 0 ? l : L - 1 - l);
      return reinterpret_cast<const float*>(reinterpret_cast<const char*>(smem) + wv * wbytes + off);
    };
    if (L == kMaxL && (nl & 3) == 0) {
      const float* s0 = slice(0);
      const float* s1 = slice(1);
      const float* s2 = slice(2);
      const float* s3 = slice(3);
      for (int o = tid; o < nout; o += nth)
        *reinterpret_cast<float4*>(dst + 4 * o) = make_float4(s0[o], s1[o], s2[o], s3[o]);
    } else {
      for (int e = tid; e < nl; e += nth) {
        const int o = e / L, l = e - o * L;
        dst[e] = slice(l)[o];
      }
    }
  }
}

// [count, C, H, W] -> [count, H, W, C] (one 32 x 32 tile of (c, hw) per block)
template <typename T>
__global__ void __launch_bounds__(256)
    nchw_to_nhwc_kernel(const T* __restrict__ src, T* __restrict__ dst, int C, int HW) {
  __shared__ T tile[32][33];
  const size_t f = blockIdx.z;
  const int c0 = blockIdx.y * 32, p0 = blockIdx.x * 32;
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;  // 32 x 8
  const T* s = src + f * C * (size_t)HW;
  T* d = dst + f * C * (size_t)HW;
  for (int j = ty; j < 32; j += 8) {
    const int c = c0 + j, p = p0 + tx;
    if (c < C && p < HW) tile[j][tx] = s[(size_t)c * HW + p];
  }
  __syncthreads();
  for (int j = ty; j < 32; j += 8) {
    const int p = p0 + j, c = c0 + tx;
    if (c < C && p < HW) d[(size_t)p * C + c] = tile[tx][j];
  }
}


// ---------------------------------------------------------------------------
// Frame insertion of a channels-last pyramid (dpvo.py frame insertion: the
// level-1 fmap written into the ring slot, level s = avg_pool2d(fmap, s, s),
// dpvo.py __call__ / net.py:411).  One launch for every level: a workgroup
// stages an 8 x 32 pixel x 32 channel tile of the NCHW level-1 frame in LDS
// (coalesced 128-B row reads), writes the channels-last level-1 pixels and
// every pooled level whose s x s windows the tile holds (s | 8, s | 32), as
// 128-B channel runs.  Pool order = torch's avg_pool2d (row-major sum in
// fp32, then / s^2), so the pooled levels are bit-identical to it.
// ---------------------------------------------------------------------------
template <typename T>
__global__ void __launch_bounds__(256)
    pyramid_insert_kernel(const T* __restrict__ src, InsLevels lv, int L, int C, int H,
                          int W) {
  __shared__ float tile[kInsTC * kInsCS];
  ins_tile<T>(src, lv, L, C, H, W, blockIdx.x, blockIdx.y, blockIdx.z, threadIdx.x, true, tile);
}

}  // namespace dpvo

using namespace dpvo;

DPVO_EXPORT int dpvo_corr_forward_levels_nhwc_ordered(
    const void* fmap1, const void* const* fmap2, const int* H2, const int* W2, const float* scale,
    int L, const float* coords, const int64_t* ii, const int64_t* jj, const int32_t* order, int B,
    int M, int C, int H, int W, int N1, int N2, int radius, int dtype, float* out, void* stream) {
  if (L <= 0 || radius < 0 || radius > 7 || C <= 0 || H <= 0 || W <= 0) return DPVO_ERR_INVALID;
  const int np = H * W, Dp = 2 * radius + 1;
  if ((dtype != DPVO_F32 && dtype != DPVO_F16) || C != kNhwcC || L > kMaxL || np > kNpMax ||
      Dp * Dp * np > kOutPerLane * kWave)
    return DPVO_ERR_UNSUPPORTED;
  if (B * M == 0) return DPVO_OK;
  if (!fmap1 || !coords || !ii || !jj || !out) return DPVO_ERR_INVALID;
  NhwcLevels lv = {};
  for (int l = 0; l < L; l++) {
    if (!fmap2[l] || H2[l] <= 0 || W2[l] <= 0 || !(scale[l] > 0.f)) return DPVO_ERR_INVALID;
    lv.f2[l] = fmap2[l];
    lv.H2[l] = H2[l];
    lv.W2[l] = W2[l];
    lv.scale[l] = scale[l];
  }
  // G: np rows x kLvlBoxStride per wave; the raw path (boxes past
  // kLvlMaxTiles tiles) keeps np x D x D raw dot products there
  const int D = 2 * radius + 2;
  if (D * D > kLvlBoxStride) return DPVO_ERR_UNSUPPORTED;
  const bool ordered = order && B == 1;
  const int* ord = ordered ? (const int*)order : (const int*)nullptr;
  hipStream_t st = as_stream(stream);
  // one wave per (edge, level) unit, two units per wave, whole-line tiles
  const int npair = corr_lvl_npos(L);
  const size_t lsm = (size_t)npair * L * corr_lvl_wave_bytes(np, radius);
  const unsigned per = ordered ? (unsigned)((M + 7) / 8) : (unsigned)(B * M);
  const unsigned nwg = ((corr_lvl_paired(L) ? (per + 1) / 2 : per) + npair - 1) / npair;
  const unsigned lg = ordered ? 8u * nwg : nwg;
  const dim3 g(lg), blk(npair * L * kWave);
  const bool r9 = np == 9 && radius == 3;  // DPVO: p = 3, R = 3
#define LVL_LAUNCH(TT, R9, PR)                                                                \
  hipLaunchKernelGGL((corr_nhwc_lvl_kernel<TT, 2, R9, PR>), g, blk, lsm, st, (const TT*)fmap1, lv, \
                     L, coords, ii, jj, B, M, np, N1, N2, radius, ord, out)
#define LVL_LAUNCH_P(TT, R9)              \
  if (corr_lvl_paired(L)) LVL_LAUNCH(TT, R9, true); \
  else LVL_LAUNCH(TT, R9, false)
  if (dtype == DPVO_F32) {
    if (r9) { LVL_LAUNCH_P(float, true); } else { LVL_LAUNCH_P(float, false); }
  } else {
    if (r9) { LVL_LAUNCH_P(__half, true); } else { LVL_LAUNCH_P(__half, false); }
  }
#undef LVL_LAUNCH_P
#undef LVL_LAUNCH
  return launch_status();
}

DPVO_EXPORT int dpvo_corr_forward_levels_nhwc(const void* fmap1, const void* const* fmap2,
                                              const int* H2, const int* W2, const float* scale,
                                              int L, const float* coords, const int64_t* ii,
                                              const int64_t* jj, int B, int M, int C, int H,
                                              int W, int N1, int N2, int radius, int dtype,
                                              float* out, void* stream) {
  return dpvo_corr_forward_levels_nhwc_ordered(fmap1, fmap2, H2, W2, scale, L, coords, ii, jj,
                                               nullptr, B, M, C, H, W, N1, N2, radius, dtype, out,
                                               stream);
}

DPVO_EXPORT int dpvo_feature_to_nhwc(const void* src, void* dst, int count, int C, int H, int W,
                                     int dtype, void* stream) {
  if (count < 0 || C <= 0 || H <= 0 || W <= 0 || !src || !dst) return DPVO_ERR_INVALID;
  if (count == 0) return DPVO_OK;
  const int HW = H * W;
  const dim3 grid((HW + 31) / 32, (C + 31) / 32, count), block(256);
  hipStream_t s = as_stream(stream);
  switch (dtype) {
    case DPVO_F32:
      hipLaunchKernelGGL(nchw_to_nhwc_kernel<float>, grid, block, 0, s, (const float*)src,
                         (float*)dst, C, HW);
      return launch_status();
    case DPVO_F16:
      hipLaunchKernelGGL(nchw_to_nhwc_kernel<__half>, grid, block, 0, s, (const __half*)src,
                         (__half*)dst, C, HW);
      return launch_status();
  }
  return DPVO_ERR_UNSUPPORTED;
}

static int pyramid_insert_impl(const void* src, void* const* dst, const int* scale, int L, int C,
                               int H, int W, int dtype, void* stream, const int32_t* slot_dev,
                               int mem, const int64_t* slot_bytes) {
  if (!src || !dst || !scale || L <= 0 || C <= 0 || H <= 0 || W <= 0) return DPVO_ERR_INVALID;
  if ((dtype != DPVO_F32 && dtype != DPVO_F16) || L > kMaxL) return DPVO_ERR_UNSUPPORTED;
  if (slot_dev && (mem <= 0 || !slot_bytes)) return DPVO_ERR_INVALID;
  InsLevels lv = {};
  lv.slot_dev = (const int*)slot_dev;
  lv.mem = mem > 0 ? mem : 1;
  for (int l = 0; l < L && slot_dev; l++) lv.slot_bytes[l] = slot_bytes[l];
  for (int l = 0; l < L; l++) {
    const int s = scale[l];
    if (!dst[l]) return DPVO_ERR_INVALID;
    if (s != 1 && s != 2 && s != 4 && s != 8) return DPVO_ERR_UNSUPPORTED;
    lv.dst[l] = dst[l];
    lv.s[l] = s;
  }
  const dim3 grid((W + kInsTX - 1) / kInsTX, (H + kInsTY - 1) / kInsTY, (C + kInsTC - 1) / kInsTC);
  if (dtype == DPVO_F16)
    hipLaunchKernelGGL(pyramid_insert_kernel<__half>, grid, dim3(256), 0, as_stream(stream),
                       (const __half*)src, lv, L, C, H, W);
  else
    hipLaunchKernelGGL(pyramid_insert_kernel<float>, grid, dim3(256), 0, as_stream(stream),
                       (const float*)src, lv, L, C, H, W);
  return launch_status();
}

DPVO_EXPORT int dpvo_feature_pyramid_insert(const void* src, void* const* dst, const int* scale,
                                            int L, int C, int H, int W, int dtype, void* stream) {
  return pyramid_insert_impl(src, dst, scale, L, C, H, W, dtype, stream, nullptr, 0, nullptr);
}

DPVO_EXPORT int dpvo_feature_pyramid_insert_ring(const void* src, void* const* dst0,
                                                 const int64_t* slot_bytes, const int* scale,
                                                 int L, int C, int H, int W, int mem,
                                                 const int32_t* slot_dev, int dtype, void* stream) {
  if (!slot_dev) return DPVO_ERR_INVALID;
  return pyramid_insert_impl(src, dst0, scale, L, C, H, W, dtype, stream, slot_dev, mem,
                             slot_bytes);
}
