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
// bilinear + permute reads the windows out of G.  Two kernels:
//   corr_nhwc_lvl_kernel  fp32 features: one wave per (edge, level) unit,
//                         whole-line tile loads through an LDS stage, exact
//                         fp32 products (v_mfma_f32_16x16x4_f32);
//   corr_nhwc_kernel      fp16 features (the fork's MIXED_PRECISION rings):
//                         one wave per edge over every level,
//                         v_mfma_f32_16x16x32_f16 with fp32 accumulation.
#include <type_traits>

#include "common.hpp"
#include "pyr_insert.hpp"


namespace dpvo {

constexpr int kNhwcWaves = 4;   // edges per workgroup
constexpr int kNhwcC = 128;     // channels (DPVO gmap / fmap width)
constexpr int kMaxTiles = 10;   // box up to 160 pixels through the matrix path
constexpr int kBoxStride = 16 * kMaxTiles + 4;  // +4: the 4 row groups of a G tile store hit distinct LDS banks
constexpr int kMaxL = 4;        // levels per launch
constexpr int kOutPerLane = 8;  // (2R+1)^2 * p*p <= 512 outputs per level
constexpr int kNpMax = 16;      // p*p <= 16 (one MFMA row tile)
// Box tiles per wave in the register ring (kRing - 1 in flight).  A 4-deep
// ring (two waves per SIMD, al' fragments in LDS to fit 256 VGPRs) measured
// 55.7 us against 53.9 for 3 (scripts/micro/corr_bench, cfg2 shape), and
// round 4's deeper rings at one wave per SIMD were no faster either.
constexpr int kRing = 3;

struct NhwcLevels {
  const void* f2[kMaxL];  // float or __half, [B, N2, H, W, C]
  int H2[kMaxL], W2[kMaxL];
  float scale[kMaxL];
};

// floats of a wave's output block: nout * L, rounded to whole float4s
__host__ __device__ inline int corr_obuf_floats(int np, int R, int L) {
  return ((2 * R + 1) * (2 * R + 1) * np * L + 3) & ~3;
}

struct NhwcGeom {
  int x0[kNpMax], y0[kNpMax];
  float dx[kNpMax], dy[kNpMax];
  int xlo, ylo, bw, bh, ntile, pad[3];  // the level's (wave-uniform) box
};

// Box tiles of flattened position j (level level_at(j)) of a wave's edge, in
// LDS: the per-tile load address is one broadcast LDS read plus a few VALU
// ops (selecting among per-level registers by a run-time position compiled
// to chains of scalar branches: ~80 SALU instructions per tile)
struct alignas(16) TileDesc {
  const void* base;  // box origin (frame, level)
  int row, bw;       // elements per map row (W2 * C), box width
  int npx;           // box pixels
  float rbw;         // 1 / bw
  int c0, c1;        // flattened tile range [c0, c1) of the position
  int lvl, pad[3];
};

// LDS bytes of one corr_nhwc_kernel workgroup: per wave G, the level
// geometry, the output block and the tile descriptors
inline size_t corr_nhwc_lds_bytes(int np, int R, int L) {
  return sizeof(float) * kNhwcWaves * np * kBoxStride + sizeof(NhwcGeom) * kNhwcWaves * kMaxL +
         sizeof(float) * kNhwcWaves * corr_obuf_floats(np, R, L) +
         sizeof(TileDesc) * kNhwcWaves * kMaxL;
}

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef _Float16 f16x4 __attribute__((ext_vector_type(4)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
// 16-B tile vector (a native vector: a uint4 struct copy is a memcpy that
// keeps the ring in scratch)
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
// global-address-space view of a tile vector: the box base comes out of LDS
// (TileDesc), where the compiler loses the pointer's address space -- a
// generic pointer makes every tile load a flat load, which counts in both
// vmcnt and lgkmcnt and makes the wait before each tile drain the whole ring
typedef const __attribute__((address_space(1))) u32x4 gu32x4;

// fp16 features (DPVO's MIXED_PRECISION runtime, correlation_kernel.py:552-654):
// v_mfma_f32_16x16x16_f16, fp32 accumulation (documented deviation: the
// reference accumulates fp16 products in fp16).  K order: lane group q
// (= lane >> 4) owns channels [32q, 32q + 32); K step h uses its channels
// 32q + 4h .. + 3 for both A (gmap patch) and B (box pixels), so a lane's
// B data of a tile is ONE contiguous 64-B run of its pixel (4 x 16-B loads).
template <typename T>
struct CorrT;
template <>
struct CorrT<float> {
  static constexpr int kVecs = 8;  // 16-B loads per lane per tile (128 B)
  static constexpr int kLaneCh = 4;  // channel offset of lane group q: 4 q (+ 16 h)
};
template <>
struct CorrT<__half> {
  static constexpr int kVecs = 4;  // 4 x 16 B = 32 halves per lane per tile
  static constexpr int kLaneCh = 32;
};

// wave-uniform per-level parameter without a dynamic index into the kernel
// argument struct (that would route every access through scratch / flat
// loads, which count in vmcnt and force full drains in the tile loop)
template <typename X>
__device__ __forceinline__ X sel4(int l, X a, X b, X c, X d) {
  return l == 0 ? a : l == 1 ? b : l == 2 ? c : d;
}
#define LV_SEL(field, l) sel4((l), lv.field[0], lv.field[1], lv.field[2], lv.field[3])

__device__ __forceinline__ f16x4 h4_lo(u32x4 v) {
  typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
  return __builtin_bit_cast(f16x4, (u32x2){v.x, v.y});
}
__device__ __forceinline__ f16x4 h4_hi(u32x4 v) {
  typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
  return __builtin_bit_cast(f16x4, (u32x2){v.z, v.w});
}

// fp16 features: one wave per edge, every level (the gmap patch and the
// coordinates are loaded once per edge).  The kernel is latency-bound: at DPVO sizes there
// are only 8 edges per CU, so the bytes each wave keeps in flight decide the
// bandwidth.  Design:
//  * the gmap patch arrives with 16-B coalesced loads, staged through LDS;
//  * the geometry of every level is computed up front (power-of-two level
//    scales are applied as exact reciprocal multiplies);
//  * the box tiles of all levels form ONE flattened sequence with two more
//    tiles in flight (a 3-deep register ring; 4 deep would need > 256 VGPRs
//    and halve the occupancy) while the current one multiplies; the loop body
//    is not unrolled (the bilinear is inlined once): kernel code stays small;
//  * a level's bilinear + permute runs as soon as its last tile is in LDS,
//    from per-lane output codes computed once (no integer division per level).

// RAW9: p = 3, R = 3 (DPVO): the bilinear runs on the raw (2R+2)^2 = 64 grid
// with one lane per raw point (see below); otherwise one lane per output.
template <typename T, bool RAW9>
__global__ void __launch_bounds__(kNhwcWaves* kWave, 2)  // 2 workgroups (8 waves) per CU: every edge resident at once
    corr_nhwc_kernel(const T* __restrict__ fmap1, NhwcLevels lv, int L,
                     const float* __restrict__ coords, const int64_t* __restrict__ ii,
                     const int64_t* __restrict__ jj, int B, int M, int np, int N1, int N2, int R,
                     const int* __restrict__ order, float* __restrict__ out) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int wid = wave_uniform(threadIdx.x / kWave), lane = threadIdx.x & (kWave - 1);
  float* G = smem + wid * (np * kBoxStride);
  NhwcGeom* geo = reinterpret_cast<NhwcGeom*>(smem + kNhwcWaves * np * kBoxStride) + wid * kMaxL;
  // the edge's [nout][L] output block, assembled level by level (stored once,
  // coalesced, at the end: no output registers held across the tile loop)
  const int ostride = corr_obuf_floats(np, R, L);
  float* obuf = reinterpret_cast<float*>(reinterpret_cast<NhwcGeom*>(smem + kNhwcWaves * np * kBoxStride) +
                                         kNhwcWaves * kMaxL);
  obuf += wid * ostride;
  // tile descriptors after the output blocks of all waves
  TileDesc* td = reinterpret_cast<TileDesc*>(obuf - wid * ostride + kNhwcWaves * ostride) +
                 wid * kMaxL;
  int edge;
  if (order) {
    // XCD-aware: workgroups are dispatched round-robin over the 8 XCDs, so
    // workgroup w runs on XCD w % 8.  XCD x takes the x-th eighth of the edges
    // grouped by target frame (order[], B == 1): a frame's coarse levels then
    // stay in that XCD's 4 MB L2 instead of being fetched by every XCD.
    const int nwg = (M + kNhwcWaves - 1) / kNhwcWaves, per = (nwg + 7) / 8;
    const int chunk = (blockIdx.x % 8) * per + blockIdx.x / 8;
    const int p = chunk * kNhwcWaves + wid;
    if (chunk >= nwg || p >= M) return;
    edge = wave_uniform(order[p]);
  } else {
    edge = blockIdx.x * kNhwcWaves + wid;
    if (edge >= B * M) return;  // waves are independent: no block barrier below
  }
  const int b = edge / M, m = edge % M;
  const int ix = wave_uniform((int)ii[m]), jx = wave_uniform((int)jj[m]);
  const bool idx_ok = ix >= 0 && ix < N1 && jx >= 0 && jx < N2;
  const int C = kNhwcC, D = 2 * R + 2, Dp = D - 1, nout = Dp * Dp * np;
  const float cv = (lane < 2 * np) ? coords[((size_t)b * M + m) * 2 * np + lane] : 0.f;
  __builtin_amdgcn_sched_barrier(0);  // coords first: the geometry then waits for them only

  // ---- gmap patch [C][np] -> LDS (in G, free until the first tile) -> A
  // fragments: lane (i = lane & 15, q = lane >> 4) holds f1[c][i] for
  // c = 16h + 4q + s at K step 4h + s (the same channel order as the B loads)
  const int ai = lane & 15, aq = lane >> 4;
  static_assert(std::is_same<T, __half>::value,
                "fp16 features only: fp32 runs corr_nhwc_lvl_kernel (exact fp32 products)");
  constexpr bool kHalf = true;
  f16x4 Afh[kNhwcC / 16];
  // the patch's loads are issued here; they are staged into the A fragments
  // only after the first box tiles have been issued (build_A below), so the
  // gmap round trip and the first tiles' round trip overlap
  constexpr int kPerA = 16 / sizeof(T);  // 16-B units of the [C][np] patch
  constexpr int kRA = (kNhwcC * kNpMax / kPerA + kWave - 1) / kWave;
  const int n16 = (C * np) / kPerA;  // C * np is a multiple of 8 (C = 128)
  u32x4 st[kRA];
  {
    const T* f1 = fmap1 + ((size_t)b * N1 + (idx_ok ? ix : 0)) * C * np;
#pragma unroll
    for (int r = 0; r < kRA; r++) {
      const int v = lane + kWave * r;
      // unconditional (clamped) loads: no branch around them, so the waits below
      // count exactly (a conditional load makes the compiler drain everything)
      st[r] = reinterpret_cast<const u32x4*>(f1)[min(v, n16 - 1)];
    }
  }
  auto build_A = [&]() __attribute__((always_inline)) {
    // unconditional: lanes past the end rewrite the last unit with its own value
#pragma unroll
    for (int r = 0; r < kRA; r++)
      reinterpret_cast<u32x4*>(G)[min(lane + kWave * r, n16 - 1)] = st[r];
    wave_lds_sync();
    const bool arow = idx_ok && ai < np;
    if constexpr (kHalf) {
      const __half* Gh = reinterpret_cast<const __half*>(G);
#pragma unroll
      for (int h = 0; h < kNhwcC / 16; h++)
#pragma unroll
        for (int s = 0; s < 4; s++) {
          Afh[h][s] = arow ? (_Float16)__half2float(Gh[(32 * aq + 4 * h + s) * np + ai])
                           : (_Float16)0.0f;
        }
    }
    wave_lds_sync();  // A fragments read: G free again
  };

  // ---- geometry of every level up front, lane-parallel: lane (l = lane >> 4,
  // k = lane & 15) takes patch pixel k at level l (floor / frac), 16-lane
  // min / max reductions give each level's box (kept in LDS: levels are
  // indexed dynamically below)
  int cum[kMaxL + 1];  // flattened fast-path tile offsets (wave-uniform)
  {
    const int gl = lane >> 4, gk = lane & 15;
    const bool act = gl < L && gk < np;
    const float xr = __shfl(cv, min(gk, np - 1), kWave), yr = __shfl(cv, np + min(gk, np - 1), kWave);
    const float sc = LV_SEL(scale, gl < L ? gl : 0);
    const bool pow2 = (__float_as_uint(sc) & 0x7fffffu) == 0u;  // x / 2^k == x * 2^-k
    const float rs = 1.0f / sc;
    const float x = pow2 ? xr * rs : xr / sc, y = pow2 ? yr * rs : yr / sc;
    const int xf = ifloor_safe(x), yf = ifloor_safe(y);
    if (act) {
      geo[gl].x0[gk] = xf;
      geo[gl].y0[gk] = yf;
      geo[gl].dx[gk] = x - floorf(x);  // correlation_kernel.cu:262
      geo[gl].dy[gk] = y - floorf(y);
    }
    int xlo = act ? xf : 0x7fffffff, ylo = act ? yf : 0x7fffffff;
    int xhi = act ? xf : -0x7fffffff, yhi = act ? yf : -0x7fffffff;
#pragma unroll
    for (int o = 8; o > 0; o >>= 1) {
      xlo = min(xlo, __shfl_xor(xlo, o, kWave));
      ylo = min(ylo, __shfl_xor(ylo, o, kWave));
      xhi = max(xhi, __shfl_xor(xhi, o, kWave));
      yhi = max(yhi, __shfl_xor(yhi, o, kWave));
    }
    if (gk == 0 && gl < L) {
      const int H2 = LV_SEL(H2, gl), W2 = LV_SEL(W2, gl);
      xlo = max(xlo - R, 0);
      ylo = max(ylo - R, 0);
      xhi = min(xhi + R + 1, W2 - 1);
      yhi = min(yhi + R + 1, H2 - 1);
      int bw = xhi - xlo + 1, bh = yhi - ylo + 1;
      if (bw <= 0 || bh <= 0 || !idx_ok) bw = bh = 0;
      geo[gl].xlo = xlo;
      geo[gl].ylo = ylo;
      geo[gl].bw = bw;
      geo[gl].bh = bh;
      geo[gl].ntile = (bw * bh + 15) >> 4;
    }
  }
  wave_lds_sync();  // geo visible
  // Level order: the fine level streams from HBM / the Infinity Cache, the
  // coarse levels hit in L2 and are matrix-core bound.  The second wave on a
  // SIMD (hardware wave slot, HW_ID[3:0]) walks the levels coarse -> fine, so
  // the two waves of a SIMD are in opposite phases instead of both waiting on
  // memory first and both multiplying later.
  const bool rev = (__builtin_amdgcn_s_getreg((3 << 11) | 4) & 1) != 0;
  auto level_at = [&](int j) { return rev ? L - 1 - j : j; };  // position -> level
  cum[0] = 0;
#pragma unroll
  for (int j = 0; j < kMaxL; j++) {
    const int nt = (j < L) ? wave_uniform(geo[level_at(j)].ntile) : 0;
    cum[j + 1] = cum[j] + ((nt <= kMaxTiles) ? nt : 0);
  }

  // ---- outputs.  Generic: lane owns outputs o = lane + 64u, decoded once
  // into (k, yy, xx).  RAW9: lane = (rx, ry) = (lane >> 3, lane & 7) owns the
  // raw window point (rx, ry) of every patch pixel k and, for rx, ry < 7, the
  // outputs (k, yy = ry, xx = rx) of every k: o = (rx * 7 + ry) * 9 + k, i.e.
  // 9 x L contiguous floats per lane.
  constexpr int kOuts = RAW9 ? 9 : kOutPerLane;
  int code[RAW9 ? 1 : kOutPerLane];
  if constexpr (!RAW9) {
#pragma unroll
    for (int u = 0; u < kOutPerLane; u++) {
      const int o = lane + kWave * u;
      const int k = o % np, t = o / np, yy = t % Dp, xx = t / Dp;
      code[u] = (o < nout) ? (k | (yy << 8) | (xx << 16)) : -1;
    }
  }
  const int rx = lane >> 3, ry = lane & 7;

  // bilinear + permute of level l from G (correlation_kernel.cu:260-271).
  // Branch-free: every tap is loaded from a clamped (valid) LDS address and
  // zeroed by a select.  RAW9: each lane loads ONE raw value per k, the other
  // three taps come from lanes +1 (y + 1), +8 (x + 1), +9 by cross-lane
  // shuffles: 9 LDS reads per lane and level instead of 32.
  auto bilinear_raw = [&](int l, bool fast) __attribute__((always_inline)) {
    const NhwcGeom* gg = geo + l;
    const int xlo = wave_uniform(gg->xlo), ylo = wave_uniform(gg->ylo);
    const int bw = wave_uniform(gg->bw), bh = wave_uniform(gg->bh);
    const int cap = max(bw * bh - 1, 0);
    // every LDS read of the level first, the obuf writes last: a write between
    // them (possible alias for the compiler) would serialise the 9 patch pixels
    float r[9], dxv[9], dyv[9];
#pragma unroll
    for (int k = 0; k < 9; k++) {
      dxv[k] = gg->dx[k];
      dyv[k] = gg->dy[k];
      if (fast) {
        const int gy = gg->y0[k] + ry - R - ylo, gx = gg->x0[k] + rx - R - xlo;
        const bool in = gy >= 0 && gy < bh && gx >= 0 && gx < bw;
        const float a = G[k * kBoxStride + min(max(gy * bw + gx, 0), cap)];
        r[k] = in ? a : 0.f;
      } else {
        r[k] = G[k * 64 + ry * 8 + rx];
      }
    }
    float v[9];
#pragma unroll
    for (int k = 0; k < 9; k++) {
      const float r10 = __shfl_down(r[k], 1, kWave);   // (y + 1, x)
      const float r01 = __shfl_down(r[k], 8, kWave);   // (y, x + 1)
      const float r11 = __shfl_down(r[k], 9, kWave);   // (y + 1, x + 1)
      const float dx = dxv[k], dy = dyv[k];
      float t = ((1.f - dx) * (1.f - dy)) * r[k];
      t = t + (dx * (1.f - dy)) * r01;
      t = t + ((1.f - dx) * dy) * r10;
      t = t + (dx * dy) * r11;
      v[k] = t;
    }
    if (rx < 7 && ry < 7) {
#pragma unroll
      for (int k = 0; k < 9; k++) obuf[((rx * 7 + ry) * 9 + k) * L + l] = v[k];
    }
  };
  auto bilinear_gen = [&](int l, bool fast) __attribute__((always_inline)) {
    const NhwcGeom* gg = geo + l;
    const int xlo = wave_uniform(gg->xlo), ylo = wave_uniform(gg->ylo);
    const int bw = wave_uniform(gg->bw), bh = wave_uniform(gg->bh);
    const int cap = max(bw * bh - 1, 0);
    float vout[kOuts];
#pragma unroll
    for (int u = 0; u < kOuts; u++) {
      const int cd = max(code[RAW9 ? 0 : u], 0);
      const int k = cd & 0xff, yy = (cd >> 8) & 0xff, xx = cd >> 16;
      float r00, r01, r10, r11;
      if (fast) {
        const int gy = gg->y0[k] + yy - R - ylo, gx = gg->x0[k] + xx - R - xlo;
        const float* g = G + k * kBoxStride;
        const bool y0i = gy >= 0 && gy < bh, y1i = gy + 1 >= 0 && gy + 1 < bh;
        const bool x0i = gx >= 0 && gx < bw, x1i = gx + 1 >= 0 && gx + 1 < bw;
        const int i00 = min(max(gy * bw + gx, 0), cap);
        const int i01 = min(max(gy * bw + gx + 1, 0), cap);
        const int i10 = min(max((gy + 1) * bw + gx, 0), cap);
        const int i11 = min(max((gy + 1) * bw + gx + 1, 0), cap);
        const float a00 = g[i00], a01 = g[i01], a10 = g[i10], a11 = g[i11];
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
      const float dx = gg->dx[k], dy = gg->dy[k];
      float v = ((1.f - dx) * (1.f - dy)) * r00;
      v = v + (dx * (1.f - dy)) * r01;
      v = v + ((1.f - dx) * dy) * r10;
      v = v + (dx * dy) * r11;
      vout[u] = v;
    }
    // writes after every read (see bilinear_raw)
#pragma unroll
    for (int u = 0; u < kOuts; u++)
      if (code[RAW9 ? 0 : u] >= 0) obuf[(lane + kWave * u) * L + l] = vout[u];
  };
  auto bilinear = [&](int l, bool fast) __attribute__((always_inline)) {
    if constexpr (RAW9) bilinear_raw(l, fast);
    else bilinear_gen(l, fast);
  };

  // ---- flattened fast-path tiles, kRing - 1 in flight
  const int nT = cum[kMaxL];  // == cum[L]: positions >= L add no tiles
  constexpr int V = CorrT<T>::kVecs;  // 16-B loads per lane per tile
  // Per flattened position j (level level_at(j)): the box origin pointer, the
  // box row stride, width, pixel count and 1 / width and the position's tile
  // range, one TileDesc per position in LDS (lane j writes entry j)
  if (lane < kMaxL) {
    const int j = lane;
    const int l = (j < L) ? level_at(j) : 0;
    const NhwcGeom* gg = geo + l;
    const int H2 = LV_SEL(H2, l), W2 = LV_SEL(W2, l);
    const int gbw = gg->bw, gbh = gg->bh;
    const int bw0 = max(gbw, 1);
    // an empty box reads the frame's first pixel (in range whatever the
    // coordinates): the ring preload below is then unconditional
    const bool empty = gbw <= 0 || gbh <= 0;
    TileDesc d;
    d.base = static_cast<const T*>(LV_SEL(f2, l)) +
             (((size_t)b * N2 + (idx_ok ? jx : 0)) * H2 * W2 +
              (empty ? 0 : (size_t)gg->ylo * W2 + gg->xlo)) * C;
    d.row = W2 * C;
    d.bw = bw0;
    d.npx = bw0 * gbh;
    d.rbw = 1.0f / (float)bw0;
    d.c0 = j == 0 ? cum[0] : j == 1 ? cum[1] : j == 2 ? cum[2] : cum[3];
    d.c1 = j == 0 ? cum[1] : j == 1 ? cum[2] : j == 2 ? cum[3] : cum[4];
    d.lvl = l;
    d.pad[0] = d.pad[1] = d.pad[2] = 0;
    td[j] = d;
  }
  wave_lds_sync();
  auto pos_of = [&](int i) __attribute__((always_inline)) {  // flattened tile -> position
    return (i >= cum[1]) + (i >= cum[2]) + (i >= cum[3]);
  };
  // Tile i's loads: lane (i, q) reads 16 B of box pixel i directly in the MFMA
  // B layout (16 pixels x 64 B per instruction).  (Whole-line loads staged
  // through an LDS image and read back as B fragments measured 5-8 % slower.)
  auto load_tile = [&](u32x4 (&dst)[V], int i) __attribute__((always_inline)) {
    i = min(i, max(nT - 1, 0));  // past the end: re-read the last tile (never used)
    const TileDesc d = td[pos_of(i)];
    const int t = i - d.c0;
    auto pix = [&](int q) __attribute__((always_inline)) -> int {  // element offset of box pixel 16t + q
      const int px = min(16 * t + q, max(d.npx - 1, 0));  // pad columns read pixel npx-1
      const int r = (int)(((float)px + 0.5f) * d.rbw), cc = px - r * d.bw;
      return r * d.row + cc * C;
    };
    {
      const T* s = static_cast<const T*>(d.base) + pix(ai) + CorrT<T>::kLaneCh * aq;
#pragma unroll
      for (int h = 0; h < V; h++)
        dst[h] = *reinterpret_cast<const gu32x4*>(
            reinterpret_cast<uintptr_t>(s + (kHalf ? 8 * h : 16 * h)));
    }
  };
  u32x4 ring[kRing][V];
  // register ring of kRing tiles, rotated by NAME (the loop is unrolled by
  // kRing): while tile i multiplies, tiles i + 1 .. i + kRing - 1 are in
  // flight and the wait before tile i only drains tile i's own loads.  (A
  // rotation by register moves forces a full vmcnt(0) drain every tile:
  // moving the youngest tile's registers waits for its loads.)
  // issue order slot 0, 1, ... (sched barriers): the wait before the first
  // tile then drains only slot 0's loads.  Unconditional: under an `if (nT > 0)`
  // the wait before the patch staging (build_A) counted only the patch loads
  // of the no-tile path and drained two tiles of the ring.
#pragma unroll
  for (int k = 0; k < kRing; k++) {
    load_tile(ring[k], k);
    __builtin_amdgcn_sched_barrier(0);
  }
  build_A();
  // Level l the scalar way: raw[k][yy][xx] as fp32 dot products straight
  // from HBM into G, then the bilinear (levels off the fast path: windows too
  // spread for it).
  auto raw_level = [&](int l) {
    const int H2 = LV_SEL(H2, l), W2 = LV_SEL(W2, l);
    const T* f2 = static_cast<const T*>(LV_SEL(f2, l)) + ((size_t)b * N2 + jx) * H2 * W2 * C;
    wave_lds_sync();  // G's tiles (if any) read
    for (int e = lane; e < np * D * D; e += kWave) {
      const int k = e / (D * D), t = e % (D * D), yy = t / D, xx = t % D;
      const int i1 = geo[l].y0[k] + yy - R, j1 = geo[l].x0[k] + xx - R;
      float sacc = 0.f;
      if (idx_ok && i1 >= 0 && i1 < H2 && j1 >= 0 && j1 < W2) {
        const T* px = f2 + ((size_t)i1 * W2 + j1) * C;
        const T* f1 = fmap1 + ((size_t)b * N1 + ix) * C * np;
        for (int c = 0; c < C; c++) sacc += to_acc(f1[(size_t)c * np + k]) * to_acc(px[c]);
      }
      G[e] = sacc;
    }
    wave_lds_sync();
    bilinear(l, false);
    wave_lds_sync();
  };
  // levels off the fast path (empty box, or windows too spread for it) first
  for (int l = 0; l < L; l++) {
    const int nt = wave_uniform(geo[l].ntile);
    if (nt > kMaxTiles) {
      raw_level(l);
    } else if (nt == 0) {
      bilinear(l, true);  // every tap reads 0 (out of the empty box)
    }
  }

  if (nT > 0) {
    // Deferred G store: tile i's sums are written in step i + 1, after that
    // step's MFMAs are issued, so the wave never stalls on the chain it has
    // just issued (a level's last tile is stored at once, before the bilinear)
    f32x4 pg0 = {0.f, 0.f, 0.f, 0.f}, pg1 = {0.f, 0.f, 0.f, 0.f};
    int pgoff = -1;  // G column of the pending tile (16 t), -1: none
    auto store_g = [&](const f32x4& a0, const f32x4& a1, int toff) __attribute__((always_inline)) {
      // D: lane holds rows 4q + r (patch pixels), column lane & 15 (box pixel)
#pragma unroll
      for (int r = 0; r < 4; r++) {
        const int row = 4 * aq + r;
        if (row < np) {
          G[row * kBoxStride + toff + ai] = a0[r] + a1[r];
        }
      }
    };
    auto step = [&](u32x4 (&cur)[V], int i) __attribute__((always_inline)) {
      const bool live = i < nT;  // the last group may hold 1-2 slots past the end
      // the tile's G values: acc0 + acc1
      f32x4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
      auto mma = [&](const u32x4 (&B)[V]) __attribute__((always_inline)) {
        if constexpr (kHalf) {
          // 4 K steps of 32 channels: vector h holds the lane's channels
          // 32q + 8h .. + 7, A the same channels (Afh[2h], Afh[2h + 1])
#pragma unroll
          for (int h = 0; h < V; h++) {
            const f16x8 a8 = __builtin_shufflevector(Afh[2 * h], Afh[2 * h + 1], 0, 1, 2, 3, 4, 5,
                                                     6, 7);
            const f16x8 b8 = __builtin_bit_cast(f16x8, B[h]);
            if (h & 1) acc1 = __builtin_amdgcn_mfma_f32_16x16x32_f16(a8, b8, acc1, 0, 0, 0);
            else acc0 = __builtin_amdgcn_mfma_f32_16x16x32_f16(a8, b8, acc0, 0, 0, 0);
          }
        }
      };
      if (live) mma(cur);
      if (pgoff >= 0) {  // the previous tile's sums (its MFMA chain has drained)
        store_g(pg0, pg1, pgoff);
        pgoff = -1;
      }
      {
        // refill this slot with tile i + kRing (past the end: the last tile again,
        // never used); unconditional, so every path into the next group has the
        // same load order and the wait before a tile drains only that tile's loads
        load_tile(cur, i + kRing);
      }
      if (!live) return;
      const TileDesc& d = td[pos_of(i)];
      const int t = i - d.c0, l = wave_uniform(d.lvl);
      const bool lend = i + 1 == wave_uniform(d.c1);
      if (!lend) {
        pg0 = acc0;
        pg1 = acc1;
        pgoff = wave_uniform(16 * t);
      }
      if (lend) {  // level complete: its last sums, the bilinear, then G is free again
        store_g(acc0, acc1, 16 * t);
        wave_lds_sync();
        bilinear(l, true);
        wave_lds_sync();
      }
    };
    // no early exit inside a group: a break path into the loop's flow block
    // would make the compiler wait for every outstanding load at the top
    for (int i = 0; i < nT; i += kRing) {
#pragma unroll
      for (int k = 0; k < kRing; k++) step(ring[k], i + k);
    }
  }

  // ---- one contiguous [nout][L] row block per edge
  float* dst = out + ((size_t)b * M + m) * nout * L;
  wave_lds_sync();
  if (((nout * L) & 3) == 0) {  // whole float4s; the block start is 16-B aligned then too
    for (int e = 4 * lane; e < nout * L; e += 4 * kWave)
      *reinterpret_cast<float4*>(dst + e) = *reinterpret_cast<const float4*>(obuf + e);
  } else {
    for (int e = lane; e < nout * L; e += kWave) dst[e] = obuf[e];
  }
}

// ---------------------------------------------------------------------------
// corr_nhwc_lvl_kernel: fp32 features, exact fp32 products
// (v_mfma_f32_16x16x4_f32), one wave per (edge, pyramid level) unit.
//
// What bounds A-CORR is the vector-memory path, not the matrix cores: the
// loads alone of the per-edge kernel's B layout (16 box pixels x 64 B per
// global_load_dwordx4 = 16 half-used 128-B lines per KiB) take 46.6 us at
// cfg2, the same bytes as whole lines (8 pixels x 128 B per instruction)
// 28.0 us (scripts/micro/load_pattern.hip).  So the box tiles are loaded as
// whole lines and turned into the MFMA B layout through a 2-KiB LDS stage per
// wave (one 32-channel quarter of the tile's 16 pixels at a time, XOR-swizzled
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
constexpr int kLvlStage = 16 * 128;                // bytes: 16 pixels x one 128-B quarter

struct LvlGeom {
  int x0[kNpMax], y0[kNpMax];
  float dx[kNpMax], dy[kNpMax];
};
// per wave: G [np][kLvlBoxStride] floats, the stage, the geometry
__host__ __device__ inline int corr_lvl_wave_bytes(int np) {
  return (int)(sizeof(float) * np * kLvlBoxStride + kLvlStage + sizeof(LvlGeom));
}

// RAW9: p = 3, R = 3 (DPVO) as compile-time constants; otherwise run-time np, R
template <int RING, bool RAW9>
__global__ void __launch_bounds__(kMaxL* kWave) __attribute__((amdgpu_waves_per_eu(RING > 2 ? 3 : 4)))
    corr_nhwc_lvl_kernel(const float* __restrict__ fmap1, NhwcLevels lv, int L,
                         const float* __restrict__ coords, const int64_t* __restrict__ ii,
                         const int64_t* __restrict__ jj, int B, int M, int np_, int N1, int N2,
                         int R_, const int* __restrict__ order, float* __restrict__ out) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int np = RAW9 ? 9 : np_, R = RAW9 ? 3 : R_;
  const int w = wave_uniform(threadIdx.x / kWave), lane = threadIdx.x & (kWave - 1);
  const int C = kNhwcC, D = 2 * R + 2, Dp = D - 1, nout = Dp * Dp * np;
  char* wl = reinterpret_cast<char*>(smem) + (size_t)w * corr_lvl_wave_bytes(np);
  float* G = reinterpret_cast<float*>(wl);
  char* stage = wl + sizeof(float) * np * kLvlBoxStride;
  LvlGeom* geo = reinterpret_cast<LvlGeom*>(stage + kLvlStage);
  const int ai = lane & 15, aq = lane >> 4;

  // edge positions of this workgroup: with an order (B == 1, XCD-aware) XCD
  // x = blockIdx % 8 takes the x-th eighth of the edges grouped by target
  // frame, a workgroup two positions of it half an eighth apart
  const int nE = B * M;
  const int per = order ? (M + 7) / 8 : nE, half = (per + 1) / 2;
  const int x8 = order ? (int)(blockIdx.x % 8) : 0, j8 = order ? (int)(blockIdx.x / 8) : (int)blockIdx.x;
  if (j8 >= half) return;

  // ---- one (edge position p, level lev) unit
  auto run_unit = [&](int p, int lev) __attribute__((always_inline)) {
    const int edge = order ? wave_uniform(order[p]) : p;
    const int b = edge / M, m = edge % M;
    const int ix = wave_uniform((int)ii[m]), jx = wave_uniform((int)jj[m]);
    const bool idx_ok = ix >= 0 && ix < N1 && jx >= 0 && jx < N2;

    // the gmap patch [C][np] (whole lines, 16 B per lane), staged through G
    // once the first box tiles are in flight
    constexpr int kPA = (kNhwcC * (RAW9 ? 9 : kNpMax) / 4 + kWave - 1) / kWave;
    const int n16 = C * np / 4;
    u32x4 pa[kPA];
    {
      const float* f1 = fmap1 + ((size_t)b * N1 + (idx_ok ? ix : 0)) * C * np;
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
    float* dst = out + ((size_t)b * M + m) * nout * L + lev;

    // bilinear + permute from G (correlation_kernel.cu:260-271), then this
    // level's slice of the edge's [nout][L] block straight to HBM: output o
    // of lane o % 64 (consecutive outputs in consecutive lanes, 16 B apart)
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
        float* so = reinterpret_cast<float*>(stage);
        if (on) {
#pragma unroll
          for (int k = 0; k < 9; k++) so[(xx * Dp + yy) * 9 + k] = v[k];
        }
        wave_lds_sync();
#pragma unroll
        for (int u = 0; u < 7; u++) {
          const int o = lane + kWave * u;
          const float vo = so[min(o, 440)];
          if (o < 441) dst[(size_t)o * L] = vo;
        }
        wave_lds_sync();  // stage free again
      } else {
#pragma unroll
        for (int u = 0; u < kOutPerLane; u++) {
          const int o = lane + kWave * u;
          const int k = min(o % np, np - 1), t = o / np, yy = min(t % Dp, Dp - 1),
                    xx = min(t / Dp, Dp - 1);
          float r00, r01, r10, r11;
          tap4(k, yy, xx, mat, r00, r01, r10, r11);
          const float v = bil(k, r00, r01, r10, r11);
          if (o < nout) dst[(size_t)o * L] = v;
        }
      }
    };
    wave_lds_sync();  // geo visible
    if (!fast) {
      // windows too spread for the matrix path: raw[k][yy][xx] as fp32 dot
      // products straight from HBM into G, then the bilinear
      const float* f2 = static_cast<const float*>(LV_SEL(f2, lev)) +
                        ((size_t)b * N2 + (idx_ok ? jx : 0)) * H2 * W2 * C;
      const float* f1 = fmap1 + ((size_t)b * N1 + (idx_ok ? ix : 0)) * C * np;
      for (int e = lane; e < np * D * D; e += kWave) {
        const int k = e / (D * D), t = e % (D * D), yy = t / D, xx = t % D;
        const int i1 = geo->y0[k] + yy - R, j1 = geo->x0[k] + xx - R;
        float sacc = 0.f;
        if (idx_ok && i1 >= 0 && i1 < H2 && j1 >= 0 && j1 < W2) {
          const float* px = f2 + ((size_t)i1 * W2 + j1) * C;
          for (int c = 0; c < C; c++) sacc += f1[(size_t)c * np + k] * px[c];
        }
        G[e] = sacc;
      }
      wave_lds_sync();
      bilinear_store(false);
      wave_lds_sync();
      return;
    }

    // box tiles as whole lines: instruction h of tile t covers pixels
    // 16 t + 8 (h & 1) + (lane >> 3), 128-B quarter h >> 1, 16 B (lane & 7) each
    const int npx = max(bw * bh, 1), bw1 = max(bw, 1);
    const float* base = static_cast<const float*>(LV_SEL(f2, lev)) +
                        (((size_t)b * N2 + (idx_ok ? jx : 0)) * H2 * W2 +
                         (ntile > 0 ? (size_t)ylo * W2 + xlo : 0)) * C +
                        4 * (lane & 7);
    const int rowe = W2 * C;
    const float rbw = 1.0f / (float)bw1;
    const float* base0 = static_cast<const float*>(LV_SEL(f2, lev));
    auto load_tile = [&](u32x4 (&d)[8], int t) __attribute__((always_inline)) {
      // past the end (ring refills, never used): every lane reads the same 16 B,
      // one line request per instruction instead of eight
      const bool past = t >= ntile;
      const float* s[2];
#pragma unroll
      for (int ph = 0; ph < 2; ph++) {
        const int px = min(16 * t + 8 * ph + (lane >> 3), npx - 1);  // pad lanes: pixel npx - 1
        const int r = (int)(((float)px + 0.5f) * rbw), cc = px - r * bw1;
        s[ph] = past ? base0 : base + r * rowe + cc * C;
      }
#pragma unroll
      for (int h = 0; h < 8; h++)
        d[h] = *reinterpret_cast<const gu32x4*>(reinterpret_cast<uintptr_t>(s[h & 1] + 32 * (h >> 1)));
    };
    u32x4 ring[RING][8];
    // unconditional preload (an empty box reads the frame's first pixel): the
    // waits below then count exactly
#pragma unroll
    for (int k = 0; k < RING; k++) {
      load_tile(ring[k], k);
      __builtin_amdgcn_sched_barrier(0);
    }

    // A fragments: lane (i = lane & 15, q = lane >> 4) holds patch row i,
    // channels 16 h + 4 q + s at a[4 h + s] (zero for rows i >= np)
    float a[32];
    {
#pragma unroll
      for (int r = 0; r < kPA; r++) reinterpret_cast<u32x4*>(G)[min(lane + kWave * r, n16 - 1)] = pa[r];
      wave_lds_sync();
      const bool arow = idx_ok && ai < np;
      const int fi = min(ai, np - 1);
#pragma unroll
      for (int h = 0; h < 8; h++)
#pragma unroll
        for (int s = 0; s < 4; s++) {
          const float v = G[(16 * h + 4 * aq + s) * np + fi];
          a[4 * h + s] = arow ? v : 0.0f;
        }
      wave_lds_sync();  // G free again
    }

    // stage addresses: a lane writes its 16 B of pixel pt = 8 ph + (lane >> 3),
    // chunk c = lane & 7 at pt * 128 + ((c ^ (pt & 7)) * 16); B fragment of
    // lane (n, q), half j of the quarter: chunk 4 j + q of pixel n
    const int wr0 = (lane >> 3) * 128 + (((lane & 7) ^ (lane >> 3)) << 4);
    const int rd0 = ai * 128 + ((aq ^ (ai & 7)) << 4), rd1 = ai * 128 + (((4 + aq) ^ (ai & 7)) << 4);
    auto step = [&](u32x4 (&cur)[8], int t) __attribute__((always_inline)) {
      const bool live = t < ntile;
      f32x4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
      if (live) {
#pragma unroll
        for (int qt = 0; qt < 4; qt++) {
          *reinterpret_cast<u32x4*>(stage + wr0) = cur[2 * qt];
          *reinterpret_cast<u32x4*>(stage + 1024 + wr0) = cur[2 * qt + 1];
          const float4 b0 = *reinterpret_cast<const float4*>(stage + rd0);
          const float4 b1 = *reinterpret_cast<const float4*>(stage + rd1);
          const float bb[8] = {b0.x, b0.y, b0.z, b0.w, b1.x, b1.y, b1.z, b1.w};
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

  if (w < L) {
    const int pA = x8 * per + j8, pB = pA + half;
    const int lim = order ? min(per * (x8 + 1), M) : nE;
    if (pA < lim) run_unit(pA, w);
    if (pB < lim && pB < x8 * per + per) run_unit(pB, L - 1 - w);
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
  // G: np rows x kBoxStride per wave (the slow path's np x D x D fits too:
  // D * D <= 256 > kBoxStride only for R > 5, which the fast path covers)
  const int D = 2 * radius + 2;
  if (D * D > kBoxStride) return DPVO_ERR_UNSUPPORTED;
  const bool ordered = order && B == 1;
  const int* ord = ordered ? (const int*)order : (const int*)nullptr;
  hipStream_t st = as_stream(stream);
  if (dtype == DPVO_F32) {
    // fp32: one wave per (edge, level) unit, two units per wave, whole-line
    // tiles, exact fp32 products
    const size_t lsm = (size_t)L * corr_lvl_wave_bytes(np);
    const unsigned per = ordered ? (unsigned)((M + 7) / 8) : (unsigned)(B * M);
    const unsigned lg = ordered ? 8u * ((per + 1) / 2) : (per + 1) / 2;
    const dim3 g(lg), blk(L * kWave);
    if (np == 9 && radius == 3)
      hipLaunchKernelGGL((corr_nhwc_lvl_kernel<2, true>), g, blk, lsm, st, (const float*)fmap1, lv,
                         L, coords, ii, jj, B, M, np, N1, N2, radius, ord, out);
    else
      hipLaunchKernelGGL((corr_nhwc_lvl_kernel<2, false>), g, blk, lsm, st, (const float*)fmap1, lv,
                         L, coords, ii, jj, B, M, np, N1, N2, radius, ord, out);
    return launch_status();
  }
  const size_t smem = corr_nhwc_lds_bytes(np, radius, L);
  const long long units = (long long)B * M;
  unsigned grid = (unsigned)((units + kNhwcWaves - 1) / kNhwcWaves);
  if (ordered) grid = 8u * (unsigned)((grid + 7) / 8);
  const bool raw9 = np == 9 && radius == 3;  // DPVO: p = 3, R = 3
  const dim3 g(grid), blk(kNhwcWaves * kWave);
  const __half* f1 = (const __half*)fmap1;
  if (raw9)
    hipLaunchKernelGGL((corr_nhwc_kernel<__half, true>), g, blk, smem, st, f1, lv, L, coords, ii,
                       jj, B, M, np, N1, N2, radius, ord, out);
  else
    hipLaunchKernelGGL((corr_nhwc_kernel<__half, false>), g, blk, smem, st, f1, lv, L, coords, ii,
                       jj, B, M, np, N1, N2, radius, ord, out);
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
