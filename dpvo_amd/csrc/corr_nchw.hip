// corr_nchw.hip -- A-CORR on the matrix cores for NCHW feature maps (fp16 and
// fp32): the layout DPVO allocates (dpvo.py:111-112, fp16 under its default
// MIXED_PRECISION runtime, fp32 without it), behind the unchanged per-level entry
// (correlation.cpp:32-38 -> cuda_corr.forward, called per level at
// dpvo.py:462-465) and the fused multi-level one.
//
// Same semantics as corr.hip (correlation_kernel.cu:82-175 + 232-272) and the
// same per-edge GEMM as corr_nhwc.hip,
//     G[k][px] = sum_c f1[c][k] * f2[c][px]     over the union box of the
// edge's p*p windows, but a channel-plane box row is only ~10 contiguous
// halves, so a B fragment (8 channels of one pixel per lane) cannot come
// straight from HBM.  Each wave (one edge, one level):
//   * loads the box 32 channels at a time: per channel, bh rows x npr aligned
//     pieces of G halves (16-B pieces when W2 % 8 == 0, 8-B when W2 % 4 == 0);
//     one load instruction takes the whole box of 2 channels (16-B pieces) or
//     1 channel (8-B pieces), lane = (channel, row, piece): the lines a box
//     row needs are shared by the lanes of the row.  (Lane = (channel, row
//     parity), every lane on its own 128-B line, made the level-1 call 1.6x
//     slower: the line requests, not the bytes, bound the load path);
//   * writes them to an LDS image [32 channels][P pixels], P = bh x Wp
//     (Wp = npr x G) padded to an ODD number of 16-pixel tiles;
//   * reads B fragments with ds_read_b64_tr_b16 (gfx950's transposing LDS
//     read: a 16-lane group receives 4 channel rows x 16 pixels one pixel per
//     lane, i.e. the channel-major image arrives in the MFMA's k-per-lane
//     layout).  The 8 channel rows one 32-lane half reads are P/2 = 8 x odd
//     dwords apart, so they fall on 8 disjoint 8-bank groups: conflict-free;
//   * multiplies with v_mfma_f32_16x16x32_f16 (fp32 accumulation, the
//     documented deviation of every fp16 path here), one accumulator tile per
//     16 image pixels (pad pixels produce columns nobody reads);
//   * while the next 32-channel chunk's loads are in flight;
//   * then the bilinear + permute from G in LDS, as corr.hip.
// K order of one 32-channel chunk u: lane group g (= lane >> 4) holds, in
// element j of its fragment, channel 32u + 4g + j (j < 4) or 32u + 16 + 4g +
// j - 4 (j >= 4) -- the rows of its two transposed reads -- in both the A
// (gmap patch) and the B (box) fragment.
// fp32 features: the same image holds 16 channels (the same bytes), B comes
// back with plain ds_read_b32 (lane (n, q): channel 4s + q, pixel n) and
// v_mfma_f32_16x16x4_f32 forms exact fp32 products (K step s: channels
// 16u + 4s .. + 3); 8 chunks per level.
#include "common.hpp"

namespace dpvo {
namespace {

constexpr int kNcWaves = 4;      // edges per workgroup
constexpr int kNcC = 128;        // channels (DPVO fmap width)
constexpr int kNcImgElemBytes = 64;  // channels per LDS image x element bytes
constexpr int kNcMaxTiles = 17;  // odd; box image <= 272 px
constexpr int kNcMaxPx = 16 * kNcMaxTiles;
constexpr int kNcNpMax = 16;     // p * p <= 16 (one MFMA row tile)
constexpr int kNcMaxL = 4;
// per wave: the image (32 fp16 / 16 fp32 channels x P; reused as G: np x P
// floats <= 16 x 272, or the slow path's np x D x D <= 16 x 256) + geometry
constexpr int kNcImgBytes = kNcImgElemBytes * kNcMaxPx;

struct NcLevels {
  const void* f2[kNcMaxL];  // [B, N2, C, H2, W2] (__half or float)
  int H2[kNcMaxL], W2[kNcMaxL], pb[kNcMaxL];  // pb: widest piece in bytes (16 or 8)
  float scale[kNcMaxL];
};

struct NcGeom {
  int x0[kNcNpMax], y0[kNcNpMax];
  float dx[kNcNpMax], dy[kNcNpMax];
};
constexpr int kNcWaveBytes = kNcImgBytes + (int)sizeof(NcGeom);
static_assert(kNcWaveBytes % 16 == 0, "per-wave LDS carve must keep 16-B alignment");

typedef _Float16 h4 __attribute__((ext_vector_type(4)));
typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef short s4 __attribute__((ext_vector_type(4)));
typedef float f4 __attribute__((ext_vector_type(4)));
typedef unsigned u2 __attribute__((ext_vector_type(2)));
typedef unsigned u4 __attribute__((ext_vector_type(4)));

template <int PB>
struct NcPiece;
template <>
struct NcPiece<16> { typedef u4 type; };
template <>
struct NcPiece<8> { typedef u2 type; };

// global-address-space load (a generic pointer would be a flat load, counted
// in both vmcnt and lgkmcnt)
template <typename V>
__device__ __forceinline__ V ldg(const void* p) {
  return *reinterpret_cast<const __attribute__((address_space(1))) V*>(reinterpret_cast<uintptr_t>(p));
}

__device__ __forceinline__ h4 tr_read(const char* lds) {
  const s4 v = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (__attribute__((address_space(3))) s4*)(lds));
  return __builtin_bit_cast(h4, v);
}

template <typename X>
__device__ __forceinline__ X nc_sel(int l, X a, X b, X c, X d) {
  return l == 0 ? a : l == 1 ? b : l == 2 ? c : d;
}

// The matrix-core part of one edge at one level: G[k][px] for every image
// pixel into Gs (np rows of P floats).  T: __half or float; PB: piece bytes
// (16 or 8); CH: channels per load instruction (2: the box fits 32 lanes).
template <typename T, int PB, int CH>
__device__ __forceinline__ void nc_fast(const T* __restrict__ fmap1, const T* __restrict__ f2lvl,
                                        int H2, int W2, int b, int ix, int jx, int np, int N1,
                                        int N2, int ylo, int bh, int xs, int npr, int Wp, int nt,
                                        char* wlds) {
  constexpr bool kHalf = std::is_same<T, __half>::value;
  constexpr int G = PB / (int)sizeof(T);                 // elements per piece
  constexpr int KC = kNcImgElemBytes / (int)sizeof(T);   // channels per image (32 / 16)
  constexpr int kChunks = kNcC / KC;
  constexpr int kLc = kWave / CH, kIns = KC / CH;        // lanes per channel, loads per chunk
  using PT = typename NcPiece<PB>::type;
  const int lane = threadIdx.x & (kWave - 1);
  float* Gs = reinterpret_cast<float*>(wlds);
  const int P = nt * 16;
  const size_t HW2 = (size_t)H2 * W2;
  const T* f2 = f2lvl + ((size_t)b * N2 + jx) * kNcC * HW2;
  const T* f1 = fmap1 + ((size_t)b * N1 + ix) * kNcC * np;
  // per-lane piece (fixed for every chunk and instruction): an instruction
  // then touches CH x bh x (1-2) 128-B lines, not one line per lane
  const int pidx = lane % kLc, pch = lane / kLc;
  const bool pv = pidx < bh * npr;
  const int prow = pv ? pidx / npr : 0, ppc = pv ? pidx - prow * npr : 0;
  const T* src0 = f2 + (size_t)pch * HW2 + (size_t)(ylo + prow) * W2 + xs + ppc * G;
  PT buf[kIns];
  auto issue = [&](int u) __attribute__((always_inline)) {
    if (pv) {
      const T* su = src0 + (size_t)u * KC * HW2;
#pragma unroll
      for (int i = 0; i < kIns; i++) buf[i] = ldg<PT>(su + (size_t)(CH * i) * HW2);
    }
  };
  // the lane's piece in channel row 0 of the image
  char* wb = wlds + (size_t)(pch * P + prow * Wp + ppc * G) * sizeof(T);
  auto stage = [&]() __attribute__((always_inline)) {
    if (pv) {
#pragma unroll
      for (int i = 0; i < kIns; i++)
        *reinterpret_cast<PT*>(wb + (size_t)CH * i * P * sizeof(T)) = buf[i];
    }
  };

  // gmap patch [C][np] (16-B units, C * np * sizeof(T) is a multiple of 16) ->
  // LDS -> A fragments; its loads overlap chunk 0's
  constexpr int kPer16 = 16 / (int)sizeof(T);
  constexpr int kRA = (kNcC * kNcNpMax / kPer16 + kWave - 1) / kWave;
  const int n16 = kNcC * np / kPer16;
  u4 pa[kRA];
#pragma unroll
  for (int r = 0; r < kRA; r++) pa[r] = ldg<u4>(f1 + kPer16 * min(lane + kWave * r, n16 - 1));
  issue(0);
#pragma unroll
  for (int r = 0; r < kRA; r++)
    if (lane + kWave * r < n16) reinterpret_cast<u4*>(wlds)[lane + kWave * r] = pa[r];
  wave_lds_sync();
  const int g4 = lane >> 4, am = lane & 15;
  const bool arow = am < np;
  // A fragments: fp16 h8 per 32-channel chunk; fp32 one float per K step
  h8 Ah[kHalf ? kChunks : 1];
  float Af[kHalf ? 1 : kChunks * 4];
  if constexpr (kHalf) {
    const _Float16* ph = reinterpret_cast<const _Float16*>(wlds);
#pragma unroll
    for (int u = 0; u < kChunks; u++)
#pragma unroll
      for (int j = 0; j < 8; j++) {
        const int c = KC * u + (j < 4 ? 4 * g4 + j : 16 + 4 * g4 + j - 4);
        Ah[u][j] = arow ? ph[c * np + am] : (_Float16)0.0f;
      }
  } else {
    const float* pf = reinterpret_cast<const float*>(wlds);
#pragma unroll
    for (int u = 0; u < kChunks; u++)
#pragma unroll
      for (int s4 = 0; s4 < 4; s4++) {
        const int c = KC * u + 4 * s4 + g4;
        Af[4 * u + s4] = arow ? pf[c * np + am] : 0.0f;
      }
  }
  wave_lds_sync();  // patch read: the image may overwrite it

  // fp16: transposed-read address of lane (g4, row q' = (lane >> 2) & 3,
  // col 4 (lane & 3)); fp32: B of K step s from channel row 4 s + g4, pixel am
  const char* ta = kHalf ? wlds + ((4 * g4 + ((lane >> 2) & 3)) * P + 4 * (lane & 3)) * 2
                         : wlds + (g4 * P + am) * 4;
  const int ta1 = kHalf ? 16 * P * 2 : 4 * P * 4;  // fp16: rows 16 + 4 g4 + q'; fp32: next K step
  f4 acc[kNcMaxTiles];
#pragma unroll
  for (int t = 0; t < kNcMaxTiles; t++) acc[t] = (f4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int u = 0; u < kChunks; u++) {
    stage();
    wave_lds_sync();
    if (u + 1 < kChunks) issue(u + 1);
#pragma unroll
    for (int t = 0; t < kNcMaxTiles; t++) {
      if (t < nt) {
        if constexpr (kHalf) {
          const h4 b0 = tr_read(ta + 32 * t), b1 = tr_read(ta + ta1 + 32 * t);
          const h8 bb = __builtin_shufflevector(b0, b1, 0, 1, 2, 3, 4, 5, 6, 7);
          acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_f16(Ah[u], bb, acc[t], 0, 0, 0);
        } else {
          float bv[4];
#pragma unroll
          for (int s4 = 0; s4 < 4; s4++)
            bv[s4] = *reinterpret_cast<const float*>(ta + s4 * ta1 + 64 * t);
#pragma unroll
          for (int s4 = 0; s4 < 4; s4++)
            acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(Af[4 * u + s4], bv[s4], acc[t], 0, 0, 0);
        }
      }
    }
    wave_lds_sync();  // this chunk's reads before the next chunk's writes
  }
  // D tile t: lane (col n = lane & 15, rows 4 g4 + r) -> G[k][16 t + n]
#pragma unroll
  for (int t = 0; t < kNcMaxTiles; t++) {
    if (t < nt) {
#pragma unroll
      for (int r = 0; r < 4; r++) {
        const int k = 4 * g4 + r;
        if (k < np) Gs[k * P + 16 * t + am] = acc[t][r];
      }
    }
  }
}

// One edge at one level; pbmax = the level's widest piece in bytes (16 or 8).
template <typename T>
__device__ __forceinline__ void nc_edge(const T* __restrict__ fmap1, const T* __restrict__ f2lvl,
                                        int H2, int W2, int pbmax, float scale, bool use_scale,
                                        const float* __restrict__ coords, int b, int m, int ix,
                                        int jx, int M, int np, int N1, int N2, int R, char* wlds,
                                        T* __restrict__ out_t, float* __restrict__ out_f,
                                        int out_stride, int out_off) {
  const int lane = threadIdx.x & (kWave - 1);
  const int D = 2 * R + 2, Dp = D - 1;
  float* Gs = reinterpret_cast<float*>(wlds);
  NcGeom* geo = reinterpret_cast<NcGeom*>(wlds + kNcImgBytes);

  // ---- geometry: lane k < np takes patch pixel k (floor / frac) ----
  float cv = 0.f;
  if (lane < 2 * np) {
    cv = coords[((size_t)b * M + m) * 2 * np + lane];
    if (use_scale) cv = cv / scale;  // coords / scale (dpvo.py:462-463)
  }
  const float cy = __shfl(cv, min(lane + np, kWave - 1), kWave);
  int xf = 0x7fffffff, yf = 0x7fffffff, xg = -0x7fffffff, yg = -0x7fffffff;
  if (lane < np) {
    xf = xg = ifloor_safe(cv);
    yf = yg = ifloor_safe(cy);
    geo->x0[lane] = xf;
    geo->y0[lane] = yf;
    geo->dx[lane] = cv - floorf(cv);  // correlation_kernel.cu:262
    geo->dy[lane] = cy - floorf(cy);
  }
  // union bounding box of all windows, clipped to the map (wave-uniform)
  const int xlo = wave_uniform(max(wave_min_i(xf) - R, 0));
  const int ylo = wave_uniform(max(wave_min_i(yf) - R, 0));
  const int xhi = wave_uniform(min(wave_max_i(xg) + R + 1, W2 - 1));
  const int yhi = wave_uniform(min(wave_max_i(yg) + R + 1, H2 - 1));
  wave_lds_sync();
  const bool idx_ok = ix >= 0 && ix < N1 && jx >= 0 && jx < N2;
  int bw = xhi - xlo + 1, bh = yhi - ylo + 1;
  if (bw <= 0 || bh <= 0 || !idx_ok) bw = bh = 0;
  const int npx = bw * bh;
  // image geometry: rows start at the piece-aligned column xs <= xlo.  Load
  // shape: 16-B pieces and 2 channels per instruction when the box fits 32
  // lanes, else 16-B pieces and 1 channel, else 8-B pieces, else the raw path
  int xs = 0, npr = 0, Wp = 0, nt = 1, mode = 0;
  auto fits = [&](int pbytes, int lanes) {
    const int G = pbytes / (int)sizeof(T);
    xs = xlo & ~(G - 1);
    npr = (xhi - xs) / G + 1;  // pieces per box row
    Wp = npr * G;
    nt = ((bh * Wp + 15) >> 4) | 1;  // odd tile count (bank-conflict-free reads)
    return nt <= kNcMaxTiles && bh * npr <= lanes;
  };
  // (fp16 skips mode 2: 32 channels x 16 B per lane would be 128 VGPRs of loads)
  constexpr bool kHalf = std::is_same<T, __half>::value;
  if (npx > 0) {
    if (pbmax == 16 && fits(16, kWave / 2)) mode = 1;
    else if (!kHalf && pbmax == 16 && fits(16, kWave)) mode = 2;
    else if (fits(8, kWave)) mode = 3;
  }
  const bool fast = mode != 0;
  const int P = nt * 16;
  const int xoff = xlo - xs;
  const size_t HW2 = (size_t)H2 * W2;

  if (mode == 1) {
    nc_fast<T, 16, 2>(fmap1, f2lvl, H2, W2, b, ix, jx, np, N1, N2, ylo, bh, xs, npr, Wp, nt, wlds);
  } else if (!kHalf && mode == 2) {
    nc_fast<T, 16, 1>(fmap1, f2lvl, H2, W2, b, ix, jx, np, N1, N2, ylo, bh, xs, npr, Wp, nt, wlds);
  } else if (mode == 3) {
    nc_fast<T, 8, 1>(fmap1, f2lvl, H2, W2, b, ix, jx, np, N1, N2, ylo, bh, xs, npr, Wp, nt, wlds);
  } else if (npx > 0) {
    // ---- rare: windows too spread for the image; raw[k][yy][xx] directly ----
    const T* f2 = f2lvl + ((size_t)b * N2 + jx) * kNcC * HW2;
    const T* f1 = fmap1 + ((size_t)b * N1 + ix) * kNcC * np;
    const int nraw = np * D * D;
    for (int e = lane; e < nraw; e += kWave) {
      const int k = e / (D * D), t = e % (D * D), yy = t / D, xx = t % D;
      const int i1 = geo->y0[k] + yy - R, j1 = geo->x0[k] + xx - R;
      float s = 0.f;
      if (i1 >= 0 && i1 < H2 && j1 >= 0 && j1 < W2) {
        const T* p2 = f2 + (size_t)i1 * W2 + j1;
        for (int c = 0; c < kNcC; c++) s += to_acc(f1[c * np + k]) * to_acc(p2[(size_t)c * HW2]);
      }
      Gs[e] = s;
    }
  }
  wave_lds_sync();

  // ---- bilinear + permute, fused into the store (correlation_kernel.cu:260-271) ----
  const int total = Dp * Dp * np;
  const size_t ebase = ((size_t)b * M + m) * total;
  for (int o = lane; o < total; o += kWave) {
    const int k = o % np, t = o / np, yy = t % Dp, xx = t / Dp;
    float r00, r01, r10, r11;
    if (fast || npx == 0) {
      const int gy = geo->y0[k] + yy - R - ylo, gx = geo->x0[k] + xx - R - xlo;
      const float* g = Gs + k * P + xoff;
      auto at = [&](int y, int x) -> float {
        return (y >= 0 && y < bh && x >= 0 && x < bw) ? g[y * Wp + x] : 0.f;
      };
      r00 = at(gy, gx);
      r01 = at(gy, gx + 1);
      r10 = at(gy + 1, gx);
      r11 = at(gy + 1, gx + 1);
    } else {
      const float* g = Gs + k * D * D;
      r00 = g[yy * D + xx];
      r01 = g[yy * D + xx + 1];
      r10 = g[(yy + 1) * D + xx];
      r11 = g[(yy + 1) * D + xx + 1];
    }
    const float dx = geo->dx[k], dy = geo->dy[k];
    float v = ((1.f - dx) * (1.f - dy)) * r00;
    v = v + (dx * (1.f - dy)) * r01;
    v = v + ((1.f - dx) * dy) * r10;
    v = v + (dx * dy) * r11;
    if (out_t)
      out_t[ebase + o] = from_acc<T>(v);
    else
      out_f[(ebase + o) * out_stride + out_off] = v;
  }
  wave_lds_sync();
}

// ---- XCD-aware edge order, computed by every workgroup (no extra launch) ----
// Workgroups run on XCD blockIdx.x % 8 (round-robin dispatch, gridDim.x a
// multiple of 8).  XCD x takes the x-th eighth of the edges sorted by target
// frame (stable counting sort of jj), so the 128-B lines of a frame's channel
// planes are fetched into one XCD's L2 instead of every XCD's: an NCHW box row
// uses ~20 B of each line it touches, so re-fetching lines, not bytes, bounds
// the level-1 call (cfg2: 51 -> 28 us, scripts/nchw_order_probe.py).  The
// workgroup's chunk c holds sorted positions 4c .. 4c+3; thread t counts the
// edges of its contiguous slice of jj per target bin, a block scan of the
// counts gives the rank of every match, and the owner of each wanted rank
// writes its edge id.  Edge ids are a bijection of positions, so the results
// are those of the unordered launch (every edge writes only its own output).
constexpr int kOrdMaxE = 16384, kOrdMaxN2 = 2048;

__device__ __forceinline__ int ord_bin(int64_t v, int N2) {
  return (v >= 0 && v < N2) ? (int)v : N2;  // out-of-range indices: one last bin
}

// LDS scratch (the waves' areas, before any image): bin of every edge u16 [M],
// hist [N2 + 2] ints, wave totals, the wanted (bin, rank) pairs; sel [4] is
// outside the waves' areas (read after the last barrier)
__device__ __forceinline__ void nc_order(const int64_t* __restrict__ jj, int M, int N2, int c,
                                         char* smem, int* sel) {
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  constexpr int T = kNcWaves * kWave;
  const int nb = N2 + 1;
  unsigned short* ebin = reinterpret_cast<unsigned short*>(smem);  // [M]
  int* hist = reinterpret_cast<int*>(smem + 2 * ((M + 7) & ~7));   // [nb + 1]: counts -> starts
  int2* wtot = reinterpret_cast<int2*>(hist + ((nb + 2) & ~1));    // [kNcWaves]
  int* want = reinterpret_cast<int*>(wtot + kNcWaves);             // [8]
  for (int v = tid; v <= nb; v += T) hist[v] = 0;
  __syncthreads();
  for (int e = tid; e < M; e += T) {
    const int v = ord_bin(jj[e], N2);
    ebin[e] = (unsigned short)v;
    atomicAdd(&hist[v], 1);
  }
  __syncthreads();
  if (wid == 0) {  // exclusive scan of the bins by one wave, 64 at a time
    int carry = 0;
    for (int b0 = 0; b0 < nb; b0 += kWave) {
      const int bb = b0 + lane, v = bb < nb ? hist[bb] : 0;
      const int inc = wave_incl_sum(v);
      if (bb < nb) hist[bb] = carry + inc - v;
      carry += __builtin_amdgcn_readlane(inc, 63);
    }
    if (lane == 0) hist[nb] = carry;
  }
  __syncthreads();
  if (tid < kNcWaves) {  // bin and rank of position 4c + tid (binary search of the starts)
    const int p = 4 * c + tid;
    int lo = 0, hi = nb;  // largest b with start[b] <= p
    while (hi - lo > 1) {
      const int mid = (lo + hi) >> 1;
      if (hist[mid] <= p) lo = mid; else hi = mid;
    }
    want[2 * tid] = p < M ? lo : -1;
    want[2 * tid + 1] = p - hist[lo];
  }
  __syncthreads();
  int wb[kNcWaves];
#pragma unroll
  for (int w = 0; w < kNcWaves; w++) wb[w] = want[2 * w];
  // this thread's contiguous slice of the edges (rank = slices before + order
  // inside): matches of the 4 wanted bins, packed 16 bits each (<= M < 2^16)
  const int K = (M + T - 1) / T, e0 = min(tid * K, M), e1 = min(e0 + K, M);
  int c01 = 0, c23 = 0;
  for (int e = e0; e < e1; e++) {
    const int v = ebin[e];
    c01 += (v == wb[0] ? 1 : 0) + (v == wb[1] ? 1 << 16 : 0);
    c23 += (v == wb[2] ? 1 : 0) + (v == wb[3] ? 1 << 16 : 0);
  }
  const int i01 = wave_incl_sum(c01), i23 = wave_incl_sum(c23);
  if (lane == 63) wtot[wid] = make_int2(i01, i23);
  __syncthreads();
  int x01 = i01 - c01, x23 = i23 - c23;  // exclusive prefix over the block
  for (int w = 0; w < wid; w++) {
    x01 += wtot[w].x;
    x23 += wtot[w].y;
  }
#pragma unroll
  for (int w = 0; w < kNcWaves; w++) {
    const int pre = ((w < 2 ? x01 : x23) >> (16 * (w & 1))) & 0xffff;
    const int cnt = ((w < 2 ? c01 : c23) >> (16 * (w & 1))) & 0xffff;
    const int r = want[2 * w + 1];
    if (wb[w] >= 0 && r >= pre && r < pre + cnt) {  // exactly one thread
      int seen = pre;
      for (int e = e0; e < e1; e++)
        if (ebin[e] == wb[w]) {
          if (seen == r) sel[w] = e;
          ++seen;
        }
    }
    if (wb[w] < 0 && tid == 0) sel[w] = -1;
  }
  __syncthreads();
}

template <typename T>
__global__ void __launch_bounds__(kNcWaves* kWave, 2)  // 2 workgroups (8 waves) per CU
    corr_nchw_kernel(const T* __restrict__ fmap1, NcLevels lv, int use_scale,
                     const float* __restrict__ coords, const int64_t* __restrict__ ii,
                     const int64_t* __restrict__ jj, int B, int M, int np, int N1, int N2, int R,
                     int L, int ordered, T* __restrict__ out_t, float* __restrict__ out_f) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int wid = wave_uniform(threadIdx.x / kWave);
  char* wlds = smem + wid * kNcWaveBytes;
  int unit;
  if (ordered) {  // B == 1
    int* sel = reinterpret_cast<int*>(smem + kNcWaves * kNcWaveBytes);
    const int nwg = (M + kNcWaves - 1) / kNcWaves, per = (nwg + 7) / 8;
    const int c = (blockIdx.x % 8) * per + blockIdx.x / 8;
    if (c >= nwg) return;  // workgroup-uniform
    nc_order(jj, M, N2, c, smem, sel);
    unit = wave_uniform(sel[wid]);
    if (unit < 0) return;
  } else {
    unit = blockIdx.x * kNcWaves + wid;
    if (unit >= B * M) return;  // waves are independent: no block barrier below
  }
  const int l = blockIdx.y;
  const int b = unit / M, m = unit % M;
  const int ix = wave_uniform((int)ii[m]), jx = wave_uniform((int)jj[m]);
  const T* f2 = reinterpret_cast<const T*>(nc_sel(l, lv.f2[0], lv.f2[1], lv.f2[2], lv.f2[3]));
  const int H2 = nc_sel(l, lv.H2[0], lv.H2[1], lv.H2[2], lv.H2[3]);
  const int W2 = nc_sel(l, lv.W2[0], lv.W2[1], lv.W2[2], lv.W2[3]);
  const int pb = nc_sel(l, lv.pb[0], lv.pb[1], lv.pb[2], lv.pb[3]);
  const float s = nc_sel(l, lv.scale[0], lv.scale[1], lv.scale[2], lv.scale[3]);
  nc_edge<T>(fmap1, f2, H2, W2, pb, s, use_scale != 0, coords, b, m, ix, jx, M, np, N1, N2, R,
             wlds, out_t, out_f, L, l);
}

template <typename T>
int nc_launch(const void* fmap1, const NcLevels& lv, bool use_scale, const float* coords,
              const int64_t* ii, const int64_t* jj, int B, int M, int np, int N1, int N2, int R,
              int L, int ordered, void* out_t, float* out_f, hipStream_t s) {
  // 4 x 17.7 KB per workgroup (+ the order's 4 edge ids): above 64 KB, set
  // once per device; if the attribute cannot be set the caller's VALU kernel
  // runs instead (DPVO_ERR_UNSUPPORTED)
  static bool attr[kMaxDevices] = {};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= kMaxDevices) return DPVO_ERR_UNSUPPORTED;
  if (!attr[dev]) {
    if (hipFuncSetAttribute((const void*)corr_nchw_kernel<T>,
                            hipFuncAttributeMaxDynamicSharedMemorySize,
                            kNcWaves * kNcWaveBytes + 16) != hipSuccess) {
      (void)hipGetLastError();  // not sticky: report it here, not at a later launch
      return DPVO_ERR_UNSUPPORTED;
    }
    attr[dev] = true;
  }
  unsigned gx = (unsigned)(((long long)B * M + kNcWaves - 1) / kNcWaves);
  if (ordered) gx = 8u * ((gx + 7u) / 8u);
  const dim3 grid(gx, L), block(kNcWaves * kWave);
  hipLaunchKernelGGL(corr_nchw_kernel<T>, grid, block, (size_t)kNcWaves * kNcWaveBytes + 16, s,
                     (const T*)fmap1, lv, use_scale ? 1 : 0, coords, ii, jj, B, M, np, N1, N2, R,
                     L, ordered, (T*)out_t, out_f);
  return launch_status();
}

}  // namespace

// The matrix-core NCHW forward, or DPVO_ERR_UNSUPPORTED when the call is
// outside its shape (then the caller runs corr.hip's VALU kernel): fp16 or
// fp32, C = 128, p*p <= 16, L <= 4, every level with 8-B pieces at least
// (W2 and the base aligned to 8 B).  out_t: [B, M, Dp, Dp, p, p] in the fmap
// dtype (L = 1); else out_f [.., L] float32.
int corr_nchw_mma(const void* fmap1, const void* const* fmap2, const int* H2, const int* W2,
                  const float* scale, int L, bool use_scale, const float* coords,
                  const int64_t* ii, const int64_t* jj, int B, int M, int C, int np, int N1,
                  int N2, int R, int dtype, void* out_t, float* out_f, hipStream_t s) {
  if ((dtype != DPVO_F16 && dtype != DPVO_F32) || C != kNcC || np < 1 || np > kNcNpMax ||
      L < 1 || L > kNcMaxL || R < 0 || R > 7)
    return DPVO_ERR_UNSUPPORTED;
  if (out_t && L != 1) return DPVO_ERR_INVALID;
  if (reinterpret_cast<uintptr_t>(fmap1) % 16) return DPVO_ERR_UNSUPPORTED;
  const int es = dtype == DPVO_F16 ? 2 : 4;
  NcLevels lv = {};
  for (int l = 0; l < L; l++) {
    const uintptr_t p = reinterpret_cast<uintptr_t>(fmap2[l]);
    int pb = 0;  // widest piece whose alignment every row start keeps
    if ((W2[l] * es) % 16 == 0 && p % 16 == 0) pb = 16;
    else if ((W2[l] * es) % 8 == 0 && p % 8 == 0) pb = 8;
    if (!pb || H2[l] <= 0) return DPVO_ERR_UNSUPPORTED;
    lv.f2[l] = fmap2[l];
    lv.H2[l] = H2[l];
    lv.W2[l] = W2[l];
    lv.pb[l] = pb;
    lv.scale[l] = scale ? scale[l] : 1.0f;
  }
  if ((long long)B * M == 0) return DPVO_OK;
  // XCD-aware order for a single batch of a DPVO-sized graph, when some level's
  // ring is larger than the L2s together (8 x 4 MB): the order's prologue costs
  // ~6 us per workgroup and pays only where lines are re-fetched from the
  // Infinity Cache / HBM (cfg2 fp16 level 1, 177 MB: 51 -> 31 us; level 4,
  // 11 MB: 21 -> 23 us)
  size_t ring = 0;
  for (int l = 0; l < L; l++) {
    const size_t r = (size_t)N2 * kNcC * H2[l] * W2[l] * es;
    ring = r > ring ? r : ring;
  }
  const int ordered = B == 1 && M <= kOrdMaxE && N2 >= 1 && N2 <= kOrdMaxN2 &&
                      ring > ((size_t)32 << 20);
  if (dtype == DPVO_F16)
    return nc_launch<__half>(fmap1, lv, use_scale, coords, ii, jj, B, M, np, N1, N2, R, L,
                             ordered, out_t, out_f, s);
  return nc_launch<float>(fmap1, lv, use_scale, coords, ii, jj, B, M, np, N1, N2, R, L, ordered,
                          out_t, out_f, s);
}

}  // namespace dpvo
