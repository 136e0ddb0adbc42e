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
// bounding box of the edge's windows) runs on the matrix cores:
// v_mfma_f32_16x16x4_f32 with A = f1 (16 rows >= p*p, loaded once per edge
// and shared by every level), B = 16 box pixels x 4 channels straight from
// HBM as one 16-B load per lane (a lane's float4 holds 4 channels = 4
// consecutive K steps), D = G tile -> LDS.  One wave per edge handles every
// level; the bilinear + permute of all levels is kept in registers and
// stored once per edge as contiguous [.., L] float4 rows.
#include "common.hpp"

namespace dpvo {

constexpr int kNhwcWaves = 4;   // edges per workgroup
constexpr int kNhwcC = 128;     // channels (DPVO gmap / fmap width)
constexpr int kMaxTiles = 10;   // box up to 160 pixels through the matrix path
constexpr int kBoxStride = 16 * kMaxTiles;
constexpr int kMaxL = 4;        // levels per launch
constexpr int kOutPerLane = 8;  // (2R+1)^2 * p*p <= 512 outputs per level
constexpr int kNpMax = 16;      // p*p <= 16 (one MFMA row tile)

struct NhwcLevels {
  const float* f2[kMaxL];
  int H2[kMaxL], W2[kMaxL];
  float scale[kMaxL];
};

struct NhwcGeom {
  int x0[kNpMax], y0[kNpMax];
  float dx[kNpMax], dy[kNpMax];
};

typedef float f32x4 __attribute__((ext_vector_type(4)));

__global__ void __launch_bounds__(kNhwcWaves* kWave)
    corr_nhwc_kernel(const float* __restrict__ fmap1, NhwcLevels lv, int L,
                     const float* __restrict__ coords, const int64_t* __restrict__ ii,
                     const int64_t* __restrict__ jj, int B, int M, int np, int N1, int N2, int R,
                     float* __restrict__ out) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int wid = wave_uniform(threadIdx.x / kWave), lane = threadIdx.x & (kWave - 1);
  float* G = smem + wid * (kNpMax * kBoxStride);
  NhwcGeom* geo = reinterpret_cast<NhwcGeom*>(smem + kNhwcWaves * kNpMax * kBoxStride) + wid;
  const int unit = blockIdx.x * kNhwcWaves + wid;
  if (unit >= B * M) return;  // waves are independent: no block barrier below
  const int b = unit / M, m = unit % M;
  const int ix = wave_uniform((int)ii[m]), jx = wave_uniform((int)jj[m]);
  const bool idx_ok = ix >= 0 && ix < N1 && jx >= 0 && jx < N2;
  const int C = kNhwcC, D = 2 * R + 2, Dp = D - 1, nout = Dp * Dp * np;

  // ---- A fragments: lane (i = lane & 15, q = lane >> 4) holds f1[c][i] for
  // c = 16h + 4q + s at K step 4h + s (the same channel order as the B loads)
  const int ai = lane & 15, aq = lane >> 4;
  float Af[kNhwcC / 4];
  {
    const float* f1 = fmap1 + ((size_t)b * N1 + (idx_ok ? ix : 0)) * C * np;
    const bool arow = idx_ok && ai < np;
#pragma unroll
    for (int h = 0; h < kNhwcC / 16; h++)
#pragma unroll
      for (int s = 0; s < 4; s++)
        Af[4 * h + s] = arow ? f1[(size_t)(16 * h + 4 * aq + s) * np + ai] : 0.0f;
  }

  float outv[kOutPerLane][kMaxL];
  for (int l = 0; l < L; l++) {
    const int H2 = lv.H2[l], W2 = lv.W2[l];
    // ---- geometry: coords [B,M,2,np] / scale -> floor / frac per patch pixel
    float cv = 0.f;
    if (lane < 2 * np) cv = coords[((size_t)b * M + m) * 2 * np + lane] / lv.scale[l];
    int xlo = 0x7fffffff, xhi = -0x7fffffff, ylo = 0x7fffffff, yhi = -0x7fffffff;
#pragma unroll
    for (int k = 0; k < kNpMax; k++) {
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
    xlo = wave_uniform(max(xlo - R, 0));
    ylo = wave_uniform(max(ylo - R, 0));
    xhi = wave_uniform(min(xhi + R + 1, W2 - 1));
    yhi = wave_uniform(min(yhi + R + 1, H2 - 1));
    int bw = xhi - xlo + 1, bh = yhi - ylo + 1;
    if (bw <= 0 || bh <= 0 || !idx_ok) bw = bh = 0;
    const int npx = bw * bh, ntile = (npx + 15) >> 4;
    const bool fast = ntile <= kMaxTiles;
    const float* f2 = lv.f2[l] + ((size_t)b * N2 + (idx_ok ? jx : 0)) * H2 * W2 * C;
    wave_lds_sync();  // geo visible; previous level's G reads done

    if (fast) {
      // ---- G tile t: 16 box pixels x 128 channels, 8 x 16-B loads per lane
      auto tile_src = [&](int t) -> const float* {
        const int j = min(16 * t + ai, max(npx - 1, 0));  // pad columns read pixel npx-1
        const int r = j / max(bw, 1), cc = j - r * max(bw, 1);
        return f2 + ((size_t)(ylo + r) * W2 + xlo + cc) * C + 4 * aq;
      };
      float4 cur[8], nxt[8];
      if (ntile > 0) {
        const float* src = tile_src(0);
#pragma unroll
        for (int h = 0; h < 8; h++) cur[h] = *reinterpret_cast<const float4*>(src + 16 * h);
      }
      for (int t = 0; t < ntile; t++) {
        if (t + 1 < ntile) {  // next tile in flight while this one multiplies
          const float* src = tile_src(t + 1);
#pragma unroll
          for (int h = 0; h < 8; h++) nxt[h] = *reinterpret_cast<const float4*>(src + 16 * h);
        }
        f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int h = 0; h < 8; h++) {
          acc = __builtin_amdgcn_mfma_f32_16x16x4f32(Af[4 * h + 0], cur[h].x, acc, 0, 0, 0);
          acc = __builtin_amdgcn_mfma_f32_16x16x4f32(Af[4 * h + 1], cur[h].y, acc, 0, 0, 0);
          acc = __builtin_amdgcn_mfma_f32_16x16x4f32(Af[4 * h + 2], cur[h].z, acc, 0, 0, 0);
          acc = __builtin_amdgcn_mfma_f32_16x16x4f32(Af[4 * h + 3], cur[h].w, acc, 0, 0, 0);
        }
        // D: lane holds rows 4q + r (patch pixels), column lane & 15 (box pixel)
#pragma unroll
        for (int r = 0; r < 4; r++) {
          const int row = 4 * aq + r;
          if (row < np) G[row * kBoxStride + 16 * t + ai] = acc[r];
        }
#pragma unroll
        for (int h = 0; h < 8; h++) cur[h] = nxt[h];
      }
    } else {
      // ---- rare: windows too spread for the box: raw[k][yy][xx] directly
      for (int e = lane; e < np * D * D; e += kWave) {
        const int k = e / (D * D), t = e % (D * D), yy = t / D, xx = t % D;
        const int i1 = geo->y0[k] + yy - R, j1 = geo->x0[k] + xx - R;
        float s = 0.f;
        if (i1 >= 0 && i1 < H2 && j1 >= 0 && j1 < W2) {
          const float* px = f2 + ((size_t)i1 * W2 + j1) * C;
          const float* f1 = fmap1 + ((size_t)b * N1 + ix) * C * np;
          for (int c = 0; c < C; c++) s += f1[(size_t)c * np + k] * px[c];
        }
        G[e] = s;
      }
    }
    wave_lds_sync();

    // ---- bilinear + permute (correlation_kernel.cu:260-271) into registers
#pragma unroll
    for (int u = 0; u < kOutPerLane; u++) {
      const int o = lane + kWave * u;
      float v = 0.f;
      if (o < nout) {
        const int k = o % np, t = o / np, yy = t % Dp, xx = t / Dp;
        float r00, r01, r10, r11;
        if (fast) {
          const int gy = geo->y0[k] + yy - R - ylo, gx = geo->x0[k] + xx - R - xlo;
          const float* g = G + k * kBoxStride;
          auto at = [&](int y, int x) -> float {
            return (y >= 0 && y < bh && x >= 0 && x < bw) ? g[y * bw + x] : 0.f;
          };
          r00 = at(gy, gx);
          r01 = at(gy, gx + 1);
          r10 = at(gy + 1, gx);
          r11 = at(gy + 1, gx + 1);
        } else {
          const float* g = G + k * D * D;
          r00 = g[yy * D + xx];
          r01 = g[yy * D + xx + 1];
          r10 = g[(yy + 1) * D + xx];
          r11 = g[(yy + 1) * D + xx + 1];
        }
        const float dx = geo->dx[k], dy = geo->dy[k];
        v = ((1.f - dx) * (1.f - dy)) * r00;
        v = v + (dx * (1.f - dy)) * r01;
        v = v + ((1.f - dx) * dy) * r10;
        v = v + (dx * dy) * r11;
      }
#pragma unroll
      for (int ll = 0; ll < kMaxL; ll++)
        if (ll == l) outv[u][ll] = v;
    }
  }
  // ---- one contiguous [nout][L] row block per edge
  float* dst = out + ((size_t)b * M + m) * nout * L;
#pragma unroll
  for (int u = 0; u < kOutPerLane; u++) {
    const int o = lane + kWave * u;
    if (o >= nout) continue;
    if (L == 4) {
      *reinterpret_cast<float4*>(dst + (size_t)o * 4) =
          make_float4(outv[u][0], outv[u][1], outv[u][2], outv[u][3]);
    } else if (L == 2) {
      *reinterpret_cast<float2*>(dst + (size_t)o * 2) = make_float2(outv[u][0], outv[u][1]);
    } else {
#pragma unroll
      for (int ll = 0; ll < kMaxL; ll++)
        if (ll < L) dst[(size_t)o * L + ll] = outv[u][ll];
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
constexpr int kInsTY = 8, kInsTX = 32, kInsTC = 32;
constexpr int kInsCS = kInsTY * kInsTX + 1;  // channel stride (+1: no bank conflicts)

struct InsLevels {
  float* dst[kMaxL];
  int s[kMaxL];
};

// level-1 copy of the LDS tile: one float4 (4 channels) per lane, 8 lanes per
// pixel = one 128-B run of the channels-last row
__device__ __forceinline__ void ins_copy(const float* tile, float* dstl, int tx0, int ty0,
                                         int c0, int C, int H, int W, int tid) {
  for (int it = tid; it < kInsTY * kInsTX * 8; it += 256) {
    const int cg = it & 7, q = it >> 3, py = q / kInsTX, px = q % kInsTX;
    const int oy = ty0 + py, ox = tx0 + px, gc = c0 + 4 * cg;
    if (oy >= H || ox >= W || gc >= C) continue;
    const float* t = tile + (4 * cg) * kInsCS + py * kInsTX + px;
    float* dst = dstl + ((size_t)oy * W + ox) * C + gc;
    if (gc + 4 <= C && (C & 3) == 0) {
      *reinterpret_cast<float4*>(dst) =
          make_float4(t[0], t[kInsCS], t[2 * kInsCS], t[3 * kInsCS]);
    } else {
      for (int k = 0; k < 4 && gc + k < C; k++) dst[k] = t[k * kInsCS];
    }
  }
}

// pooled level S (avg_pool2d kernel = stride = S): one channel per lane, 32
// lanes per pixel (a 128-B run); the S*S window is summed in avg_pool2d's
// row-major order and divided by S^2, fully unrolled so the LDS reads issue
// back to back (bit-exact with torch)
template <int S>
__device__ __forceinline__ void ins_pool(const float* tile, float* dstl, int tx0, int ty0,
                                         int c0, int C, int H, int W, int tid) {
  constexpr int nty = kInsTY / S, ntx = kInsTX / S;
  const int Hs = H / S, Ws = W / S, oy0 = ty0 / S, ox0 = tx0 / S;
  for (int it = tid; it < nty * ntx * kInsTC; it += 256) {
    const int c = it & (kInsTC - 1), q = it / kInsTC, py = q / ntx, px = q % ntx;
    const int oy = oy0 + py, ox = ox0 + px, gc = c0 + c;
    if (oy >= Hs || ox >= Ws || gc >= C) continue;
    const float* t = tile + c * kInsCS + py * S * kInsTX + px * S;
    float w[S * S];
#pragma unroll
    for (int a = 0; a < S; a++)
#pragma unroll
      for (int b = 0; b < S; b++) w[a * S + b] = t[a * kInsTX + b];
    float acc = 0.0f;
#pragma unroll
    for (int k = 0; k < S * S; k++) acc += w[k];
    dstl[((size_t)oy * Ws + ox) * C + gc] = acc / (float)(S * S);
  }
}

__global__ void __launch_bounds__(256)
    pyramid_insert_kernel(const float* __restrict__ src, InsLevels lv, int L, int C, int H,
                          int W) {
  __shared__ float tile[kInsTC * kInsCS];
  const int tx0 = blockIdx.x * kInsTX, ty0 = blockIdx.y * kInsTY, c0 = blockIdx.z * kInsTC;
  const int tid = threadIdx.x;
  // load: 32 channels x 8 rows x 32 px as float4 (8 per thread, all issued
  // before the first LDS store: one HBM latency per tile, not eight)
  if ((W & 3) == 0) {
    float4 v[8];
#pragma unroll
    for (int r = 0; r < 8; r++) {
      const int k = tid + 256 * r;  // (c, y, x4) = (k >> 6, (k >> 3) & 7, k & 7)
      const int c = k >> 6, y = (k >> 3) & 7, x = 4 * (k & 7);
      const int gx = tx0 + x, gy = ty0 + y, gc = c0 + c;
      v[r] = (gx < W && gy < H && gc < C)
                 ? *reinterpret_cast<const float4*>(src + ((size_t)gc * H + gy) * W + gx)
                 : make_float4(0.f, 0.f, 0.f, 0.f);
    }
#pragma unroll
    for (int r = 0; r < 8; r++) {
      const int k = tid + 256 * r;
      const int c = k >> 6, y = (k >> 3) & 7, x = 4 * (k & 7);
      float* t = tile + c * kInsCS + y * kInsTX + x;
      t[0] = v[r].x;
      t[1] = v[r].y;
      t[2] = v[r].z;
      t[3] = v[r].w;
    }
  } else {
    float v[32];
#pragma unroll
    for (int r = 0; r < 32; r++) {
      const int k = tid + 256 * r;
      const int x = k & 31, y = (k >> 5) & 7, c = k >> 8;
      const int gx = tx0 + x, gy = ty0 + y, gc = c0 + c;
      v[r] = (gx < W && gy < H && gc < C) ? src[((size_t)gc * H + gy) * W + gx] : 0.0f;
    }
#pragma unroll
    for (int r = 0; r < 32; r++) {
      const int k = tid + 256 * r;
      tile[(k >> 8) * kInsCS + ((k >> 5) & 7) * kInsTX + (k & 31)] = v[r];
    }
  }
  __syncthreads();
  // level 1: one float4 (4 channels) per lane, 8 lanes per pixel = one 128-B run
  for (int l = 0; l < L; l++) {
    switch (lv.s[l]) {
      case 1: ins_copy(tile, lv.dst[l], tx0, ty0, c0, C, H, W, tid); break;
      case 2: ins_pool<2>(tile, lv.dst[l], tx0, ty0, c0, C, H, W, tid); break;
      case 4: ins_pool<4>(tile, lv.dst[l], tx0, ty0, c0, C, H, W, tid); break;
      default: ins_pool<8>(tile, lv.dst[l], tx0, ty0, c0, C, H, W, tid); break;
    }
  }
}

}  // namespace dpvo

using namespace dpvo;

DPVO_EXPORT int dpvo_corr_forward_levels_nhwc(const void* fmap1, const void* const* fmap2,
                                              const int* H2, const int* W2, const float* scale,
                                              int L, const float* coords, const int64_t* ii,
                                              const int64_t* jj, int B, int M, int C, int H,
                                              int W, int N1, int N2, int radius, int dtype,
                                              float* out, void* stream) {
  if (L <= 0 || radius < 0 || radius > 7 || C <= 0 || H <= 0 || W <= 0) return DPVO_ERR_INVALID;
  const int np = H * W, Dp = 2 * radius + 1;
  if (dtype != DPVO_F32 || C != kNhwcC || L > kMaxL || np > kNpMax ||
      Dp * Dp * np > kOutPerLane * kWave)
    return DPVO_ERR_UNSUPPORTED;
  if (B * M == 0) return DPVO_OK;
  if (!fmap1 || !coords || !ii || !jj || !out) return DPVO_ERR_INVALID;
  NhwcLevels lv = {};
  for (int l = 0; l < L; l++) {
    if (!fmap2[l] || H2[l] <= 0 || W2[l] <= 0 || !(scale[l] > 0.f)) return DPVO_ERR_INVALID;
    lv.f2[l] = (const float*)fmap2[l];
    lv.H2[l] = H2[l];
    lv.W2[l] = W2[l];
    lv.scale[l] = scale[l];
  }
  const size_t smem = sizeof(float) * kNhwcWaves * kNpMax * kBoxStride +
                      sizeof(NhwcGeom) * kNhwcWaves;
  hipLaunchKernelGGL(corr_nhwc_kernel, dim3((B * M + kNhwcWaves - 1) / kNhwcWaves),
                     dim3(kNhwcWaves * kWave), smem, as_stream(stream), (const float*)fmap1, lv,
                     L, coords, ii, jj, B, M, np, N1, N2, radius, out);
  return launch_status();
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

DPVO_EXPORT int dpvo_feature_pyramid_insert(const void* src, void* const* dst, const int* scale,
                                            int L, int C, int H, int W, int dtype, void* stream) {
  if (!src || !dst || !scale || L <= 0 || C <= 0 || H <= 0 || W <= 0) return DPVO_ERR_INVALID;
  if (dtype != DPVO_F32 || L > kMaxL) return DPVO_ERR_UNSUPPORTED;
  InsLevels lv = {};
  for (int l = 0; l < L; l++) {
    const int s = scale[l];
    if (!dst[l]) return DPVO_ERR_INVALID;
    if (s != 1 && s != 2 && s != 4 && s != 8) return DPVO_ERR_UNSUPPORTED;
    lv.dst[l] = (float*)dst[l];
    lv.s[l] = s;
  }
  const dim3 grid((W + kInsTX - 1) / kInsTX, (H + kInsTY - 1) / kInsTY, (C + kInsTC - 1) / kInsTC);
  hipLaunchKernelGGL(pyramid_insert_kernel, grid, dim3(256), 0, as_stream(stream),
                     (const float*)src, lv, L, C, H, W);
  return launch_status();
}
