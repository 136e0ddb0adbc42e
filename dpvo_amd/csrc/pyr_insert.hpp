// pyr_insert.hpp -- frame insertion of a channels-last feature pyramid
// (dpvo.py __call__: the level-1 fmap written into its ring slot and level s =
// avg_pool2d(fmap, s, s), net.py:411), as a per-tile device routine shared by
// the standalone insertion kernel (corr_nhwc.hip) and the fused start-of-update
// launch (ba_window.hip: insertion tiles beside the reprojection and the BA
// plan, which leave most CUs idle).
#pragma once

#include "common.hpp"

namespace dpvo {

constexpr int kInsMaxL = 4;  // levels per insertion
// 8 x 16 pixel x 32 channel tiles: 600 workgroups for a 160 x 120 x 128 frame, all
// resident at once (32 x 8 x 32 tiles gave 300: 1.2 rounds over 256 CUs, the tail
// round nearly empty)
constexpr int kInsTY = 8, kInsTX = 16, kInsTC = 32;
constexpr int kInsCS = kInsTY * kInsTX + 1;  // channel stride (+1: no bank conflicts)

struct InsLevels {
  void* dst[kInsMaxL];  // float or __half (the source's dtype)
  int s[kInsMaxL];
  // ring variant (graph-replayed frames): dst[l] is slot 0 of level l, the
  // slot is *slot_dev % mem, slots slot_bytes[l] apart; null = dst as given
  const int* slot_dev;
  int mem;
  long long slot_bytes[kInsMaxL];
};

// level-1 copy of the LDS tile: one float4 (4 channels) per lane, 8 lanes per
// pixel = one 128-B run of the channels-last row
// fp16 pyramids (MIXED_PRECISION): the tile holds the exact fp32 values of
// the halves, pools accumulate in fp32 and round once (torch's avg_pool2d
// accscalar_t path), copies are exact
__device__ __forceinline__ void st4(float* d, float a, float b, float c, float e) {
  *reinterpret_cast<float4*>(d) = make_float4(a, b, c, e);
}
__device__ __forceinline__ void st4(__half* d, float a, float b, float c, float e) {
  __half2 lo = __floats2half2_rn(a, b), hi = __floats2half2_rn(c, e);
  uint2 u;
  __builtin_memcpy(&u.x, &lo, 4);
  __builtin_memcpy(&u.y, &hi, 4);
  *reinterpret_cast<uint2*>(d) = u;
}
__device__ __forceinline__ void st1(float* d, float v) { *d = v; }
__device__ __forceinline__ void st1(__half* d, float v) { *d = __float2half_rn(v); }
__device__ __forceinline__ float4 ld4(const float* s) { return *reinterpret_cast<const float4*>(s); }
__device__ __forceinline__ float4 ld4(const __half* s) {
  const uint2 u = *reinterpret_cast<const uint2*>(s);
  __half2 lo, hi;
  __builtin_memcpy(&lo, &u.x, 4);
  __builtin_memcpy(&hi, &u.y, 4);
  const float2 a = __half22float2(lo), b = __half22float2(hi);
  return make_float4(a.x, a.y, b.x, b.y);
}

template <typename T>
__device__ __forceinline__ void ins_copy(const float* tile, T* dstl, int tx0, int ty0,
                                         int c0, int C, int H, int W, int tid) {
  for (int it = tid; it < kInsTY * kInsTX * 8; it += 256) {
    const int cg = it & 7, q = it >> 3, py = q / kInsTX, px = q % kInsTX;
    const int oy = ty0 + py, ox = tx0 + px, gc = c0 + 4 * cg;
    if (oy >= H || ox >= W || gc >= C) continue;
    const float* t = tile + (4 * cg) * kInsCS + py * kInsTX + px;
    T* dst = dstl + ((size_t)oy * W + ox) * C + gc;
    if (gc + 4 <= C && (C & 3) == 0) {
      st4(dst, t[0], t[kInsCS], t[2 * kInsCS], t[3 * kInsCS]);
    } else {
      for (int k = 0; k < 4 && gc + k < C; k++) st1(dst + k, t[k * kInsCS]);
    }
  }
}

// pooled level S (avg_pool2d kernel = stride = S): one channel per lane, 32
// lanes per pixel (a 128-B run); the S*S window is summed in avg_pool2d's
// row-major order and divided by S^2, fully unrolled so the LDS reads issue
// back to back (bit-exact with torch)
template <int S, typename T>
__device__ __forceinline__ void ins_pool(const float* tile, T* dstl, int tx0, int ty0,
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
    st1(dstl + ((size_t)oy * Ws + ox) * C + gc, acc / (float)(S * S));
  }
}

// One 8 x 16 pixel x 32 channel tile (bx, by, bz) by 256 threads (tid < 256)
// with `tile` (kInsTC * kInsCS floats of LDS).  Contains one __syncthreads():
// every thread of the workgroup calls it, `act` = false skips the work.
// Load: 32 channels x 8 rows x 16 px, 4 px per load (all issued before the
// first LDS store: one HBM latency per tile).
template <typename T>
__device__ __forceinline__ void ins_tile(const T* __restrict__ src, const InsLevels& lv, int L,
                                         int C, int H, int W, int bx, int by, int bz, int tid,
                                         bool act, float* tile) {
  const int tx0 = bx * kInsTX, ty0 = by * kInsTY, c0 = bz * kInsTC;
  constexpr int kX4 = kInsTX / 4, kV4 = kInsTC * kInsTY * kX4 / 256;
  constexpr int kV1 = kInsTC * kInsTY * kInsTX / 256;
  if ((W & 3) == 0) {
    float4 v[kV4];
#pragma unroll
    for (int r = 0; r < kV4; r++) {
      const int k = tid + 256 * r;  // (c, y, x4)
      const int c = k / (kInsTY * kX4), y = (k / kX4) % kInsTY, x = 4 * (k % kX4);
      const int gx = tx0 + x, gy = ty0 + y, gc = c0 + c;
      v[r] = (act && gx < W && gy < H && gc < C) ? ld4(src + ((size_t)gc * H + gy) * W + gx)
                                          : make_float4(0.f, 0.f, 0.f, 0.f);
    }
#pragma unroll
    for (int r = 0; r < kV4; r++) {
      const int k = tid + 256 * r;
      const int c = k / (kInsTY * kX4), y = (k / kX4) % kInsTY, x = 4 * (k % kX4);
      float* t = tile + c * kInsCS + y * kInsTX + x;
      t[0] = v[r].x;
      t[1] = v[r].y;
      t[2] = v[r].z;
      t[3] = v[r].w;
    }
  } else {
    float v[kV1];
#pragma unroll
    for (int r = 0; r < kV1; r++) {
      const int k = tid + 256 * r;
      const int x = k % kInsTX, y = (k / kInsTX) % kInsTY, c = k / (kInsTX * kInsTY);
      const int gx = tx0 + x, gy = ty0 + y, gc = c0 + c;
      v[r] = (act && gx < W && gy < H && gc < C) ? to_acc(src[((size_t)gc * H + gy) * W + gx])
                                                 : 0.0f;
    }
#pragma unroll
    for (int r = 0; r < kV1; r++) {
      const int k = tid + 256 * r;
      tile[(k / (kInsTX * kInsTY)) * kInsCS + ((k / kInsTX) % kInsTY) * kInsTX + (k % kInsTX)] = v[r];
    }
  }
  __syncthreads();
  if (!act) return;  // no barrier below
  // level 1: one float4 (4 channels) per lane, 8 lanes per pixel = one 128-B run
  const long long slot = lv.slot_dev ? (long long)(((*lv.slot_dev) % lv.mem + lv.mem) % lv.mem) : 0;
  for (int l = 0; l < L; l++) {
    T* d = reinterpret_cast<T*>(static_cast<char*>(lv.dst[l]) + slot * lv.slot_bytes[l]);
    switch (lv.s[l]) {
      case 1: ins_copy(tile, d, tx0, ty0, c0, C, H, W, tid); break;
      case 2: ins_pool<2>(tile, d, tx0, ty0, c0, C, H, W, tid); break;
      case 4: ins_pool<4>(tile, d, tx0, ty0, c0, C, H, W, tid); break;
      default: ins_pool<8>(tile, d, tx0, ty0, c0, C, H, W, tid); break;
    }
  }
}

}  // namespace dpvo
