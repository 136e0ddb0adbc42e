// Box-tile load patterns of A-CORR (cfg2 shape: 2048 edges x 4 levels, one
// wave per (edge, level), 160x120x128 fp32 channels-last level 1): the loads
// alone, consumed by an xor checksum, to separate the memory path from the
// compute.  Pattern 0: 16 pixels x 64 B per global_load_dwordx4 (the MFMA B
// layout: 16 line requests per KiB); pattern 1: 8 pixels x 128 B (whole
// lines, 8 per KiB); pattern 2: pattern 0 as buffer loads, ring refills past
// the last tile out of range (no memory traffic).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 scripts/micro/load_pattern.hip -o scripts/micro/load_pattern
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <random>
#include <vector>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef const __attribute__((address_space(1))) u32x4 gu32x4;

struct Lv {
  const float* f2[4];
  int H2[4], W2[4];
  float sc[4];
};

template <int PAT, int RING>
__global__ void __launch_bounds__(256) load_kernel(Lv lv, const float* __restrict__ coords,
                                                   const int64_t* __restrict__ jj,
                                                   const int* __restrict__ order, int M, int mem,
                                                   unsigned* __restrict__ out) {
  const int l = threadIdx.x / 64, lane = threadIdx.x & 63;
  const int per = (M + 7) / 8;
  const int chunk = (blockIdx.x % 8) * per + blockIdx.x / 8;
  if (chunk >= M) return;
  const int m = __builtin_amdgcn_readfirstlane(order[chunk]);
  const int jx = __builtin_amdgcn_readfirstlane((int)(jj[m] % mem));
  const float cv = lane < 18 ? coords[(size_t)m * 18 + lane] : 0.f;
  const float sc = l == 0 ? lv.sc[0] : l == 1 ? lv.sc[1] : l == 2 ? lv.sc[2] : lv.sc[3];
  const int H2 = l == 0 ? lv.H2[0] : l == 1 ? lv.H2[1] : l == 2 ? lv.H2[2] : lv.H2[3];
  const int W2 = l == 0 ? lv.W2[0] : l == 1 ? lv.W2[1] : l == 2 ? lv.W2[2] : lv.W2[3];
  const float* f2 = l == 0 ? lv.f2[0] : l == 1 ? lv.f2[1] : l == 2 ? lv.f2[2] : lv.f2[3];
  const int gk = lane & 15;
  const bool act = lane < 9;
  const float x = __shfl(cv, gk < 9 ? gk : 8) / sc, y = __shfl(cv, 9 + (gk < 9 ? gk : 8)) / sc;
  const int xf = (int)floorf(x), yf = (int)floorf(y);
  int lx = act ? xf : 1 << 30, ly = act ? yf : 1 << 30, hx = act ? xf : -(1 << 30), hy = act ? yf : -(1 << 30);
  for (int o = 8; o > 0; o >>= 1) {
    lx = min(lx, __shfl_xor(lx, o));
    ly = min(ly, __shfl_xor(ly, o));
    hx = max(hx, __shfl_xor(hx, o));
    hy = max(hy, __shfl_xor(hy, o));
  }
  const int xlo = __builtin_amdgcn_readfirstlane(max(lx - 3, 0)), ylo = __builtin_amdgcn_readfirstlane(max(ly - 3, 0));
  const int bw = __builtin_amdgcn_readfirstlane(min(hx + 4, W2 - 1) - xlo + 1);
  const int bh = __builtin_amdgcn_readfirstlane(min(hy + 4, H2 - 1) - ylo + 1);
  const int npx = max(bw * bh, 1), ntile = bw > 0 && bh > 0 ? (npx + 15) / 16 : 0;
  const float rbw = 1.0f / (float)max(bw, 1);
  const float* base = f2 + ((size_t)jx * H2 * W2 + (size_t)ylo * W2 + xlo) * 128;
  const int rowe = W2 * 128;
  unsigned acc = 0;
  // descriptor over the frame's level (buffer pattern)
  const size_t fbytes = (size_t)H2 * W2 * 512 - ((size_t)ylo * W2 + xlo) * 512;
  __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)base, 0, (int)min(fbytes, (size_t)0x7fffffff), 0x00020000);
  auto load = [&](u32x4 (&d)[8], int t) __attribute__((always_inline)) {
    if constexpr (PAT == 1) {
      // 8 pixels x 128 B per instruction: lane (p = lane >> 3, c = lane & 7);
      // tile t = 16 pixels x 512 B = 8 instructions (2 pixel halves x 4 line quarters)
      t = min(t, max(ntile - 1, 0));
#pragma unroll
      for (int h = 0; h < 8; h++) {
        const int px = min(16 * t + 8 * (h & 1) + (lane >> 3), npx - 1);
        const int r = (int)(((float)px + 0.5f) * rbw), cc = px - r * max(bw, 1);
        const float* s = base + r * rowe + cc * 128 + 32 * (h >> 1) + 4 * (lane & 7);
        d[h] = *reinterpret_cast<const gu32x4*>(reinterpret_cast<uintptr_t>(s));
      }
    } else {
      const bool past = t >= ntile;
      t = min(t, max(ntile - 1, 0));
      const int px = min(16 * t + (lane & 15), npx - 1);
      const int r = (int)(((float)px + 0.5f) * rbw), cc = px - r * max(bw, 1);
      const int off = (r * rowe + cc * 128 + 4 * (lane >> 4)) * 4;
#pragma unroll
      for (int h = 0; h < 8; h++) {
        if constexpr (PAT == 2) {
          const int o = past ? 0x7ffffff0 : off + 64 * h;
          d[h] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, o, 0, 0));
        } else {
          d[h] = *reinterpret_cast<const gu32x4*>(reinterpret_cast<uintptr_t>(
              reinterpret_cast<const char*>(base) + off + 64 * h));
        }
      }
    }
  };
  u32x4 ring[RING][8];
#pragma unroll
  for (int k = 0; k < RING; k++) load(ring[k], k);
  for (int t = 0; t < ntile; t += RING) {
#pragma unroll
    for (int k = 0; k < RING; k++) {
      if (t + k < ntile) {
#pragma unroll
        for (int h = 0; h < 8; h++) acc ^= ring[k][h].x ^ ring[k][h].y ^ ring[k][h].z ^ ring[k][h].w;
      }
      load(ring[k], t + k + RING);
    }
  }
  out[(size_t)m * 256 + threadIdx.x] = acc;
}

int main(int argc, char** argv) {
  const int F = 12, Mp = 96, E = 2048, mem = 36, C = 128, P = 3, L = 4;
  const int H = 120, W = 160, scales[4] = {1, 2, 4, 8};
  std::mt19937 rng(0);
  std::uniform_real_distribution<float> U(0.f, 1.f);
  std::vector<int64_t> jj(E);
  for (int e = 0; e < E; e++) {
    const int k = (e < F * Mp) ? e : (int)(U(rng) * F * Mp) % (F * Mp);
    const int i = k / Mp;
    int j;
    do { j = i - 5 + (int)(U(rng) * 11); } while (j < 0 || j >= F);
    jj[e] = j;
  }
  std::vector<float> coords((size_t)E * 2 * P * P);
  for (int e = 0; e < E; e++) {
    const float cx = 4 + U(rng) * 151, cy = 4 + U(rng) * 111;
    for (int a = 0; a < P; a++)
      for (int c = 0; c < P; c++) {
        coords[((size_t)e * 2 + 0) * 9 + a * 3 + c] = cx + (c - 1) + 0.3f * U(rng);
        coords[((size_t)e * 2 + 1) * 9 + a * 3 + c] = cy + (a - 1) + 0.3f * U(rng);
      }
  }
  std::vector<int> order(E);
  for (int e = 0; e < E; e++) order[e] = e;
  std::stable_sort(order.begin(), order.end(), [&](int a, int b) { return jj[a] < jj[b]; });
  Lv lv;
  for (int l = 0; l < L; l++) {
    lv.H2[l] = H / scales[l];
    lv.W2[l] = W / scales[l];
    lv.sc[l] = (float)scales[l];
    const size_t n = (size_t)mem * lv.H2[l] * lv.W2[l] * C;
    float* d;
    hipMalloc(&d, n * 4);
    hipMemset(d, 1, n * 4);
    lv.f2[l] = d;
  }
  float* dco;
  int64_t* djj;
  int* dord;
  unsigned* dout;
  hipMalloc(&dco, coords.size() * 4);
  hipMemcpy(dco, coords.data(), coords.size() * 4, hipMemcpyHostToDevice);
  hipMalloc(&djj, E * 8);
  hipMemcpy(djj, jj.data(), E * 8, hipMemcpyHostToDevice);
  hipMalloc(&dord, E * 4);
  hipMemcpy(dord, order.data(), E * 4, hipMemcpyHostToDevice);
  hipMalloc(&dout, (size_t)E * 256 * 4);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  auto run = [&](auto kern, const char* name) {
    std::vector<float> ms;
    for (int r = 0; r < 60; r++) {
      hipEventRecord(a, 0);
      hipLaunchKernelGGL(kern, dim3(8 * ((E + 7) / 8)), dim3(256), 0, 0, lv, dco, djj, dord, E, mem, dout);
      hipEventRecord(b, 0);
      hipEventSynchronize(b);
      float t;
      hipEventElapsedTime(&t, a, b);
      if (r >= 10) ms.push_back(t);
    }
    std::sort(ms.begin(), ms.end());
    printf("%-40s median %.1f us\n", name, 1e3 * ms[ms.size() / 2]);
  };
  run(load_kernel<0, 2>, "16px x 64B, ring 2 (current)");
  run(load_kernel<1, 2>, "8px x 128B (whole lines), ring 2");
  run(load_kernel<2, 2>, "16px x 64B buffer, OOB refills, ring 2");
  run(load_kernel<0, 3>, "16px x 64B, ring 3");
  run(load_kernel<2, 3>, "16px x 64B buffer, OOB refills, ring 3");
  run(load_kernel<1, 3>, "8px x 128B, ring 3");
  run(load_kernel<2, 1>, "16px x 64B buffer, ring 1");
  return 0;
}
