// Per-wave phase stamps of corr_nhwc_lvl_kernel (diagnostic build of
// dpvo_amd/csrc/corr_nhwc.hip): cfg2-shaped synthetic graph (12 frames x 96
// patches, 2048 edges, targets within +-5 frames), 36-frame channels-last
// pyramid, levels [1,2,4,8], 160x120 level-1 maps, 128 channels.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I include -I dpvo_amd/csrc \
//         scripts/micro/lvl_stamps.hip -o scripts/micro/lvl_stamps
//   ./scripts/micro/lvl_stamps [variant=1]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

__device__ int64_t* g_lvl_st;  // [position * 4 + level][16]
typedef __attribute__((address_space(1))) int64_t gi64;
#define LVL_STAMP_INIT gi64* const lst_ = (gi64*)(uintptr_t)g_lvl_st
#define LVL_STAMP(k)                                                                      \
  do {                                                                                    \
    __builtin_amdgcn_sched_barrier(0);                                                    \
    if (lane == 0) {                                                                      \
      const size_t w_ = ((size_t)p * 4 + lev) * 16;                 \
      lst_[w_ + (k)] = __builtin_amdgcn_s_memtime();                                      \
      if ((k) == 0) {                                                                     \
        lst_[w_ + 8] = __builtin_amdgcn_s_memrealtime();                                  \
        lst_[w_ + 10] = ((int64_t)__builtin_amdgcn_s_getreg(63508) << 32) |              \
                        (uint32_t)__builtin_amdgcn_s_getreg(63492);                       \
      }                                                                                   \
      if ((k) == 6) lst_[w_ + 9] = __builtin_amdgcn_s_memrealtime();                      \
    }                                                                                     \
    __builtin_amdgcn_sched_barrier(0);                                                    \
  } while (0)

#include "corr_nhwc.hip"

int main(int argc, char** argv) {
  const int variant = argc > 1 ? atoi(argv[1]) : 1;
  const int F = 12, Mp = 96, E = 2048, mem = 36, C = 128, P = 3, L = 4, R = 3;
  const int H = 120, W = 160, scales[4] = {1, 2, 4, 8};
  std::mt19937 rng(0);
  std::uniform_real_distribution<float> U(0.f, 1.f);
  std::normal_distribution<float> Nn(0.f, 0.25f);
  std::vector<int64_t> jj(E), kk(E);
  for (int e = 0; e < E; e++) {
    const int k = (e < F * Mp) ? e : (int)(U(rng) * F * Mp) % (F * Mp);
    const int i = k / Mp;
    int j;
    do {
      j = i - 5 + (int)(U(rng) * 11);
    } while (j < 0 || j >= F);
    kk[e] = k;
    jj[e] = j;
  }
  std::vector<float> coords((size_t)E * 2 * P * P);
  for (int e = 0; e < E; e++) {
    const float cx = 4 + U(rng) * 151, cy = 4 + U(rng) * 111;
    for (int a = 0; a < P; a++)
      for (int c = 0; c < P; c++) {
        coords[((size_t)e * 2 + 0) * P * P + a * P + c] = cx + (c - 1) + 0.3f * U(rng);
        coords[((size_t)e * 2 + 1) * P * P + a * P + c] = cy + (a - 1) + 0.3f * U(rng);
      }
  }
  std::vector<int> order(E);
  for (int e = 0; e < E; e++) order[e] = e;
  std::stable_sort(order.begin(), order.end(), [&](int a, int b) { return jj[a] < jj[b]; });
  const void* f2[4];
  int H2[4], W2[4];
  float sc[4];
  for (int l = 0; l < L; l++) {
    H2[l] = H / scales[l];
    W2[l] = W / scales[l];
    sc[l] = (float)scales[l];
    const size_t n = (size_t)mem * H2[l] * W2[l] * C;
    std::vector<float> h(n);
    for (auto& v : h) v = Nn(rng);
    void* d;
    hipMalloc(&d, n * sizeof(float));
    hipMemcpy(d, h.data(), n * sizeof(float), hipMemcpyHostToDevice);
    f2[l] = d;
  }
  const size_t ng = (size_t)mem * Mp * C * P * P;
  std::vector<float> hg(ng);
  for (auto& v : hg) v = Nn(rng);
  float *gmap, *dco, *dout;
  int64_t *dii, *djj, *dst;
  int* dord;
  hipMalloc(&gmap, ng * 4);
  hipMemcpy(gmap, hg.data(), ng * 4, hipMemcpyHostToDevice);
  hipMalloc(&dco, coords.size() * 4);
  hipMemcpy(dco, coords.data(), coords.size() * 4, hipMemcpyHostToDevice);
  hipMalloc(&dii, E * 8);
  hipMalloc(&djj, E * 8);
  hipMemcpy(dii, kk.data(), E * 8, hipMemcpyHostToDevice);
  hipMemcpy(djj, jj.data(), E * 8, hipMemcpyHostToDevice);
  hipMalloc(&dord, E * 4);
  hipMemcpy(dord, order.data(), E * 4, hipMemcpyHostToDevice);
  hipMalloc(&dout, (size_t)E * 49 * 9 * L * 4);
  const size_t nst = (size_t)E * 4 * 16;
  hipMalloc(&dst, nst * 8);
  hipMemcpyToSymbol(HIP_SYMBOL(g_lvl_st), &dst, sizeof(dst));
  dpvo_corr_nhwc_variant(variant);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  std::vector<float> ms;
  for (int r = 0; r < 60; r++) {
    hipMemset(dst, 0, nst * 8);
    hipEventRecord(a, 0);
    int st = dpvo_corr_forward_levels_nhwc_ordered(gmap, f2, H2, W2, sc, L, dco, dii, djj, dord,
                                                   1, E, C, P, P, mem * Mp, mem, R, DPVO_F32, dout, 0);
    hipEventRecord(b, 0);
    hipEventSynchronize(b);
    if (st) {
      printf("status %d\n", st);
      return 1;
    }
    float t;
    hipEventElapsedTime(&t, a, b);
    if (r >= 10) ms.push_back(t);
  }
  std::sort(ms.begin(), ms.end());
  printf("variant %d: kernel median %.1f us (stamped build)\n", variant, 1e3 * ms[ms.size() / 2]);
  std::vector<int64_t> h(nst);
  hipMemcpy(h.data(), dst, nst * 8, hipMemcpyDeviceToHost);
  const int nw = (int)(nst / 16);
  int64_t r0 = INT64_MAX, r1 = 0;
  std::vector<int> live;
  for (int w = 0; w < nw; w++)
    if (h[(size_t)w * 16 + 8] && h[(size_t)w * 16 + 9]) {
      live.push_back(w);
      r0 = std::min(r0, h[(size_t)w * 16 + 8]);
      r1 = std::max(r1, h[(size_t)w * 16 + 9]);
    }
  printf("waves %zu, realtime span %.1f us\n", live.size(), (r1 - r0) / 100.0);
  const char* nm[] = {"start->geom+patch issued", "->ring issued", "->frag barrier", "->first tile done",
                      "->tiles done", "->bilinear+store"};
  for (int lv = -1; lv < 4; lv++) {
    printf("level %s:\n", lv < 0 ? "all" : std::to_string(lv).c_str());
    for (int k = 0; k < 6; k++) {
      std::vector<long long> v;
      for (int w : live) {
        if (lv >= 0 && (w & 3) != lv) continue;
        const int64_t x = h[(size_t)w * 16 + k], y = h[(size_t)w * 16 + k + 1];
        if (x && y) v.push_back(y - x);
      }
      std::sort(v.begin(), v.end());
      if (!v.empty())
        printf("  %-26s median %7lld p90 %7lld cyc\n", nm[k], v[v.size() / 2], v[v.size() * 9 / 10]);
    }
    std::vector<long long> life;
    for (int w : live) {
      if (lv >= 0 && (w & 3) != lv) continue;
      life.push_back(h[(size_t)w * 16 + 6] - h[(size_t)w * 16]);
    }
    std::sort(life.begin(), life.end());
    if (!life.empty())
      printf("  lifetime median %lld p90 %lld cyc\n", life[life.size() / 2], life[life.size() * 9 / 10]);
  }
  // occupancy: live waves per SIMD over time (10 bins of the span)
  {
    const int nb = 20;
    std::vector<double> occ(nb, 0.0);
    for (int w : live) {
      const int64_t s0 = h[(size_t)w * 16 + 8] - r0, s1 = h[(size_t)w * 16 + 9] - r0;
      for (int k = 0; k < nb; k++) {
        const double b0 = (double)(r1 - r0) * k / nb, b1 = (double)(r1 - r0) * (k + 1) / nb;
        const double ov = std::max(0.0, std::min((double)s1, b1) - std::max((double)s0, b0));
        occ[k] += ov / (b1 - b0);
      }
    }
    printf("live waves per SIMD by time:");
    for (int k = 0; k < nb; k++) printf(" %.2f", occ[k] / 1024.0);
    printf("\n");
    std::vector<long long> st;
    for (int w : live) st.push_back(h[(size_t)w * 16 + 8] - r0);
    std::sort(st.begin(), st.end());
    printf("wave start offsets (us): p10 %.1f median %.1f p90 %.1f max %.1f\n",
           st[st.size() / 10] / 100.0, st[st.size() / 2] / 100.0, st[st.size() * 9 / 10] / 100.0,
           st.back() / 100.0);
  }
  return 0;
}
