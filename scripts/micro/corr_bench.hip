// Standalone A-CORR timing with per-wave phase stamps (diagnostic build of
// dpvo_amd/csrc/corr_nhwc.hip): cfg2-shaped synthetic graph (12 frames x 96
// patches, 2048 edges, targets within +-5 frames), 36-frame channels-last
// pyramid, levels [1,2,4,8], 160x120 level-1 maps, 128 channels.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I include -I dpvo_amd/csrc \
//         scripts/micro/corr_bench.hip -o scripts/micro/corr_bench
//   ./scripts/micro/corr_bench [ordered=1] [first level] [levels] [edges] [parts=2]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

__device__ int64_t* g_stamps;  // [edges][16]
// stamps go through a global-address-space pointer read once per wave at
// kernel entry (CORR_TSTAMP_INIT): re-reading the __device__ variable per
// stamp, or storing through a generic pointer, waits for every outstanding
// tile load
typedef __attribute__((address_space(1))) int64_t gi64;
#define CORR_STAMP(slot)                                                     \
  do {                                                                       \
    if (lane == 0) stp_[(size_t)edge * 16 + (slot)] = __builtin_amdgcn_s_memtime(); \
  } while (0)

#define CORR_STAMP_RT(slot)                                                  \
  do {                                                                       \
    if (lane == 0) stp_[(size_t)edge * 16 + (slot)] = __builtin_amdgcn_s_memrealtime(); \
  } while (0)

#define CORR_STAMP_ID(slot)                                                  \
  do {                                                                       \
    if (lane == 0)                                                           \
      stp_[(size_t)edge * 16 + (slot)] =                                     \
          ((int64_t)__builtin_amdgcn_s_getreg(63508) << 32) |                 \
          (uint32_t)__builtin_amdgcn_s_getreg(63492);                         \
  } while (0)

// per-tile stamps of the first kTS edges: [edge][tile][3] (step start, loads
// issued, G stored); s_memtime between sched barriers
constexpr int kTS = 64, kTT = 32;
__device__ int64_t* g_tst;
// the buffer pointer is read once per wave (a per-stamp reload of the
// __device__ variable would wait for every outstanding load)
#define CORR_TSTAMP_INIT                                      \
  gi64* const tst_ = (gi64*)(uintptr_t)g_tst;                 \
  gi64* const stp_ = (gi64*)(uintptr_t)g_stamps
#define CORR_TSTAMP(i, k)                                                            \
  do {                                                                               \
    __builtin_amdgcn_sched_barrier(0);                                               \
    if (lane == 0 && edge < kTS && (i) < kTT)                                        \
      tst_[((size_t)edge * kTT + (i)) * 3 + (k)] = __builtin_amdgcn_s_memtime();     \
    __builtin_amdgcn_sched_barrier(0);                                               \
  } while (0)

#include "corr_nhwc.hip"

int main(int argc, char** argv) {
  const int ordered = argc > 1 ? atoi(argv[1]) : 1;
  const int F = 12, Mp = 96, E = argc > 4 ? atoi(argv[4]) : 2048, mem = 36, C = 128, P = 3, L = 4, R = 3;
  const int H = 120, W = 160, scales[4] = {1, 2, 4, 8};
  std::mt19937 rng(0);
  std::uniform_real_distribution<float> U(0.f, 1.f);
  std::normal_distribution<float> Nn(0.f, 0.25f);
  // edges: every patch once, then random extra (k, j) with |j - i| <= 5
  std::vector<int64_t> ii(E), jj(E), kk(E);
  for (int e = 0; e < E; e++) {
    const int k = (e < F * Mp) ? e : (int)(U(rng) * F * Mp) % (F * Mp);
    const int i = k / Mp;
    int j;
    do {
      j = i - 5 + (int)(U(rng) * 11);
    } while (j < 0 || j >= F);
    kk[e] = k;
    ii[e] = i;
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
  {
    std::vector<int> idx(E);
    for (int e = 0; e < E; e++) idx[e] = e;
    std::stable_sort(idx.begin(), idx.end(), [&](int a, int b) { return jj[a] < jj[b]; });
    order = idx;
  }
  float* lvl[4];
  int H2[4], W2[4];
  float sc[4];
  for (int l = 0; l < L; l++) {
    H2[l] = H / scales[l];
    W2[l] = W / scales[l];
    sc[l] = (float)scales[l];
    const size_t n = (size_t)mem * H2[l] * W2[l] * C;
    std::vector<float> h(n);
    for (auto& v : h) v = Nn(rng);
    hipMalloc(&lvl[l], n * sizeof(float));
    hipMemcpy(lvl[l], h.data(), n * sizeof(float), hipMemcpyHostToDevice);
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
  hipMemcpy(dii, kk.data(), E * 8, hipMemcpyHostToDevice);  // fmap1 index = patch
  hipMemcpy(djj, jj.data(), E * 8, hipMemcpyHostToDevice);
  hipMalloc(&dord, E * 4);
  hipMemcpy(dord, order.data(), E * 4, hipMemcpyHostToDevice);
  hipMalloc(&dout, (size_t)E * 49 * 9 * L * 4);
  const int parts = 1;
  hipMalloc(&dst, (size_t)E * 2 * 16 * 8);
  hipMemcpyToSymbol(HIP_SYMBOL(g_stamps), &dst, sizeof(dst));
  int64_t* dts;
  hipMalloc(&dts, (size_t)kTS * kTT * 3 * 8);
  hipMemset(dts, 0, (size_t)kTS * kTT * 3 * 8);
  hipMemcpyToSymbol(HIP_SYMBOL(g_tst), &dts, sizeof(dts));
  // optional level subset: corr_bench <ordered> <first level> <count>
  const int l0 = argc > 2 ? atoi(argv[2]) : 0, Lr = argc > 3 ? atoi(argv[3]) : L;
  const void* f2[4] = {lvl[l0 % 4], lvl[(l0 + 1) % 4], lvl[(l0 + 2) % 4], lvl[(l0 + 3) % 4]};
  int H2r[4], W2r[4];
  float scr[4];
  for (int l = 0; l < 4; l++) {
    H2r[l] = H2[(l0 + l) % 4];
    W2r[l] = W2[(l0 + l) % 4];
    scr[l] = sc[(l0 + l) % 4];
  }
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  std::vector<float> ms;
  for (int r = 0; r < 60; r++) {
    hipMemset(dst, 0, (size_t)E * 2 * 16 * 8);
    hipEventRecord(a, 0);
    int st = dpvo_corr_forward_levels_nhwc_ordered(gmap, f2, H2r, W2r, scr, Lr, dco, dii, djj,
                                                   ordered ? dord : nullptr, 1, E, C, P, P,
                                                   mem * Mp, mem, R, DPVO_F32, dout, 0);
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
  printf("ordered=%d parts=%d kernel median %.1f us\n", ordered, parts, 1e3 * ms[ms.size() / 2]);
  std::vector<int64_t> h((size_t)E * 2 * 16);
  hipMemcpy(h.data(), dst, h.size() * 8, hipMemcpyDeviceToHost);
  if (parts == 2) {  // per (edge, part) stamps: analyse the waves as units
    std::vector<int64_t> h2((size_t)E * 16, 0);
    for (int e = 0; e < E; e++) for (int k = 0; k < 16; k++) h2[(size_t)e * 16 + k] = h[(size_t)(2 * e) * 16 + k];
    h.swap(h2);
  }
  int64_t t0 = INT64_MAX, t1 = 0;
  for (int e = 0; e < E; e++) {
    t0 = std::min(t0, h[(size_t)e * 16]);
    t1 = std::max(t1, h[(size_t)e * 16 + 11]);
  }
  printf("first start -> last end: %lld cyc\n", (long long)(t1 - t0));
  const char* nm[] = {"start->geom", "geom->L0 tiles", "L0 bilin", "->L1 tiles", "L1 bilin",
                      "->L2 tiles", "L2 bilin", "->L3 tiles", "L3 bilin", "->store", "store"};
  const int pa[] = {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10}, pb[] = {1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11};
  for (int k = 0; k < 11; k++) {
    std::vector<long long> v;
    for (int e = 0; e < E; e++) {
      const int64_t x = h[(size_t)e * 16 + pa[k]], y = h[(size_t)e * 16 + pb[k]];
      if (x && y) v.push_back(y - x);
    }
    std::sort(v.begin(), v.end());
    if (!v.empty())
      printf("%-16s median %7lld  p90 %7lld cyc\n", nm[k], v[v.size() / 2], v[v.size() * 9 / 10]);
  }
  {
    int64_t r0 = INT64_MAX, r1 = 0;
    std::vector<long long> rl;
    std::vector<double> clk;
    for (int e = 0; e < E; e++) {
      const int64_t a0 = h[(size_t)e * 16 + 12], a1 = h[(size_t)e * 16 + 13];
      r0 = std::min(r0, a0);
      r1 = std::max(r1, a1);
      rl.push_back(a1 - a0);
      clk.push_back((double)(h[(size_t)e * 16 + 11] - h[(size_t)e * 16]) / (double)(a1 - a0) / 10.0);
    }
    std::sort(rl.begin(), rl.end());
    std::sort(clk.begin(), clk.end());
    printf("realtime: kernel span %.1f us, wave lifetime median %.1f p90 %.1f max %.1f us, "
           "clock %.2f GHz\n",
           (r1 - r0) / 100.0, rl[E / 2] / 100.0, rl[E * 9 / 10] / 100.0, rl[E - 1] / 100.0,
           clk[E / 2]);
    std::vector<long long> so;
    for (int e = 0; e < E; e++) so.push_back(h[(size_t)e * 16 + 12] - r0);
    std::sort(so.begin(), so.end());
    printf("realtime start offsets: median %.1f p90 %.1f max %.1f us\n", so[E / 2] / 100.0,
           so[E * 9 / 10] / 100.0, so[E - 1] / 100.0);
  }
  {  // residency: waves per (XCC, SE, SH, CU) that started in the first 10 us
    int64_t r0 = INT64_MAX;
    for (int e = 0; e < E; e++) r0 = std::min(r0, h[(size_t)e * 16 + 12]);
    std::vector<int> cnt(8 * 8 * 2 * 16, 0), cntall(8 * 8 * 2 * 16, 0);
    for (int e = 0; e < E; e++) {
      const uint64_t id = (uint64_t)h[(size_t)e * 16 + 14];
      const uint32_t hw = (uint32_t)id, xcc = (uint32_t)(id >> 32) & 0xf;
      const int cu = (hw >> 8) & 0xf, sh = (hw >> 12) & 1, se = (hw >> 13) & 7;
      const int key = ((xcc * 8 + se) * 2 + sh) * 16 + cu;
      cntall[key]++;
      if (h[(size_t)e * 16 + 12] - r0 < 1000) cnt[key]++;
    }
    int used = 0, used1 = 0, mx = 0, mx1 = 0;
    for (size_t k = 0; k < cnt.size(); k++) {
      if (cntall[k]) used++;
      if (cnt[k]) used1++;
      mx = std::max(mx, cntall[k]);
      mx1 = std::max(mx1, cnt[k]);
    }
    printf("CUs used %d (first 10 us: %d), max waves per CU %d (first 10 us: %d)\n", used, used1,
           mx, mx1);
  }
  std::vector<long long> st0, life;
  for (int e = 0; e < E; e++) {
    st0.push_back(h[(size_t)e * 16] - t0);
    life.push_back(h[(size_t)e * 16 + 11] - h[(size_t)e * 16]);
  }
  std::sort(st0.begin(), st0.end());
  std::sort(life.begin(), life.end());
  printf("wave start offset median %lld p90 %lld max %lld; lifetime median %lld p90 %lld\n",
         st0[E / 2], st0[E * 9 / 10], st0[E - 1], life[E / 2], life[E * 9 / 10]);
  {  // per-tile: a = start -> loads issued (wait + split + MFMA issue), b = -> G stored,
     // c = G stored -> next step start (bilinear at level ends, loop)
    std::vector<int64_t> t((size_t)kTS * kTT * 3);
    hipMemcpy(t.data(), dts, t.size() * 8, hipMemcpyDeviceToHost);
    std::vector<long long> A, Bv, Cv;
    for (int e = 0; e < kTS; e++) {
      printf("edge %d:", e < 4 ? e : -1);
      for (int i = 0; i + 1 < kTT; i++) {
        const int64_t* p = &t[((size_t)e * kTT + i) * 3];
        const int64_t* q = p + 3;
        if (!p[0] || !p[1] || !p[2]) break;
        A.push_back(p[1] - p[0]);
        Bv.push_back(p[2] - p[1]);
        if (q[0]) Cv.push_back(q[0] - p[2]);
        if (e < 4) printf(" [%lld %lld %lld]", (long long)(p[1] - p[0]), (long long)(p[2] - p[1]),
                          q[0] ? (long long)(q[0] - p[2]) : -1LL);
      }
      if (e < 4) printf("\n");
      else { printf("\r"); }
    }
    auto med = [](std::vector<long long> v) { std::sort(v.begin(), v.end()); return v.empty() ? 0LL : v[v.size() / 2]; };
    auto p90 = [](std::vector<long long> v) { std::sort(v.begin(), v.end()); return v.empty() ? 0LL : v[v.size() * 9 / 10]; };
    printf("\ntile: start->issued median %lld p90 %lld | ->G stored median %lld p90 %lld | ->next median %lld p90 %lld cyc\n",
           med(A), p90(A), med(Bv), p90(Bv), med(Cv), p90(Cv));
  }
  return 0;
}
