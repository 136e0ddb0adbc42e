// keyframe.hip -- the frame bookkeeping around DPVO's update on the device
// (SURVEY 8(f3)): DPVO.keyframe's frame drop (dpvo/dpvo.py:601-676, with
// motionmag 586-599) and PatchGraph.edges_loop (dpvo/patchgraph.py:65-91), both
// over projective_ops.flow_mag (projective_ops.py:120-130).
//
// The reference decides on the host (.item() on the motion magnitude, numpy
// NMS in loop_closure/optim_utils.py:24-60) and moves frames with per-frame
// tensor copies.  Here every step is a kernel and no result comes back to the
// host: the frame-drop decision is a device flag {drop, k} that predicates the
// edge removal (pg.hip, dpvo_pg_remove_frame_dev), the edge index shift, the
// frame-data shift and the frame counters; edges_loop writes its edges and
// their count into device buffers that dpvo_pg_append_dev appends.
//
// Arithmetic: the lietorch chain of projective_ops.transform (Pj * Pi^-1 with
// the quaternion renormalised at every group load, so3.h:95-97; act4; proj
// with 1 / clamp(Z, 0.1)) in fp32 without FMA contraction, op by op; sums in
// fp64 in a fixed order (the reference's torch reductions are unordered).
#include <algorithm>

#include "common.hpp"

namespace dpvo {
namespace {

#pragma clang fp contract(off)

struct G7 {
  float t[3];
  float q[4];  // x y z w
};

// a lietorch group read from memory: quaternion normalised (so3.h:95-97)
__device__ __forceinline__ G7 g_load(const float* d) {
  G7 g;
  g.t[0] = d[0];
  g.t[1] = d[1];
  g.t[2] = d[2];
  const float n = sqrtf(d[3] * d[3] + d[4] * d[4] + d[5] * d[5] + d[6] * d[6]);
  g.q[0] = d[3] / n;
  g.q[1] = d[4] / n;
  g.q[2] = d[5] / n;
  g.q[3] = d[6] / n;
  return g;
}

// so3.h act: p + w uv + v x uv, uv = 2 v x p
__device__ __forceinline__ void q_act(const float* q, const float* p, float* o) {
  float uv[3];
  uv[0] = q[1] * p[2] - q[2] * p[1];
  uv[1] = q[2] * p[0] - q[0] * p[2];
  uv[2] = q[0] * p[1] - q[1] * p[0];
  uv[0] += uv[0];
  uv[1] += uv[1];
  uv[2] += uv[2];
  float c[3];
  c[0] = q[1] * uv[2] - q[2] * uv[1];
  c[1] = q[2] * uv[0] - q[0] * uv[2];
  c[2] = q[0] * uv[1] - q[1] * uv[0];
  for (int i = 0; i < 3; i++) o[i] = p[i] + q[3] * uv[i] + c[i];
}

// stored group after an op (lietorch writes 7 floats; the next op reloads,
// i.e. renormalises): g_load of the op's output
__device__ __forceinline__ G7 g_store_load(const G7& g) {
  float d[7] = {g.t[0], g.t[1], g.t[2], g.q[0], g.q[1], g.q[2], g.q[3]};
  return g_load(d);
}

__device__ __forceinline__ G7 g_inv(const G7& g) {  // se3.h inv
  G7 o;
  const float n = sqrtf(g.q[0] * g.q[0] + g.q[1] * g.q[1] + g.q[2] * g.q[2] + g.q[3] * g.q[3]);
  o.q[0] = -g.q[0] / n;
  o.q[1] = -g.q[1] / n;
  o.q[2] = -g.q[2] / n;
  o.q[3] = g.q[3] / n;
  float t[3];
  q_act(o.q, g.t, t);
  o.t[0] = -t[0];
  o.t[1] = -t[1];
  o.t[2] = -t[2];
  return o;
}

__device__ __forceinline__ G7 g_mul(const G7& a, const G7& b) {  // se3.h mul
  G7 o;
  const float x = a.q[3] * b.q[0] + a.q[0] * b.q[3] + a.q[1] * b.q[2] - a.q[2] * b.q[1];
  const float y = a.q[3] * b.q[1] + a.q[1] * b.q[3] + a.q[2] * b.q[0] - a.q[0] * b.q[2];
  const float z = a.q[3] * b.q[2] + a.q[2] * b.q[3] + a.q[0] * b.q[1] - a.q[1] * b.q[0];
  const float w = a.q[3] * b.q[3] - a.q[0] * b.q[0] - a.q[1] * b.q[1] - a.q[2] * b.q[2];
  const float n = sqrtf(x * x + y * y + z * z + w * w);
  o.q[0] = x / n;
  o.q[1] = y / n;
  o.q[2] = z / n;
  o.q[3] = w / n;
  float t[3];
  q_act(a.q, b.t, t);
  for (int i = 0; i < 3; i++) o.t[i] = a.t[i] + t[i];
  return o;
}

// projective_ops.transform of one patch pixel (x, y, inverse depth d):
// Gij = poses[jj] * poses[ii].inv() (tonly: rotation set to identity),
// X1 = Gij * iproj(p, K_i), out = proj(X1, K_j); *Z = X1's Z
__device__ __forceinline__ void transform_px(const float* Pi, const float* Pj, const float* Ki,
                                             const float* Kj, float x, float y, float d,
                                             bool tonly, float* out, float* Z) {
  const G7 gi = g_load(Pi), gj = g_load(Pj);
  const G7 ginv = g_store_load(g_inv(gi));
  G7 gij = g_store_load(g_mul(gj, ginv));
  if (tonly) {
    gij.q[0] = gij.q[1] = gij.q[2] = 0.0f;
    gij.q[3] = 1.0f;
  }
  const float X0[4] = {(x - Ki[2]) / Ki[0], (y - Ki[3]) / Ki[1], 1.0f, d};
  float p[3];
  q_act(gij.q, X0, p);
  const float X = p[0] + gij.t[0] * X0[3], Y = p[1] + gij.t[1] * X0[3],
              Zz = p[2] + gij.t[2] * X0[3];
  const float inv = 1.0f / fmaxf(Zz, 0.1f);
  out[0] = Kj[0] * (inv * X) + Kj[2];
  out[1] = Kj[1] * (inv * Y) + Kj[3];
  *Z = Zz;
}

// projective_ops.flow_mag of one pixel: beta |c1 - c0| + (1 - beta) |c2 - c0|,
// valid = Z1 > 0.2 (c0: Pi * Pi^-1, c1: Pj * Pi^-1, c2: its translation only)
__device__ __forceinline__ float flow_px(const float* Pi, const float* Pj, const float* Ki,
                                         const float* Kj, float x, float y, float d, float beta,
                                         bool* valid) {
  float c0[2], c1[2], c2[2], z0, z1, z2;
  transform_px(Pi, Pi, Ki, Ki, x, y, d, false, c0, &z0);
  transform_px(Pi, Pj, Ki, Kj, x, y, d, false, c1, &z1);
  transform_px(Pi, Pj, Ki, Kj, x, y, d, true, c2, &z2);
  const float a0 = c1[0] - c0[0], a1 = c1[1] - c0[1];
  const float b0 = c2[0] - c0[0], b1 = c2[1] - c0[1];
  const float f1 = sqrtf(a0 * a0 + a1 * a1), f2 = sqrtf(b0 * b0 + b1 * b1);
  *valid = z1 > 0.2f;
  return beta * f1 + (1.0f - beta) * f2;
}


#pragma clang fp contract(fast)

constexpr int kKfT = 256;
// PatchGraph error flags (counts[2], dpvo_amd/patchgraph.py DevicePatchGraph.errors)
constexpr int kPgErrLoopCap = 4;    // edges_loop: device frame count above n_cap, no loop edges
constexpr int kPgErrDeltaFull = 8;  // kf_shift: pg.delta log full, a record was not kept

// ---- DPVO.keyframe: motion magnitude and decision (dpvo.py:586-599, 619-624) ----
// st = {n, m} (device frame counters).  motionmag(a, b) = mean over the P x P
// pixels of the active edges a -> b of flow_mag(beta 0.5), 0 without such an
// edge.  torch's mean is sum * (1 / N) in fp32; .item() then leaves fp32 and
// the sum of both directions and the halving run in double (Python floats).
// out: kf = {drop, k = n - KI}, mag = {motionmag(i, j), motionmag(j, i)}
__global__ void __launch_bounds__(kKfT) kf_motion_kernel(
    const int64_t* __restrict__ ii, const int64_t* __restrict__ jj, const int64_t* __restrict__ kk,
    const int* __restrict__ counts, const float* __restrict__ poses,
    const float* __restrict__ patches, const float* __restrict__ intr, int P,
    const int* __restrict__ st, int KI, double thresh, int* __restrict__ kf,
    float* __restrict__ mag) {
  __shared__ double ssum[2][kKfT / 64];
  __shared__ int scnt[2][kKfT / 64];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int n = st[0], num = counts[0], PP = P * P;
  const int i = n - KI - 1, j = n - KI + 1;
  double s0 = 0.0, s1 = 0.0;
  int c0 = 0, c1 = 0;
  for (int e = tid; e < num; e += kKfT) {
    const int64_t a = ii[e], b = jj[e];
    const bool f = (a == i && b == j), r = (a == j && b == i);
    if (!f && !r) continue;
    const float* pk = patches + kk[e] * 3 * PP;
    double s = 0.0;
    for (int px = 0; px < PP; px++) {
      bool v;
      s += (double)flow_px(poses + 7 * a, poses + 7 * b, intr + 4 * a, intr + 4 * b, pk[px],
                           pk[PP + px], pk[2 * PP + px], 0.5f, &v);
    }
    if (f) {
      s0 += s;
      c0 += PP;
    } else {
      s1 += s;
      c1 += PP;
    }
  }
  s0 = wave_sum(s0);
  s1 = wave_sum(s1);
  c0 = wave_sum(c0);
  c1 = wave_sum(c1);
  if (lane == 0) {
    ssum[0][wid] = s0;
    ssum[1][wid] = s1;
    scnt[0][wid] = c0;
    scnt[1][wid] = c1;
  }
  __syncthreads();
  if (tid == 0) {
    double t0 = 0.0, t1 = 0.0;
    int n0 = 0, n1 = 0;
    for (int w = 0; w < kKfT / 64; w++) {
      t0 += ssum[0][w];
      t1 += ssum[1][w];
      n0 += scnt[0][w];
      n1 += scnt[1][w];
    }
    const float m0 = n0 ? __fmul_rn((float)t0, 1.0f / (float)n0) : 0.0f;
    const float m1 = n1 ? __fmul_rn((float)t1, 1.0f / (float)n1) : 0.0f;
    const double m = (double)m0 + (double)m1;
    kf[0] = (i >= 0 && m / 2.0 < thresh) ? 1 : 0;
    kf[1] = n - KI;
    mag[0] = m0;
    mag[1] = m1;
  }
}

// ---- dpvo.py:626-631: pg.delta[t1] = (t0, poses_[k] * poses_[k-1].inv()) ----
// a device log of (t1, t0, dP) records; runs before the frame shift
__global__ void kf_delta_kernel(const int* __restrict__ kf, const float* __restrict__ poses,
                                const int64_t* __restrict__ tstamps, float* __restrict__ dlog,
                                int64_t* __restrict__ tlog, int* __restrict__ dcnt, int cap,
                                int* __restrict__ errors) {
  if (threadIdx.x != 0 || blockIdx.x != 0 || !kf[0]) return;
  const int k = kf[1];
  const int slot = *dcnt;
  if (slot >= cap) {  // the record would be lost (the reference dict never drops one): flag it
    atomicOr(errors, kPgErrDeltaFull);
    return;
  }
  const G7 dp = g_mul(g_load(poses + 7 * k), g_store_load(g_inv(g_load(poses + 7 * (k - 1)))));
  for (int c = 0; c < 3; c++) dlog[7 * slot + c] = dp.t[c];
  for (int c = 0; c < 4; c++) dlog[7 * slot + 3 + c] = dp.q[c];
  tlog[2 * slot] = tstamps[k];
  tlog[2 * slot + 1] = tstamps[k - 1];
  *dcnt = slot + 1;
}

// ---- dpvo.py:644-656: active edges past frame k move back one frame ----
__global__ void kf_shift_edges_kernel(int64_t* __restrict__ ii, int64_t* __restrict__ jj,
                                      int64_t* __restrict__ kk, const int* __restrict__ counts,
                                      const int* __restrict__ kf, int M) {
  if (!kf[0]) return;
  const int k = kf[1], num = counts[0];
  for (int e = blockIdx.x * blockDim.x + threadIdx.x; e < num; e += gridDim.x * blockDim.x) {
    const int64_t a = ii[e], b = jj[e];
    if (a > k) {
      kk[e] -= M;
      ii[e] = a - 1;
    }
    if (b > k) jj[e] = b - 1;
  }
}

// ---- dpvo.py:658-673: frame data k+1 .. n-1 -> k .. n-2, then n -= 1, m -= M ----
constexpr int kMaxShift = 12;
constexpr int kMaxMoved = 16;
struct ShiftArrays {
  char* base[kMaxShift];
  long long bytes[kMaxShift];  // per frame
  int ring[kMaxShift];         // 0: row = frame; else row = frame % ring
  int count;
};

// each thread owns one 4-byte word (or byte) offset of every moved frame of an
// array: it reads them all, then writes, so in-place ring moves are race-free
template <typename W>
__device__ __forceinline__ void shift_array(W* base, long long words, int ring, int k, int nm) {
  for (long long w = (long long)blockIdx.x * blockDim.x + threadIdx.x; w < words;
       w += (long long)gridDim.x * blockDim.x) {
    W v[kMaxMoved];
#pragma unroll
    for (int f = 0; f < kMaxMoved; f++)
      if (f < nm) v[f] = base[(long long)(ring ? (k + 1 + f) % ring : k + 1 + f) * words + w];
#pragma unroll
    for (int f = 0; f < kMaxMoved; f++)
      if (f < nm) base[(long long)(ring ? (k + f) % ring : k + f) * words + w] = v[f];
  }
}

__global__ void kf_shift_frames_kernel(ShiftArrays sa, const int* __restrict__ kf,
                                       const int* __restrict__ st) {
  if (!kf[0]) return;
  const int k = kf[1], nm = st[0] - 1 - k;  // KEYFRAME_INDEX - 1 frames
  if (nm <= 0 || nm > kMaxMoved) return;
  for (int a = 0; a < sa.count; a++) {
    if (sa.bytes[a] % 4 == 0)
      shift_array(reinterpret_cast<int*>(sa.base[a]), sa.bytes[a] / 4, sa.ring[a], k, nm);
    else
      shift_array(reinterpret_cast<unsigned char*>(sa.base[a]), sa.bytes[a], sa.ring[a], k, nm);
  }
}

__global__ void kf_decrement_kernel(int* __restrict__ st, const int* __restrict__ kf, int M) {
  if (threadIdx.x == 0 && blockIdx.x == 0 && kf[0]) {
    st[0] -= 1;
    st[1] -= M;
  }
}

// ---- PatchGraph.edges_loop (patchgraph.py:65-91) + its caller's gate (dpvo.py:984-988) ----
// candidates: meshgrid(jj in [n - GOF, n - KI), kk in [lo M, l M)) 'ij', with
// l = n - REMOVAL_WINDOW, lo = max(l - MAX_EDGE_AGE, 0); each M consecutive
// candidates are one group g = (target frame j0 + g / nf, source patches of
// frame-group lo + g % nf).  flow_mag(beta 0.5) at patch pixel (1, 1)
// (patches[..., 1, 1]).  Group value: sum(flow * valid) / max(count, 1) in
// fp32 if count > 0.75 M else inf.
struct LoopCfg {
  int P, M, rw, age, gof, ki, nj, n_cap;
  float thresh;
  int max_edges, nms;
};

__device__ __forceinline__ bool loop_window(const LoopCfg& c, int n, const int* last_ba, int& j0,
                                            int& lo, int& nf) {
  // the launch (group grid, sort size, suppression bitmap) was sized for
  // n <= n_cap: a larger device frame count takes no loop edges (the caller
  // sees error bit 4, see dpvo_edges_loop)
  if (n > c.n_cap) return false;
  if (last_ba && n - last_ba[0] < c.gof) return false;  // dpvo.py:984
  const int l = n - c.rw;
  if (l <= 0) return false;  // patchgraph.py:70-71
  j0 = n - c.gof;
  lo = max(l - c.age, 0);
  nf = l - lo;
  return c.nj > 0;
}

__global__ void el_groups_kernel(const float* __restrict__ poses, const float* __restrict__ patches,
                                 const float* __restrict__ intr, const int64_t* __restrict__ ix,
                                 const int* __restrict__ st, const int* __restrict__ last_ba,
                                 LoopCfg c, float* __restrict__ gflow, int* __restrict__ gi) {
  int j0, lo, nf;
  if (!loop_window(c, st[0], last_ba, j0, lo, nf)) return;
  const int g = blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (g >= c.nj * nf) return;
  const int j = j0 + g / nf, f = lo + g % nf;
  const int PP = c.P * c.P, px = c.P + 1;
  double s = 0.0;
  int cnt = 0;
  for (int m = lane; m < c.M; m += 64) {
    const int64_t k = (int64_t)f * c.M + m;
    const int i = (int)ix[k];
    const float* pk = patches + k * 3 * PP;
    bool v;
    const float fl = flow_px(poses + 7 * i, poses + 7 * j, intr + 4 * i, intr + 4 * j, pk[px],
                             pk[PP + px], pk[2 * PP + px], 0.5f, &v);
    if (v) {
      s += (double)fl;
      cnt += 1;
    }
  }
  s = wave_sum(s);
  cnt = wave_sum(cnt);
  if (lane == 0) {
    const float fs = (float)s, fc = (float)(cnt > 1 ? cnt : 1);
    gflow[g] = ((float)cnt > 0.75f * (float)c.M) ? __fdiv_rn(fs, fc) : __builtin_inff();
    gi[g] = (int)ix[(int64_t)f * c.M];  // ii[::M]
  }
}

// reduce_edges (loop_closure/optim_utils.py:24-60) over the groups with value
// < BACKEND_THRESH: ascending by value (ties by group index: the order of a
// stable argsort), skip j - i < 30, value >= 1000 and (i, j) suppressed by an
// accepted (i +- nms, j); stop at max_edges.  One workgroup: bitonic sort of
// (value bits << 32 | group) in LDS, one thread walks it with a bitmap of
// suppressed (i, j).  Output kk = i M + arange(M), jj = j, count (edges x M),
// and last_ba = n when edges were found (dpvo.py:987).
constexpr int kElT = 1024;
constexpr int kElSort = 16384;
constexpr int kElBits = 131072;  // suppression bitmap: n x nj bits
constexpr int kElMaxOut = 1024;
__global__ void __launch_bounds__(kElT) el_select_kernel(
    const float* __restrict__ gflow, const int* __restrict__ gi, const int* __restrict__ st,
    int* __restrict__ last_ba, LoopCfg c, int64_t* __restrict__ out_kk,
    int64_t* __restrict__ out_jj, int* __restrict__ out_n, int* __restrict__ errors) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  unsigned long long* keys = reinterpret_cast<unsigned long long*>(lds);
  unsigned* bits = reinterpret_cast<unsigned*>(keys + kElSort);
  __shared__ int s_imax, s_cnt;
  __shared__ int s_ei[kElMaxOut], s_ej[kElMaxOut];
  const int tid = threadIdx.x;
  const int n = st[0];
  int j0, lo, nf;
  if (!loop_window(c, n, last_ba, j0, lo, nf)) {
    if (tid == 0) {
      *out_n = 0;
      if (n > c.n_cap && errors) atomicOr(errors, kPgErrLoopCap);
    }
    return;
  }
  const int ng = c.nj * nf;
  if (tid == 0) {
    s_imax = -1;
    s_cnt = 0;
  }
  __syncthreads();
  int P2 = 1;
  while (P2 < ng) P2 <<= 1;
  int imax = -1;
  for (int g = tid; g < P2; g += kElT) {
    unsigned long long key = ~0ull;
    if (g < ng) {
      const float f = gflow[g];
      if (f < c.thresh) {  // patchgraph.py:84 (flow values are >= 0)
        key = ((unsigned long long)__float_as_uint(f) << 32) | (unsigned)g;
        imax = max(imax, gi[g]);
      }
    }
    keys[g] = key;
  }
  atomicMax(&s_imax, imax);
  __syncthreads();
  for (int size = 2; size <= P2; size <<= 1)
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      for (int x = tid; x < P2 / 2; x += kElT) {
        const int a = 2 * x - (x & (stride - 1)), b = a + stride;
        const bool up = (a & size) == 0;
        const unsigned long long ka = keys[a], kb = keys[b];
        if ((ka > kb) == up) {
          keys[a] = kb;
          keys[b] = ka;
        }
      }
      __syncthreads();
    }
  const int Ni = s_imax + 1;  // ignore_lookup rows: ii.max() + 1
  const int words = (Ni * c.nj + 31) / 32;
  for (int w = tid; w < words; w += kElT) bits[w] = 0u;
  __syncthreads();
  if (tid == 0) {
    int cnt = 0;
    for (int p = 0; p < P2; p++) {
      const unsigned long long key = keys[p];
      if (key == ~0ull) break;
      if (cnt + 1 > c.max_edges) break;  // len(es) > max_num_edges (es holds a dummy)
      const int g = (int)(key & 0xffffffffull);
      const int i = gi[g], j = j0 + g / nf;
      if (j - i < 30) continue;
      if (__uint_as_float((unsigned)(key >> 32)) >= 1000.0f) continue;
      const int b = i * c.nj + (j - j0);
      if ((bits[b >> 5] >> (b & 31)) & 1u) continue;
      s_ei[cnt] = i;
      s_ej[cnt] = j;
      cnt++;
      for (int di = -c.nms; di <= c.nms; di++) {
        const int i1 = i + di;
        if (i1 >= 0 && i1 < Ni) {
          const int b1 = i1 * c.nj + (j - j0);
          bits[b1 >> 5] |= 1u << (b1 & 31);
        }
      }
    }
    s_cnt = cnt;
    *out_n = cnt * c.M;
    if (cnt > 0 && last_ba) last_ba[0] = n;
  }
  __syncthreads();
  const int cnt = s_cnt;
  for (int t = tid; t < cnt * c.M; t += kElT) {
    const int e = t / c.M, m = t % c.M;
    out_kk[t] = (int64_t)s_ei[e] * c.M + m;
    out_jj[t] = s_ej[e];
  }
}

}  // namespace
}  // namespace dpvo

using namespace dpvo;

DPVO_EXPORT int dpvo_kf_motion(const int64_t* ii, const int64_t* jj, const int64_t* kk,
                               const int32_t* counts, const float* poses, const float* patches,
                               const float* intrinsics, int P, const int32_t* st,
                               int keyframe_index, double keyframe_thresh, int32_t* kf,
                               float* mag, void* stream) {
  if (!ii || !jj || !kk || !counts || !poses || !patches || !intrinsics || !st || !kf || !mag ||
      P <= 0 || keyframe_index < 1)
    return DPVO_ERR_INVALID;
  hipLaunchKernelGGL(kf_motion_kernel, dim3(1), dim3(kKfT), 0, as_stream(stream), ii, jj, kk,
                     (const int*)counts, poses, patches, intrinsics, P, (const int*)st,
                     keyframe_index, keyframe_thresh, (int*)kf, mag);
  return launch_status();
}

DPVO_EXPORT int dpvo_kf_shift(const int32_t* kf, int M, int32_t* st, int64_t* ii, int64_t* jj,
                              int64_t* kk, int32_t* counts, int max_edges,
                              void* const* frame_arrays, const int64_t* bytes_per_frame,
                              const int32_t* ring, int narrays, const float* poses,
                              const int64_t* tstamps, float* delta_log, int64_t* delta_tstamps,
                              int32_t* delta_count, int delta_cap, void* stream) {
  if (!kf || !st || !ii || !jj || !kk || !counts || M <= 0 || max_edges <= 0 || narrays < 0 ||
      narrays > kMaxShift || (narrays && (!frame_arrays || !bytes_per_frame || !ring)))
    return DPVO_ERR_INVALID;
  const bool log = delta_log || delta_tstamps || delta_count;
  if (log && (!delta_log || !delta_tstamps || !delta_count || !poses || !tstamps || delta_cap <= 0))
    return DPVO_ERR_INVALID;
  hipStream_t s = as_stream(stream);
  ShiftArrays sa = {};
  long long maxw = 1;
  for (int a = 0; a < narrays; a++) {
    if (!frame_arrays[a] || bytes_per_frame[a] <= 0 || ring[a] < 0) return DPVO_ERR_INVALID;
    sa.base[a] = (char*)frame_arrays[a];
    sa.bytes[a] = bytes_per_frame[a];
    sa.ring[a] = ring[a];
    maxw = std::max<long long>(maxw, bytes_per_frame[a] % 4 ? bytes_per_frame[a]
                                                            : bytes_per_frame[a] / 4);
  }
  sa.count = narrays;
  if (log)
    hipLaunchKernelGGL(kf_delta_kernel, dim3(1), dim3(64), 0, s, (const int*)kf, poses, tstamps,
                       delta_log, delta_tstamps, (int*)delta_count, delta_cap, (int*)counts + 2);
  const int eg = (int)std::min<long long>((max_edges + 255) / 256, 1024);
  hipLaunchKernelGGL(kf_shift_edges_kernel, dim3(eg), dim3(256), 0, s, ii, jj, kk,
                     (const int*)counts, (const int*)kf, M);
  if (narrays) {
    const int fg = (int)std::min<long long>((maxw + 255) / 256, 4096);
    hipLaunchKernelGGL(kf_shift_frames_kernel, dim3(fg), dim3(256), 0, s, sa, (const int*)kf,
                       (const int*)st);
  }
  hipLaunchKernelGGL(kf_decrement_kernel, dim3(1), dim3(64), 0, s, (int*)st, (const int*)kf, M);
  return launch_status();
}

DPVO_EXPORT int dpvo_edges_loop(const float* poses, const float* patches, const float* intrinsics,
                                const int64_t* ix, int P, int M, const int32_t* st, int n_cap,
                                int32_t* last_global_ba, int removal_window, int max_edge_age,
                                int global_opt_freq, int keyframe_index, float backend_thresh,
                                int max_num_edges, int nms, float* work, int64_t* out_kk,
                                int64_t* out_jj, int32_t* out_n, int32_t* errors, void* stream) {
  if (!poses || !patches || !intrinsics || !ix || !st || !work || !out_kk || !out_jj || !out_n ||
      P < 2 || M <= 0 || n_cap < 0 || removal_window < 0 || max_edge_age < 0 || nms < 0 ||
      max_num_edges < 0)
    return DPVO_ERR_INVALID;
  LoopCfg c;
  c.P = P;
  c.M = M;
  c.rw = removal_window;
  c.age = max_edge_age;
  c.gof = global_opt_freq;
  c.ki = keyframe_index;
  c.nj = std::max(global_opt_freq - keyframe_index, 0);
  c.thresh = backend_thresh;
  c.max_edges = max_num_edges;
  c.nms = nms;
  c.n_cap = n_cap;
  const int nf_cap = std::min(std::max(n_cap - removal_window, 0), max_edge_age);
  const long long ng_cap = (long long)c.nj * nf_cap;
  // sort size, suppression bitmap (n_cap x nj bits) and the accepted-edge list
  if (ng_cap > kElSort || (long long)n_cap * c.nj > kElBits || max_num_edges > kElMaxOut)
    return DPVO_ERR_UNSUPPORTED;
  hipStream_t s = as_stream(stream);
  float* gflow = work;
  int* gi = reinterpret_cast<int*>(work + kElSort);
  if (ng_cap > 0) {
    hipLaunchKernelGGL(el_groups_kernel, dim3((unsigned)((ng_cap + 3) / 4)), dim3(256), 0, s,
                       poses, patches, intrinsics, ix, (const int*)st,
                       (const int*)last_global_ba, c, gflow, gi);
    const int rc = launch_status();
    if (rc) return rc;
  }
  const size_t lds = sizeof(unsigned long long) * kElSort + kElBits / 8;
  static const bool attr = hipFuncSetAttribute((const void*)el_select_kernel,
                                               hipFuncAttributeMaxDynamicSharedMemorySize,
                                               (int)lds) == hipSuccess;
  if (!attr) return DPVO_ERR_LAUNCH;
  hipLaunchKernelGGL(el_select_kernel, dim3(1), dim3(kElT), lds, s, gflow, gi, (const int*)st,
                     (int*)last_global_ba, c, out_kk, out_jj, (int*)out_n, (int*)errors);
  return launch_status();
}

// floats of the `work` buffer dpvo_edges_loop needs
DPVO_EXPORT size_t dpvo_edges_loop_work_floats(void) { return 2 * (size_t)kElSort; }
