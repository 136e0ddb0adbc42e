// pg.hip -- DPVO PatchGraph edge bookkeeping on the device.
//
// Reference: dpvo/dpvo.py append_factors (480-521) and remove_factors
// (523-568) over the static-shape PatchGraph buffers of dpvo/patchgraph.py
// (ii / jj / kk [MAX_EDGES], net [1, MAX_EDGES, DIM], weight / target
// [1, MAX_EDGES, 2], and the *_inac store of removed edges).  The reference
// keeps the edge counts on the host and syncs on every call (mask.sum().item(),
// boolean-mask gathers).  Here the counts live in a device int array and every
// operation is a fixed sequence of kernel launches with no host round trip:
//   counts[0] num_edges, [1] num_edges_inac, [2] error flags (1 append
//   overflow, 2 inactive store full -> removed edges not stored, as the
//   reference's warning), [3] / [4] staged new counts of a removal.
// Removal is a stable compaction (kept edges keep their order, removed ones
// are appended to the inactive store in order): bit-identical to the
// reference's boolean-mask indexing.  Active rows move to a second ("back")
// set of buffers (ping-pong; the caller swaps), so the move is race-free.
#include <algorithm>

#include "common.hpp"

namespace dpvo {
namespace {

constexpr int kPgT = 1024;

struct PgBufs {
  int64_t* ii;
  int64_t* jj;
  int64_t* kk;
  float* net;     // [max_edges][DIM] (may be null)
  float* weight;  // [max_edges][2]
  float* target;  // [max_edges][2]
};

// new edges (kk_new, jj_new) at [num, num + n); ii = ix[kk]; net rows zeroed
// n_dev (device count, e.g. edges_loop's output): n = min(*n_dev, n)
__global__ void pg_append_kernel(const int64_t* __restrict__ ix, const int64_t* __restrict__ kk_new,
                                 const int64_t* __restrict__ jj_new, int n, PgBufs b, int DIM,
                                 const int* __restrict__ counts, int max_edges,
                                 const int* __restrict__ n_dev) {
  if (n_dev) n = min(*n_dev, n);
  const int num = counts[0];
  if (num + n > max_edges) return;  // flagged by pg_count_kernel
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t < n) {
    const int64_t k = kk_new[t];
    b.kk[num + t] = k;
    b.jj[num + t] = jj_new[t];
    b.ii[num + t] = ix[k];
  }
  if (b.net) {
    const int64_t tot = (int64_t)n * DIM;
    for (int64_t q = t; q < tot; q += (int64_t)gridDim.x * blockDim.x)
      b.net[(int64_t)num * DIM + q] = 0.0f;
  }
}

__global__ void pg_count_kernel(int* counts, int n, int max_edges, const int* __restrict__ n_dev) {
  if (n_dev) n = min(*n_dev, n);
  if (threadIdx.x == 0 && blockIdx.x == 0) {
    if (counts[0] + n > max_edges) counts[2] |= 1;
    else counts[0] += n;
  }
}

// one workgroup: stable positions of kept / removed edges.
// flag source: mask (uint8, 1 = remove) or, when mask is null, the DPVO
// window rule ix[kk] < thresh (dpvo.py:684) except loop-closure edges
// (jj - ii > 30 and jj > lc_min, dpvo.py:685-688) when lc_min >= 0.
// n_dev (graph-replayed frames): thresh / lc_min are offsets from the device
// frame count *n_dev, lc_min only if lc_on.
__global__ void __launch_bounds__(kPgT) pg_plan_remove_kernel(
    const uint8_t* __restrict__ mask, const int64_t* __restrict__ ix, int64_t thresh,
    int64_t lc_min, PgBufs a, int* counts, int* __restrict__ pos, int store, int max_edges,
    const int* n_dev, int lc_on, const int* kf) {
  if (n_dev) {
    const int64_t n = *n_dev;
    thresh += n;
    lc_min = lc_on ? lc_min + n : -1;
  }
  __shared__ int wsum[kPgT / 64 + 1];
  __shared__ int carry[2];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int num = counts[0], inac = counts[1];
  if (tid == 0) carry[0] = carry[1] = 0;
  __syncthreads();
  for (int base = 0; base < num; base += kPgT) {
    const int e = base + tid;
    int rm = 0;
    if (e < num) {
      if (kf) {  // DPVO.keyframe frame drop (dpvo.py:638-645): kf = {drop, k}
        rm = (kf[0] && (a.ii[e] == kf[1] || a.jj[e] == kf[1])) ? 1 : 0;
      } else if (mask) {
        rm = mask[e] ? 1 : 0;
      } else {
        rm = ix[a.kk[e]] < thresh ? 1 : 0;
        if (rm && lc_min >= 0 && (a.jj[e] - a.ii[e]) > 30 && a.jj[e] > lc_min) rm = 0;
      }
    }
    // workgroup inclusive scan of rm (removed) -> kept count = index - removed
    int x = rm;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const int y = __shfl_up(x, o, 64);
      if (lane >= o) x += y;
    }
    if (lane == 63) wsum[wid] = x;
    __syncthreads();
    if (tid == 0) {
      int acc = 0;
      for (int w = 0; w < kPgT / 64; w++) {
        const int v = wsum[w];
        wsum[w] = acc;
        acc += v;
      }
      wsum[kPgT / 64] = acc;
    }
    __syncthreads();
    const int rm_before = carry[1] + wsum[wid] + x - rm;  // removed edges before e
    if (e < num) {
      const int kept_before = e - rm_before;
      // pos >= 0: new active slot; pos < 0: -(1 + inactive slot) or -1 - max (not stored)
      if (!rm) pos[e] = kept_before;
      else pos[e] = -(1 + ((store && inac + rm_before < max_edges) ? inac + rm_before : max_edges));
    }
    __syncthreads();
    if (tid == 0) carry[1] += wsum[kPgT / 64];
    __syncthreads();
  }
  if (tid == 0) {
    const int removed = carry[1];
    counts[3] = num - removed;
    // the reference stores all or nothing (dpvo.py:539-553)
    const bool fits = inac + removed <= max_edges;
    counts[4] = (store && fits) ? inac + removed : inac;
    if (store && !fits && removed > 0) counts[2] |= 2;
  }
}

// move every active row to its slot in the back buffers / the inactive store
__global__ void pg_move_kernel(PgBufs a, PgBufs back, PgBufs inac, int DIM,
                               const int* __restrict__ counts, const int* __restrict__ pos,
                               int store, int max_edges) {
  const int num = counts[0];
  const bool store_ok = store && counts[4] != counts[1];
  const int64_t t0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t e = t0; e < num; e += stride) {
    const int p = pos[e];
    if (p >= 0) {
      back.ii[p] = a.ii[e];
      back.jj[p] = a.jj[e];
      back.kk[p] = a.kk[e];
      reinterpret_cast<float2*>(back.weight)[p] = reinterpret_cast<const float2*>(a.weight)[e];
      reinterpret_cast<float2*>(back.target)[p] = reinterpret_cast<const float2*>(a.target)[e];
    } else if (store_ok) {
      const int q = -p - 1;
      if (q < max_edges) {
        inac.ii[q] = a.ii[e];
        inac.jj[q] = a.jj[e];
        inac.kk[q] = a.kk[e];
        reinterpret_cast<float2*>(inac.weight)[q] = reinterpret_cast<const float2*>(a.weight)[e];
        reinterpret_cast<float2*>(inac.target)[q] = reinterpret_cast<const float2*>(a.target)[e];
      }
    }
  }
  if (a.net) {  // hidden states of kept edges, 4 floats per thread
    const int d4 = DIM / 4;
    const int64_t tot = (int64_t)num * d4;
    for (int64_t q = t0; q < tot; q += stride) {
      const int64_t e = q / d4, c = q % d4;
      const int p = pos[e];
      if (p >= 0)
        reinterpret_cast<float4*>(back.net + (int64_t)p * DIM)[c] =
            reinterpret_cast<const float4*>(a.net + e * DIM)[c];
    }
  }
}

__global__ void pg_commit_kernel(int* counts) {
  if (threadIdx.x == 0 && blockIdx.x == 0) {
    counts[0] = counts[3];
    counts[1] = counts[4];
  }
}

PgBufs bufs(int64_t* ii, int64_t* jj, int64_t* kk, float* net, float* weight, float* target) {
  PgBufs b;
  b.ii = ii;
  b.jj = jj;
  b.kk = kk;
  b.net = net;
  b.weight = weight;
  b.target = target;
  return b;
}

}  // namespace
}  // namespace dpvo

using namespace dpvo;

static int pg_append_impl(const int64_t* ix, const int64_t* kk_new, const int64_t* jj_new, int n,
                          int64_t* ii, int64_t* jj, int64_t* kk, float* net, int DIM, int* counts,
                          int max_edges, void* stream, const int32_t* n_dev) {
  if (n <= 0) return DPVO_OK;
  if (!ix || !kk_new || !jj_new || !ii || !jj || !kk || !counts || max_edges <= 0 ||
      (net && DIM <= 0))
    return DPVO_ERR_INVALID;
  hipStream_t st = as_stream(stream);
  const int64_t work = net ? (int64_t)n * DIM : n;
  const int grid = (int)std::min<int64_t>((work + 255) / 256, 2048);
  hipLaunchKernelGGL(pg_append_kernel, dim3(grid < 1 ? 1 : grid), dim3(256), 0, st, ix, kk_new,
                     jj_new, n, bufs(ii, jj, kk, net, nullptr, nullptr), DIM, counts, max_edges,
                     (const int*)n_dev);
  int rc = launch_status();
  if (rc) return rc;
  hipLaunchKernelGGL(pg_count_kernel, dim3(1), dim3(64), 0, st, counts, n, max_edges,
                     (const int*)n_dev);
  return launch_status();
}

DPVO_EXPORT int dpvo_pg_append(const int64_t* ix, const int64_t* kk_new, const int64_t* jj_new,
                               int n, int64_t* ii, int64_t* jj, int64_t* kk, float* net, int DIM,
                               int* counts, int max_edges, void* stream) {
  return pg_append_impl(ix, kk_new, jj_new, n, ii, jj, kk, net, DIM, counts, max_edges, stream,
                        nullptr);
}

DPVO_EXPORT int dpvo_pg_append_dev(const int64_t* ix, const int64_t* kk_new, const int64_t* jj_new,
                                   const int32_t* n_dev, int n_cap, int64_t* ii, int64_t* jj,
                                   int64_t* kk, float* net, int DIM, int* counts, int max_edges,
                                   void* stream) {
  if (!n_dev) return DPVO_ERR_INVALID;
  return pg_append_impl(ix, kk_new, jj_new, n_cap, ii, jj, kk, net, DIM, counts, max_edges,
                        stream, n_dev);
}

static int pg_remove_impl(const uint8_t* mask, const int64_t* ix, int64_t thresh, int64_t lc_min,
                          int store, int64_t* ii, int64_t* jj, int64_t* kk, float* net,
                          float* weight, float* target, int64_t* ii_b, int64_t* jj_b,
                          int64_t* kk_b, float* net_b, float* weight_b, float* target_b,
                          int64_t* ii_i, int64_t* jj_i, int64_t* kk_i, float* weight_i,
                          float* target_i, int DIM, int* counts, int* pos, int max_edges,
                          void* stream, const int32_t* n_dev, int lc_on,
                          const int32_t* kf = nullptr) {
  if (!ii || !jj || !kk || !weight || !target || !ii_b || !jj_b || !kk_b || !weight_b ||
      !target_b || !counts || !pos || max_edges <= 0 || (!mask && !ix && !kf) || (net && !net_b) ||
      (net && (DIM <= 0 || DIM % 4)) || (store && (!ii_i || !jj_i || !kk_i || !weight_i || !target_i)))
    return DPVO_ERR_INVALID;
  hipStream_t st = as_stream(stream);
  const PgBufs a = bufs(ii, jj, kk, net, weight, target);
  const PgBufs b = bufs(ii_b, jj_b, kk_b, net_b, weight_b, target_b);
  const PgBufs in = bufs(ii_i, jj_i, kk_i, nullptr, weight_i, target_i);
  hipLaunchKernelGGL(pg_plan_remove_kernel, dim3(1), dim3(kPgT), 0, st, mask, ix, thresh, lc_min,
                     a, counts, pos, store, max_edges, (const int*)n_dev, lc_on,
                     (const int*)kf);
  int rc = launch_status();
  if (rc) return rc;
  const int64_t work = net ? (int64_t)max_edges * (DIM / 4) : max_edges;
  const int grid = (int)std::min<int64_t>((work + 255) / 256, 4096);
  hipLaunchKernelGGL(pg_move_kernel, dim3(grid), dim3(256), 0, st, a, b, in, DIM, counts, pos,
                     store, max_edges);
  rc = launch_status();
  if (rc) return rc;
  hipLaunchKernelGGL(pg_commit_kernel, dim3(1), dim3(64), 0, st, counts);
  return launch_status();
}

DPVO_EXPORT int dpvo_pg_remove(const uint8_t* mask, const int64_t* ix, int64_t thresh,
                               int64_t lc_min, int store, int64_t* ii, int64_t* jj, int64_t* kk,
                               float* net, float* weight, float* target, int64_t* ii_b,
                               int64_t* jj_b, int64_t* kk_b, float* net_b, float* weight_b,
                               float* target_b, int64_t* ii_i, int64_t* jj_i, int64_t* kk_i,
                               float* weight_i, float* target_i, int DIM, int* counts, int* pos,
                               int max_edges, void* stream) {
  return pg_remove_impl(mask, ix, thresh, lc_min, store, ii, jj, kk, net, weight, target, ii_b,
                        jj_b, kk_b, net_b, weight_b, target_b, ii_i, jj_i, kk_i, weight_i,
                        target_i, DIM, counts, pos, max_edges, stream, nullptr, 0);
}

DPVO_EXPORT int dpvo_pg_remove_window_dev(const int64_t* ix, const int32_t* n_dev, int64_t thresh_off,
                                          int64_t lc_off, int lc_on, int store, int64_t* ii,
                                          int64_t* jj, int64_t* kk, float* net, float* weight,
                                          float* target, int64_t* ii_b, int64_t* jj_b,
                                          int64_t* kk_b, float* net_b, float* weight_b,
                                          float* target_b, int64_t* ii_i, int64_t* jj_i,
                                          int64_t* kk_i, float* weight_i, float* target_i, int DIM,
                                          int* counts, int* pos, int max_edges, void* stream) {
  if (!n_dev || !ix) return DPVO_ERR_INVALID;
  return pg_remove_impl(nullptr, ix, thresh_off, lc_off, store, ii, jj, kk, net, weight, target,
                        ii_b, jj_b, kk_b, net_b, weight_b, target_b, ii_i, jj_i, kk_i, weight_i,
                        target_i, DIM, counts, pos, max_edges, stream, n_dev, lc_on);
}

DPVO_EXPORT int dpvo_pg_remove_frame_dev(const int32_t* kf, int64_t* ii, int64_t* jj, int64_t* kk,
                                         float* net, float* weight, float* target, int64_t* ii_b,
                                         int64_t* jj_b, int64_t* kk_b, float* net_b,
                                         float* weight_b, float* target_b, int DIM, int* counts,
                                         int* pos, int max_edges, void* stream) {
  if (!kf) return DPVO_ERR_INVALID;
  return pg_remove_impl(nullptr, nullptr, 0, -1, 0, ii, jj, kk, net, weight, target, ii_b, jj_b,
                        kk_b, net_b, weight_b, target_b, nullptr, nullptr, nullptr, nullptr,
                        nullptr, DIM, counts, pos, max_edges, stream, nullptr, 0, kf);
}
