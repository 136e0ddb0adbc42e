// Latency of cross-lane broadcast chains in one wave (gfx950): a dependent
// v_fma chain, v_readlane (constant / SGPR lane) -> v_fma, and an LDS
// store -> load broadcast -> v_fma.  Prints cycles per step (s_memtime).
#include <hip/hip_runtime.h>
#include <stdio.h>

__global__ void k(float* out, long long* cyc, int mode, int steps) {
  __shared__ float sh[64];
  const int lane = threadIdx.x;
  float w = lane * 0.001f + 1.0f, c = 0.999f;
  __syncthreads();
  const long long t0 = __builtin_amdgcn_s_memtime();
  if (mode == 0) {
    for (int s = 0; s < steps; s++) w = w * c + 0.5f;
  } else if (mode == 1) {
    for (int s = 0; s < steps; s++) {
      const float x = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(w), 5));
      w = w - c * x;
    }
  } else if (mode == 2) {
    for (int s = 0; s < steps; s++) {
      const float x = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(w), s & 63));
      w = w - c * x;
    }
  } else if (mode == 3) {
    for (int s = 0; s < steps; s++) {
      if (lane == (s & 63)) sh[0] = w;
      __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront", "local");
      __builtin_amdgcn_wave_barrier();
      const float x = sh[0];
      w = w - c * x;
      __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront", "local");
      __builtin_amdgcn_wave_barrier();
    }
  } else if (mode == 5) {  // 4 independent chains
    float a = w + 1, b = w + 2, d = w + 3;
#pragma unroll 16
    for (int s = 0; s < steps; s++) {
      w = w * c + 0.5f;
      a = a * c + 0.5f;
      b = b * c + 0.5f;
      d = d * c + 0.5f;
    }
    w += a + b + d;
  } else if (mode == 6) {  // dependent chain, unrolled 16
#pragma unroll 16
    for (int s = 0; s < steps; s++) w = w * c + 0.5f;
  } else if (mode == 7) {  // dependent LDS loads (pointer chase)
    __shared__ int ch[64];
    ch[lane] = (lane + 1) & 63;
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront", "local");
    __builtin_amdgcn_wave_barrier();
    int p = lane;
#pragma unroll 16
    for (int s = 0; s < steps; s++) p = ch[p];
    w += p;
  } else if (mode == 8) {  // ds_write + ds_read round trip (same lane)
#pragma unroll 16
    for (int s = 0; s < steps; s++) {
      sh[lane] = w;
      __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront", "local");
      w = sh[lane] + 1.0f;
    }
  } else if (mode == 4) {  // readfirstlane-free: ds_bpermute broadcast
    for (int s = 0; s < steps; s++) {
      const float x = __int_as_float(__builtin_amdgcn_ds_bpermute((s & 63) << 2, __float_as_int(w)));
      w = w - c * x;
    }
  }
  const long long t1 = __builtin_amdgcn_s_memtime();
  out[lane] = w;
  if (lane == 0) *cyc = t1 - t0;
}

int main() {
  float* o;
  long long* c;
  hipMalloc(&o, 256);
  hipMalloc(&c, 8);
  const char* names[] = {"dep fma", "readlane(const)+fma", "readlane(sgpr)+fma", "lds bcast+fma",
                         "ds_bpermute+fma", "4 indep fma chains", "dep fma unroll16", "lds ptr chase", "lds st->ld"};
  for (int mm = 0; mm < 9; mm++) { const int m = (mm + 6) % 9;
    long long best = 1LL << 60;
    for (int r = 0; r < 50; r++) {
      hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, o, c, m, 1024);
      long long h;
      hipMemcpy(&h, c, 8, hipMemcpyDeviceToHost);
      if (h < best) best = h;
    }
    printf("%-22s %.1f cycles/step\n", names[m], best / 1024.0);
  }
  return 0;
}
