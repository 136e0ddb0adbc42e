// ext_common.hpp -- shared glue of the cuda_corr / cuda_ba / lietorch_backends
// extension modules: device guard, current HIP stream, status -> RuntimeError.
#pragma once

#include <ATen/hip/impl/HIPGuardImplMasqueradingAsCUDA.h>
#include <ATen/hip/impl/HIPStreamMasqueradingAsCUDA.h>
#include <torch/extension.h>

#include "dpvo_hot.h"

namespace dpvo_ext {

inline void* current_stream() {
  return reinterpret_cast<void*>(c10::hip::getCurrentHIPStreamMasqueradingAsCUDA().stream());
}

// true while the current stream is being captured into a hipGraph
inline bool is_capturing() {
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  (void)hipStreamIsCapturing(c10::hip::getCurrentHIPStreamMasqueradingAsCUDA().stream(), &cs);
  return cs != hipStreamCaptureStatusNone;
}

inline void check_status(int st, const char* what) {
  TORCH_CHECK(st == DPVO_OK, what, " failed: ", dpvo_status_string(st), " (status ", st, ")");
}

inline void check_device(const torch::Tensor& t, const char* name) {
  TORCH_CHECK(t.is_cuda(), name, " must be a GPU (HIP) tensor; the MI355X build has no CPU path");
}

inline int dtype_code(const torch::Tensor& t) {
  switch (t.scalar_type()) {
    case torch::kFloat32: return DPVO_F32;
    case torch::kFloat16: return DPVO_F16;
    case torch::kFloat64: return DPVO_F64;
    default: TORCH_CHECK(false, "unsupported dtype ", t.scalar_type());
  }
  return -1;
}

inline torch::Tensor idx64(const torch::Tensor& t, const char* name) {
  check_device(t, name);
  TORCH_CHECK(t.scalar_type() == torch::kInt64, name, " must be int64 (long)");
  return t.contiguous();
}

}  // namespace dpvo_ext
