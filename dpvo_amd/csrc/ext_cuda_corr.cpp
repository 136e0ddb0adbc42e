// ext_cuda_corr.cpp -- the `cuda_corr` extension module (drop-in for
// dpvo/altcorr/correlation.cpp:57-63), bound to the C ABI in dpvo_hot.h.
#include "ext_common.hpp"

using namespace dpvo_ext;

// correlation.cpp:32-38 -> correlation_kernel.cu:232-272
std::vector<torch::Tensor> corr_forward(torch::Tensor fmap1, torch::Tensor fmap2,
                                        torch::Tensor coords, torch::Tensor ii, torch::Tensor jj,
                                        int radius) {
  check_device(fmap1, "fmap1");
  check_device(fmap2, "fmap2");
  check_device(coords, "coords");
  TORCH_CHECK(fmap1.dim() == 5 && fmap2.dim() == 5 && coords.dim() == 5,
              "corr: expected fmap1 [B,N1,C,H,W], fmap2 [B,N2,C,H2,W2], coords [B,M,2,H,W]");
  TORCH_CHECK(fmap1.scalar_type() == fmap2.scalar_type(), "fmap1/fmap2 dtype mismatch");
  TORCH_CHECK(coords.scalar_type() == torch::kFloat32, "coords must be float32");
  TORCH_CHECK(coords.size(2) == 2, "coords must be [B,M,2,H,W]");
  const c10::hip::OptionalHIPGuardMasqueradingAsCUDA guard(fmap1.device());
  fmap1 = fmap1.contiguous();
  coords = coords.contiguous();
  ii = idx64(ii, "ii");
  jj = idx64(jj, "jj");
  const int B = coords.size(0), M = coords.size(1), H = coords.size(3), W = coords.size(4);
  TORCH_CHECK(ii.numel() >= M && jj.numel() >= M, "ii/jj shorter than coords.size(1)");
  TORCH_CHECK(fmap1.size(3) == H && fmap1.size(4) == W, "fmap1 patch size != coords size");
  const int Dp = 2 * radius + 1;
  // a channels-last level ([B,N,C,H,W] view of [B,N,H,W,C] memory, e.g. a
  // DPVO pyramid allocated channels-last) takes the
  // matrix-core path as a one-level forward_levels (fp32 accumulation; the
  // result is returned in the fmap dtype, as the reference does) instead of
  // a transposing .contiguous() copy of the whole ring
  if (fmap2.permute({0, 1, 3, 4, 2}).is_contiguous() && fmap2.size(2) > 1) {
    auto o32 = torch::empty({B, M, Dp, Dp, H, W, 1}, fmap1.options().dtype(torch::kFloat32));
    const void* f2p = fmap2.data_ptr();
    const int H2 = fmap2.size(3), W2 = fmap2.size(4);
    const float one = 1.0f;
    const int st = dpvo_corr_forward_levels_nhwc(
        fmap1.data_ptr(), &f2p, &H2, &W2, &one, 1, coords.data_ptr<float>(),
        ii.data_ptr<int64_t>(), jj.data_ptr<int64_t>(), B, M, fmap1.size(2), H, W, fmap1.size(1),
        fmap2.size(1), radius, dtype_code(fmap1), o32.data_ptr<float>(), current_stream());
    if (st != DPVO_ERR_UNSUPPORTED) {
      check_status(st, "cuda_corr.forward");
      auto o = o32.view({B, M, Dp, Dp, H, W});
      return {fmap1.scalar_type() == torch::kFloat32 ? o : o.to(fmap1.scalar_type())};
    }
  }
  fmap2 = fmap2.contiguous();
  auto out = torch::empty({B, M, Dp, Dp, H, W}, fmap1.options());
  check_status(dpvo_corr_forward(fmap1.data_ptr(), fmap2.data_ptr(), coords.data_ptr<float>(),
                                 ii.data_ptr<int64_t>(), jj.data_ptr<int64_t>(), B, M,
                                 fmap1.size(2), H, W, fmap1.size(1), fmap2.size(1), fmap2.size(3),
                                 fmap2.size(4), radius, dtype_code(fmap1), out.data_ptr(),
                                 current_stream()),
               "cuda_corr.forward");
  return {out};
}

// Fused multi-level form (dpvo/dpvo.py:462-465): returns [B, M, Dp, Dp, H, W, L]
// float32 = torch.stack([corr(level l) for l], -1).
// src [..., C, H, W] contiguous -> dst: same shape, channels-last memory
// (dst.permute(..., H, W, C) contiguous), e.g. one frame of a pyramid level.
void feature_to_nhwc(torch::Tensor src, torch::Tensor dst) {
  check_device(src, "src");
  check_device(dst, "dst");
  TORCH_CHECK(src.dim() >= 3 && src.sizes() == dst.sizes(), "src / dst shapes differ");
  TORCH_CHECK(src.scalar_type() == dst.scalar_type(), "src / dst dtypes differ");
  const int d = src.dim();
  std::vector<int64_t> perm;
  for (int i = 0; i < d - 3; i++) perm.push_back(i);
  perm.push_back(d - 2);
  perm.push_back(d - 1);
  perm.push_back(d - 3);
  TORCH_CHECK(dst.permute(perm).is_contiguous(), "dst must be channels-last");
  const c10::hip::OptionalHIPGuardMasqueradingAsCUDA guard(src.device());
  src = src.contiguous();
  const int C = src.size(d - 3), H = src.size(d - 2), W = src.size(d - 1);
  const int count = src.numel() / ((int64_t)C * H * W);
  check_status(dpvo_feature_to_nhwc(src.data_ptr(), dst.data_ptr(), count, C, H, W,
                                    dtype_code(src), current_stream()),
               "cuda_corr.feature_to_nhwc");
}

// Frame insertion of a channels-last pyramid: src [C, H, W] (level-1 NCHW
// frame), dst[l] [C, H/s, W/s] views in channels-last memory (one ring slot).
void feature_pyramid_insert(torch::Tensor src, std::vector<torch::Tensor> dst,
                            std::vector<int64_t> scales) {
  check_device(src, "src");
  TORCH_CHECK(src.dim() == 3, "src must be [C, H, W]");
  TORCH_CHECK(dst.size() == scales.size() && !dst.empty(), "one scale per destination level");
  TORCH_CHECK(src.scalar_type() == torch::kFloat32 || src.scalar_type() == torch::kFloat16,
              "src must be float32 or float16");
  const c10::hip::OptionalHIPGuardMasqueradingAsCUDA guard(src.device());
  src = src.contiguous();
  const int C = src.size(0), H = src.size(1), W = src.size(2);
  std::vector<void*> ptrs;
  std::vector<int> sc;
  for (size_t l = 0; l < dst.size(); l++) {
    const torch::Tensor& d = dst[l];
    check_device(d, "dst");
    const int s = (int)scales[l];
    TORCH_CHECK(d.scalar_type() == src.scalar_type() && d.dim() == 3 && d.size(0) == C &&
                    s > 0 && d.size(1) == H / s && d.size(2) == W / s,
                "dst level ", l, " must be [C, H/s, W/s] of src's dtype");
    TORCH_CHECK(d.stride(0) == 1 && d.stride(2) == C && d.stride(1) == (int64_t)C * d.size(2),
                "dst level ", l, " must be channels-last");
    ptrs.push_back(d.data_ptr());
    sc.push_back(s);
  }
  check_status(dpvo_feature_pyramid_insert(src.data_ptr(), ptrs.data(), sc.data(),
                                           (int)ptrs.size(), C, H, W, dtype_code(src),
                                           current_stream()),
               "cuda_corr.feature_pyramid_insert");
}

// ring variant: slot = *slot_dev % mem read on the device (graph-replayed
// frames); rings[l] is the whole [B, mem, C, H/s, W/s] channels-last ring
void feature_pyramid_insert_ring(torch::Tensor src, std::vector<torch::Tensor> rings,
                                 std::vector<int64_t> scales, torch::Tensor slot_dev) {
  check_device(src, "src");
  check_device(slot_dev, "slot_dev");
  TORCH_CHECK(slot_dev.scalar_type() == torch::kInt32 && slot_dev.is_contiguous(),
              "slot_dev must be a contiguous int32 device tensor");
  TORCH_CHECK(src.dim() == 3, "src must be [C, H, W]");
  TORCH_CHECK(rings.size() == scales.size() && !rings.empty(), "one scale per ring level");
  TORCH_CHECK(src.scalar_type() == torch::kFloat32 || src.scalar_type() == torch::kFloat16,
              "src must be float32 or float16");
  const c10::hip::OptionalHIPGuardMasqueradingAsCUDA guard(src.device());
  src = src.contiguous();
  const int C = src.size(0), H = src.size(1), W = src.size(2);
  const int mem = rings[0].size(1);
  std::vector<void*> ptrs;
  std::vector<int64_t> slot_bytes;
  std::vector<int> sc;
  for (size_t l = 0; l < rings.size(); l++) {
    const torch::Tensor d = rings[l][0][0];  // slot 0 of the ring
    check_device(d, "ring");
    const int s = (int)scales[l];
    TORCH_CHECK(rings[l].dim() == 5 && rings[l].size(1) == mem, "rings must be [B, mem, C, h, w]");
    TORCH_CHECK(d.scalar_type() == src.scalar_type() && d.size(0) == C && s > 0 &&
                    d.size(1) == H / s && d.size(2) == W / s,
                "ring level ", l, " must be [C, H/s, W/s] of src's dtype");
    TORCH_CHECK(d.stride(0) == 1 && d.stride(2) == C && d.stride(1) == (int64_t)C * d.size(2),
                "ring level ", l, " must be channels-last");
    ptrs.push_back(d.data_ptr());
    slot_bytes.push_back(rings[l].stride(1) * (int64_t)rings[l].element_size());
    sc.push_back(s);
  }
  check_status(dpvo_feature_pyramid_insert_ring(src.data_ptr(), ptrs.data(), slot_bytes.data(),
                                                sc.data(), (int)ptrs.size(), C, H, W, mem,
                                                slot_dev.data_ptr<int32_t>(), dtype_code(src),
                                                current_stream()),
               "cuda_corr.feature_pyramid_insert_ring");
}

torch::Tensor corr_forward_levels(torch::Tensor fmap1, std::vector<torch::Tensor> fmap2,
                                  torch::Tensor coords, torch::Tensor ii, torch::Tensor jj,
                                  int radius, std::vector<double> scales,
                                  c10::optional<torch::Tensor> order) {
  check_device(fmap1, "fmap1");
  TORCH_CHECK(fmap2.size() == scales.size() && !fmap2.empty() && fmap2.size() <= 8,
              "one scale per pyramid level (1..8 levels)");
  const c10::hip::OptionalHIPGuardMasqueradingAsCUDA guard(fmap1.device());
  fmap1 = fmap1.contiguous();
  coords = coords.contiguous();
  ii = idx64(ii, "ii");
  jj = idx64(jj, "jj");
  TORCH_CHECK(coords.scalar_type() == torch::kFloat32 && coords.dim() == 5, "coords [B,M,2,H,W] f32");
  const int L = fmap2.size();
  std::vector<const void*> ptrs(L);
  std::vector<int> H2(L), W2(L);
  std::vector<float> sc(L);
  const int B = coords.size(0), M = coords.size(1), H = coords.size(3), W = coords.size(4);
  const int Dp = 2 * radius + 1;
  auto out = torch::empty({B, M, Dp, Dp, H, W, L}, fmap1.options().dtype(torch::kFloat32));
  // channels-last pyramid ([B,N,C,H,W] view of [B,N,H,W,C] memory): matrix-core path
  bool nhwc = true;
  for (int l = 0; l < L; l++) {
    check_device(fmap2[l], "fmap2");
    TORCH_CHECK(fmap2[l].dim() == 5, "fmap2 levels must be [B,N,C,H,W]");
    TORCH_CHECK(fmap2[l].scalar_type() == fmap1.scalar_type(), "fmap dtype mismatch");
    nhwc = nhwc && fmap2[l].permute({0, 1, 3, 4, 2}).is_contiguous() && fmap2[l].size(2) > 1;
    H2[l] = fmap2[l].size(3);
    W2[l] = fmap2[l].size(4);
    sc[l] = (float)scales[l];
  }
  if (nhwc) {
    for (int l = 0; l < L; l++) ptrs[l] = fmap2[l].data_ptr();
    const int32_t* ord = nullptr;
    if (order.has_value() && order->defined()) {
      check_device(*order, "order");
      TORCH_CHECK(order->scalar_type() == torch::kInt32 && order->is_contiguous() &&
                      order->numel() == M && B == 1,
                  "order: contiguous int32 [E] (B == 1)");
      ord = order->data_ptr<int32_t>();
    }
    const int st = dpvo_corr_forward_levels_nhwc_ordered(
        fmap1.data_ptr(), ptrs.data(), H2.data(), W2.data(), sc.data(), L,
        coords.data_ptr<float>(), ii.data_ptr<int64_t>(), jj.data_ptr<int64_t>(), ord, B, M,
        fmap1.size(2), H, W, fmap1.size(1), fmap2[0].size(1), radius, dtype_code(fmap1),
        out.data_ptr<float>(), current_stream());
    if (st != DPVO_ERR_UNSUPPORTED) {
      check_status(st, "cuda_corr.forward_levels");
      return out;
    }
  }
  for (int l = 0; l < L; l++) {
    fmap2[l] = fmap2[l].contiguous();
    ptrs[l] = fmap2[l].data_ptr();
  }
  check_status(dpvo_corr_forward_levels(fmap1.data_ptr(), ptrs.data(), H2.data(), W2.data(),
                                        sc.data(), L, coords.data_ptr<float>(),
                                        ii.data_ptr<int64_t>(), jj.data_ptr<int64_t>(), B, M,
                                        fmap1.size(2), H, W, fmap1.size(1), fmap2[0].size(1),
                                        radius, dtype_code(fmap1), out.data_ptr<float>(),
                                        current_stream()),
               "cuda_corr.forward_levels");
  return out;
}

// correlation.cpp:40-48 -> correlation_kernel.cu:275-325
std::vector<torch::Tensor> corr_backward(torch::Tensor fmap1, torch::Tensor fmap2,
                                         torch::Tensor coords, torch::Tensor ii, torch::Tensor jj,
                                         torch::Tensor corr_grad, int radius) {
  check_device(fmap1, "fmap1");
  check_device(corr_grad, "corr_grad");
  const c10::hip::OptionalHIPGuardMasqueradingAsCUDA guard(fmap1.device());
  const auto dtype = fmap1.scalar_type();
  // the atomic accumulation runs in fp32 for every input dtype
  auto f1 = fmap1.to(torch::kFloat32).contiguous();
  auto f2 = fmap2.to(torch::kFloat32).contiguous();
  coords = coords.to(torch::kFloat32).contiguous();
  auto g = corr_grad.to(torch::kFloat32).contiguous();
  ii = idx64(ii, "ii");
  jj = idx64(jj, "jj");
  const int B = coords.size(0), M = coords.size(1), H = coords.size(3), W = coords.size(4);
  auto g1 = torch::empty_like(f1);
  auto g2 = torch::empty_like(f2);
  check_status(dpvo_corr_backward(f1.data_ptr(), f2.data_ptr(), coords.data_ptr<float>(),
                                  ii.data_ptr<int64_t>(), jj.data_ptr<int64_t>(),
                                  g.data_ptr<float>(), B, M, f1.size(2), H, W, f1.size(1),
                                  f2.size(1), f2.size(3), f2.size(4), radius, DPVO_F32,
                                  g1.data_ptr(), g2.data_ptr(), current_stream()),
               "cuda_corr.backward");
  return {g1.to(dtype), g2.to(dtype)};
}

static std::vector<torch::Tensor> patchify_fwd_impl(torch::Tensor net, torch::Tensor coords,
                                                    int radius, bool clamp) {
  check_device(net, "net");
  check_device(coords, "coords");
  TORCH_CHECK(net.dim() == 4 && coords.dim() == 3 && coords.size(2) == 2,
              "patchify: expected net [B,C,H,W], coords [B,M,2]");
  const c10::hip::OptionalHIPGuardMasqueradingAsCUDA guard(net.device());
  net = net.contiguous();
  coords = coords.to(torch::kFloat32).contiguous();
  const int B = coords.size(0), M = coords.size(1), C = net.size(1), D = 2 * radius + 2;
  auto out = torch::empty({B, M, C, D, D}, net.options());
  check_status(dpvo_patchify_forward(net.data_ptr(), coords.data_ptr<float>(), B, C, net.size(2),
                                     net.size(3), M, radius, clamp ? 1 : 0, dtype_code(net),
                                     out.data_ptr(), current_stream()),
               "cuda_corr.patchify_forward");
  return {out};
}

// correlation.cpp:50-53 -> correlation_kernel.cu:327-346 (zero fill)
std::vector<torch::Tensor> patchify_forward(torch::Tensor net, torch::Tensor coords, int radius) {
  return patchify_fwd_impl(net, coords, radius, false);
}
// The fork's runtime patchify (clamp at the border), correlation_kernel.py:181-224
std::vector<torch::Tensor> patchify_forward_clamped(torch::Tensor net, torch::Tensor coords,
                                                    int radius) {
  return patchify_fwd_impl(net, coords, radius, true);
}

static std::vector<torch::Tensor> patchify_bwd_impl(torch::Tensor net, torch::Tensor coords,
                                                    torch::Tensor gradient, int radius,
                                                    bool clamp) {
  check_device(net, "net");
  check_device(gradient, "gradient");
  const c10::hip::OptionalHIPGuardMasqueradingAsCUDA guard(net.device());
  coords = coords.to(torch::kFloat32).contiguous();
  auto g = gradient.to(torch::kFloat32).contiguous();
  const int B = coords.size(0), M = coords.size(1), C = net.size(1);
  auto out = torch::empty({net.size(0), C, net.size(2), net.size(3)},
                          net.options().dtype(torch::kFloat32));
  check_status(dpvo_patchify_backward(g.data_ptr(), coords.data_ptr<float>(), B, C, net.size(2),
                                      net.size(3), M, radius, clamp ? 1 : 0, DPVO_F32,
                                      out.data_ptr(), current_stream()),
               "cuda_corr.patchify_backward");
  return {out.to(net.scalar_type())};
}

// correlation.cpp:55-58 -> correlation_kernel.cu:349-372
std::vector<torch::Tensor> patchify_backward(torch::Tensor net, torch::Tensor coords,
                                             torch::Tensor gradient, int radius) {
  return patchify_bwd_impl(net, coords, gradient, radius, false);
}
std::vector<torch::Tensor> patchify_backward_clamped(torch::Tensor net, torch::Tensor coords,
                                                     torch::Tensor gradient, int radius) {
  return patchify_bwd_impl(net, coords, gradient, radius, true);
}

PYBIND11_MODULE(TORCH_EXTENSION_NAME, m) {
  m.def("forward", &corr_forward, "CORR forward");
  m.def("backward", &corr_backward, "CORR backward");
  m.def("patchify_forward", &patchify_forward, "PATCHIFY forward");
  m.def("patchify_backward", &patchify_backward, "PATCHIFY backward");
  // additions (not in the reference surface)
  m.def("forward_levels", &corr_forward_levels, "CORR forward, all pyramid levels in one launch",
        py::arg("fmap1"), py::arg("fmap2"), py::arg("coords"), py::arg("ii"), py::arg("jj"),
        py::arg("radius"), py::arg("scales"), py::arg("order") = py::none());
  m.def("feature_pyramid_insert_ring", &feature_pyramid_insert_ring,
        "feature_pyramid_insert into ring slot *slot_dev % mem (device scalar, graph replay)");
  m.def("feature_pyramid_insert", &feature_pyramid_insert,
        "NCHW level-1 frame -> channels-last pyramid slot (all levels, one launch)");
  m.def("feature_to_nhwc", &feature_to_nhwc, "[..., C, H, W] -> channels-last copy into dst");
  m.def("patchify_forward_clamped", &patchify_forward_clamped, "PATCHIFY forward, border clamp");
  m.def("patchify_backward_clamped", &patchify_backward_clamped, "PATCHIFY backward, border clamp");
  m.attr("native_library") = dpvo_version();
}
