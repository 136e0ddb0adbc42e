// ext_lietorch.cpp -- the `lietorch_backends` extension module (drop-in for
// dpvo/lietorch/src/lietorch.cpp:286-316), bound to the C ABI in dpvo_hot.h.
// Group ids follow dispatch.h:24-45; this build implements SO3 (1) and SE3 (3),
// the groups on DPVO's hot path.
#include "ext_common.hpp"

using namespace dpvo_ext;

enum { OP_EXP = 0, OP_LOG, OP_INV, OP_MUL, OP_ADJ, OP_ADJT, OP_ACT, OP_ACT4, OP_MATRIX, OP_PROJ,
       OP_JINV };

static void check_group(int g) {
  TORCH_CHECK(g == 1 || g == 3, "lietorch_backends: group ", g,
              " not supported by the MI355X build (SO3=1, SE3=3 implemented)");
}
static int K_of(int g) { return g == 1 ? 3 : 6; }
static int N_of(int g) { return g == 1 ? 4 : 7; }

// lietorch.cpp:7 CHECK_CONTIGUOUS
#define CHECK_CONTIGUOUS(x) TORCH_CHECK(x.is_contiguous(), #x " must be contiguous")

static int lie_dtype(const torch::Tensor& t) {
  TORCH_CHECK(t.scalar_type() == torch::kFloat32 || t.scalar_type() == torch::kFloat64,
              "lietorch_backends: float32 / float64 only (dispatch.h:41-42)");
  return dtype_code(t);
}

static torch::Tensor fwd(int g, int op, torch::Tensor X, torch::Tensor Y, int out_dim) {
  check_group(g);
  check_device(X, "X");
  CHECK_CONTIGUOUS(X);
  if (Y.defined()) {
    CHECK_CONTIGUOUS(Y);
    TORCH_CHECK(Y.scalar_type() == X.scalar_type(), "dtype mismatch");
  }
  const c10::hip::OptionalHIPGuardMasqueradingAsCUDA guard(X.device());
  const int n = X.size(0);
  auto out = torch::empty({n, out_dim}, X.options());
  check_status(dpvo_lie_forward(g, op, lie_dtype(X), n, X.data_ptr(),
                                Y.defined() ? Y.data_ptr() : nullptr, out.data_ptr(),
                                current_stream()),
               "lietorch_backends forward");
  return out;
}

static std::vector<torch::Tensor> bwd(int g, int op, torch::Tensor grad, torch::Tensor X,
                                      torch::Tensor Y, int d0, int d1) {
  check_group(g);
  check_device(X, "X");
  CHECK_CONTIGUOUS(X);
  CHECK_CONTIGUOUS(grad);
  if (Y.defined()) CHECK_CONTIGUOUS(Y);
  const c10::hip::OptionalHIPGuardMasqueradingAsCUDA guard(X.device());
  const int n = X.size(0);
  auto o0 = torch::empty({n, d0}, grad.options());
  auto o1 = d1 > 0 ? torch::empty({n, d1}, grad.options()) : torch::Tensor();
  check_status(dpvo_lie_backward(g, op, lie_dtype(X), n, grad.data_ptr(), X.data_ptr(),
                                 Y.defined() ? Y.data_ptr() : nullptr, o0.data_ptr(),
                                 d1 > 0 ? o1.data_ptr() : nullptr, current_stream()),
               "lietorch_backends backward");
  if (d1 > 0) return {o0, o1};
  return {o0};
}

// ---- lietorch.cpp:18-283 ----
torch::Tensor expm(int g, torch::Tensor a) { return fwd(g, OP_EXP, a, {}, N_of(g)); }
std::vector<torch::Tensor> expm_backward(int g, torch::Tensor grad, torch::Tensor a) {
  return bwd(g, OP_EXP, grad, a, {}, K_of(g), 0);
}
torch::Tensor logm(int g, torch::Tensor X) { return fwd(g, OP_LOG, X, {}, K_of(g)); }
std::vector<torch::Tensor> logm_backward(int g, torch::Tensor grad, torch::Tensor X) {
  return bwd(g, OP_LOG, grad, X, {}, N_of(g), 0);
}
torch::Tensor inv(int g, torch::Tensor X) { return fwd(g, OP_INV, X, {}, N_of(g)); }
std::vector<torch::Tensor> inv_backward(int g, torch::Tensor grad, torch::Tensor X) {
  return bwd(g, OP_INV, grad, X, {}, N_of(g), 0);
}
torch::Tensor mul(int g, torch::Tensor X, torch::Tensor Y) { return fwd(g, OP_MUL, X, Y, N_of(g)); }
std::vector<torch::Tensor> mul_backward(int g, torch::Tensor grad, torch::Tensor X,
                                        torch::Tensor Y) {
  return bwd(g, OP_MUL, grad, X, Y, N_of(g), N_of(g));
}
torch::Tensor adj(int g, torch::Tensor X, torch::Tensor a) { return fwd(g, OP_ADJ, X, a, K_of(g)); }
std::vector<torch::Tensor> adj_backward(int g, torch::Tensor grad, torch::Tensor X,
                                        torch::Tensor a) {
  return bwd(g, OP_ADJ, grad, X, a, N_of(g), K_of(g));
}
torch::Tensor adjT(int g, torch::Tensor X, torch::Tensor a) {
  return fwd(g, OP_ADJT, X, a, K_of(g));
}
std::vector<torch::Tensor> adjT_backward(int g, torch::Tensor grad, torch::Tensor X,
                                         torch::Tensor a) {
  return bwd(g, OP_ADJT, grad, X, a, N_of(g), K_of(g));
}
torch::Tensor act(int g, torch::Tensor X, torch::Tensor p) { return fwd(g, OP_ACT, X, p, 3); }
std::vector<torch::Tensor> act_backward(int g, torch::Tensor grad, torch::Tensor X,
                                        torch::Tensor p) {
  return bwd(g, OP_ACT, grad, X, p, N_of(g), 3);
}
torch::Tensor act4(int g, torch::Tensor X, torch::Tensor p) { return fwd(g, OP_ACT4, X, p, 4); }
std::vector<torch::Tensor> act4_backward(int g, torch::Tensor grad, torch::Tensor X,
                                         torch::Tensor p) {
  return bwd(g, OP_ACT4, grad, X, p, N_of(g), 4);
}
torch::Tensor projector(int g, torch::Tensor X) {
  return fwd(g, OP_PROJ, X, {}, N_of(g) * N_of(g)).view({X.size(0), N_of(g), N_of(g)});
}
torch::Tensor as_matrix(int g, torch::Tensor X) {
  return fwd(g, OP_MATRIX, X, {}, 16).view({X.size(0), 4, 4});
}
torch::Tensor Jinv(int g, torch::Tensor X, torch::Tensor a) {
  return fwd(g, OP_JINV, X, a, K_of(g));
}

PYBIND11_MODULE(TORCH_EXTENSION_NAME, m) {
  m.def("expm", &expm, "exp map forward");
  m.def("expm_backward", &expm_backward, "exp map backward");
  m.def("logm", &logm, "log map forward");
  m.def("logm_backward", &logm_backward, "log map backward");
  m.def("inv", &inv, "inverse operator");
  m.def("inv_backward", &inv_backward, "inverse operator backward");
  m.def("mul", &mul, "group operator");
  m.def("mul_backward", &mul_backward, "group operator backward");
  m.def("adj", &adj, "adjoint operator");
  m.def("adj_backward", &adj_backward, "adjoint operator backward");
  m.def("adjT", &adjT, "transposed adjoint operator");
  m.def("adjT_backward", &adjT_backward, "transposed adjoint operator backward");
  m.def("act", &act, "action on point");
  m.def("act_backward", &act_backward, "action on point backward");
  m.def("act4", &act4, "action on homogeneous point");
  m.def("act4_backward", &act4_backward, "action on homogeneous point backward");
  m.def("as_matrix", &as_matrix, "convert to matrix");
  m.def("projector", &projector, "orthogonal projection matrix");
  m.def("Jinv", &Jinv, "left inverse jacobian operator");
  m.attr("native_library") = dpvo_version();
}
