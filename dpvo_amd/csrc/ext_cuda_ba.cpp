// ext_cuda_ba.cpp -- the `cuda_ba` extension module (drop-in for
// dpvo/fastba/ba.cpp:183-189), bound to the C ABI in dpvo_hot.h.
#include <map>
#include <mutex>
#include <string>

#include "ext_common.hpp"

using namespace dpvo_ext;

static torch::Tensor f32_contig(const torch::Tensor& t, const char* name) {
  check_device(t, name);
  // packed_accessor32<float> in the reference (ba_cuda.cu:496-501) rejects
  // other dtypes with a RuntimeError; keep that behaviour.
  TORCH_CHECK(t.scalar_type() == torch::kFloat32, name, " must be float32, got ",
              t.scalar_type());
  return t.contiguous();
}

// ---------------------------------------------------------------------------
// BA status surfacing.  Every forward ORs its status word into a sticky
// device int (one tiny kernel: graph-capturable, no sync) and, outside graph
// capture, copies it asynchronously to pinned host memory.  The next forward
// (or check_status()) reads a completed copy and raises RuntimeError when a
// fatal bit is set: 2 kk out of range, 4 / 8 large-graph structure limits,
// 16 cross-workgroup timeout (a dX = 0 step that the reference would not take).
// Bit 1 (Cholesky failed -> zero step, dpvo/ba.py:17-21) is recorded, not
// raised (the reference ignores `info`, ba_cuda.cu:547).  Errors therefore
// surface at most one call late, like an asynchronous HIP error.
// ---------------------------------------------------------------------------
namespace {
constexpr int kFatalBits = 2 | 4 | 8 | 16 | 32;
struct StatusSlot {
  torch::Tensor acc;     // device int32 [1], sticky OR of all statuses
  int* host = nullptr;   // pinned copy
  hipEvent_t ev = nullptr;
  bool pending = false;
  int last = 0;          // last status seen on the host (all bits)
};
std::mutex g_st_mu;
std::map<int, StatusSlot> g_st;

std::string describe_status(int s) {
  std::string m;
  if (s & 1) m += " [1: Cholesky failed, zero step]";
  if (s & 2) m += " [2: kk outside [0, num_patches)]";
  if (s & 4) m += " [4: a patch touches more free poses than the large-graph solver handles]";
  if (s & 8) m += " [8: too many border poses for the large-graph solver]";
  if (s & 16) m += " [16: cross-workgroup wait timed out]";
  if (s & 32) m += " [32: window graph exceeds the per-workgroup LDS capacity]";
  return m;
}

// consume a finished copy; raise on fatal bits (and reset the accumulator)
void consume(StatusSlot& sl, bool wait, void* stream) {
  if (!sl.pending) return;
  if (wait) {
    (void)hipEventSynchronize(sl.ev);
  } else if (hipEventQuery(sl.ev) != hipSuccess) {
    return;
  }
  sl.pending = false;
  sl.last = *sl.host;
  if (sl.last & kFatalBits) {
    const int s = sl.last;
    (void)hipMemsetAsync(sl.acc.data_ptr<int>(), 0, sizeof(int), (hipStream_t)stream);
    *sl.host = 0;
    TORCH_CHECK(false, "cuda_ba.forward: bundle adjustment reported status ", s,
                describe_status(s), "; the poses/patches of that call did not take the "
                "reference's step");
  }
}

StatusSlot& slot_for(const torch::Tensor& like) {
  const int dev = like.get_device();
  auto& sl = g_st[dev];
  if (!sl.acc.defined() && !is_capturing()) {
    sl.acc = torch::zeros({1}, like.options().dtype(torch::kInt32));
    TORCH_CHECK(hipHostMalloc((void**)&sl.host, sizeof(int), hipHostMallocDefault) == hipSuccess,
                "cuda_ba: pinned status buffer");
    *sl.host = 0;
    TORCH_CHECK(hipEventCreateWithFlags(&sl.ev, hipEventDisableTiming) == hipSuccess,
                "cuda_ba: status event");
    check_status(dpvo_ba_set_status_sink(sl.acc.data_ptr<int>()), "cuda_ba: status sink");
  }
  return sl;
}

void track_status(const torch::Tensor& ws, const torch::Tensor& like, int E, int t0, int t1) {
  std::lock_guard<std::mutex> lk(g_st_mu);
  auto& sl = slot_for(like);
  if (!sl.acc.defined()) return;  // first call happened inside a capture: untracked
  void* st = current_stream();
  check_status(dpvo_ba_status_accumulate(ws.data_ptr(), E, t0, t1, sl.acc.data_ptr<int>(), st),
               "cuda_ba.forward(status)");
  if (is_capturing() || sl.pending) return;
  TORCH_CHECK(hipMemcpyAsync(sl.host, sl.acc.data_ptr<int>(), sizeof(int), hipMemcpyDeviceToHost,
                             (hipStream_t)st) == hipSuccess, "cuda_ba: status copy");
  TORCH_CHECK(hipEventRecord(sl.ev, (hipStream_t)st) == hipSuccess, "cuda_ba: status event");
  sl.pending = true;
}

// before a launch: creates the device's slot (registering its status sink, so
// the window kernels of this very call report into it) and raises a finished
// earlier call's fatal status
void poll_status(const torch::Tensor& like) {
  if (is_capturing()) return;
  std::lock_guard<std::mutex> lk(g_st_mu);
  auto& sl = slot_for(like);
  consume(sl, false, current_stream());
}
}  // namespace

// cuda_ba.check_status(device): synchronise on the status of every forward
// issued so far on that device; raise on a fatal bit; return the OR of all
// bits seen (bit 1 included) and reset the accumulator.
int ba_check_status(torch::Tensor like) {
  TORCH_CHECK(!is_capturing(), "cuda_ba.check_status: not allowed during graph capture");
  const c10::hip::OptionalHIPGuardMasqueradingAsCUDA guard(like.device());
  std::lock_guard<std::mutex> lk(g_st_mu);
  auto it = g_st.find(like.get_device());
  if (it == g_st.end() || !it->second.acc.defined()) return 0;
  auto& sl = it->second;
  void* st = current_stream();
  consume(sl, true, st);  // may raise
  TORCH_CHECK(hipMemcpyAsync(sl.host, sl.acc.data_ptr<int>(), sizeof(int), hipMemcpyDeviceToHost,
                             (hipStream_t)st) == hipSuccess, "cuda_ba: status copy");
  TORCH_CHECK(hipEventRecord(sl.ev, (hipStream_t)st) == hipSuccess, "cuda_ba: status event");
  sl.pending = true;
  consume(sl, true, st);  // may raise
  const int all = sl.last;
  (void)hipMemsetAsync(sl.acc.data_ptr<int>(), 0, sizeof(int), (hipStream_t)st);
  *sl.host = 0;
  return all;
}

// ba.cpp:32-45 -> cuda_ba (ba_cuda.cu:433-582).  Mutates poses / patches.
static torch::Tensor ba_forward_ws(torch::Tensor poses, torch::Tensor patches,
                                      torch::Tensor intrinsics, torch::Tensor target,
                                      torch::Tensor weight, torch::Tensor lmbda, torch::Tensor ii,
                                      torch::Tensor jj, torch::Tensor kk, int PPF, int t0, int t1,
                                      int iterations, bool eff_impl) {
  check_device(poses, "poses");
  check_device(patches, "patches");
  TORCH_CHECK(poses.scalar_type() == torch::kFloat32 && patches.scalar_type() == torch::kFloat32,
              "poses / patches must be float32");
  // poses.view({-1,7}) / patches.view({-1,3,P,P}) must alias the caller's
  // storage for the in-place update to land (ba_cuda.cu:458-459)
  TORCH_CHECK(poses.is_contiguous() && patches.is_contiguous(),
              "poses and patches must be contiguous (updated in place)");
  const c10::hip::OptionalHIPGuardMasqueradingAsCUDA guard(poses.device());
  const int P = patches.size(-1);
  const int num_poses = poses.numel() / 7;
  const int num_patches = patches.numel() / (3 * P * P);
  intrinsics = f32_contig(intrinsics, "intrinsics");
  target = f32_contig(target, "target");
  weight = f32_contig(weight, "weight");
  lmbda = f32_contig(lmbda, "lmbda");
  ii = idx64(ii, "ii");
  jj = idx64(jj, "jj");
  kk = idx64(kk, "kk");
  const int E = ii.numel();
  TORCH_CHECK(jj.numel() == E && kk.numel() == E, "ii, jj, kk must have equal length");
  TORCH_CHECK(target.numel() >= 2 * E && weight.numel() >= 2 * E, "target/weight must be [.., E, 2]");
  if (E == 0 || iterations <= 0) return torch::Tensor();
  TORCH_CHECK(t1 - t0 <= dpvo_ba_max_free_poses(), "cuda_ba.forward: t1 - t0 = ", t1 - t0,
              " free poses exceeds this build's limit (", dpvo_ba_max_free_poses(), ")");
  poll_status(poses);  // a previous call's fatal status raises here
  const size_t wsb = dpvo_ba_workspace_bytes(E, t0, t1);
  auto ws = torch::empty({(int64_t)wsb}, poses.options().dtype(torch::kUInt8));
  check_status(dpvo_ba_forward(poses.data_ptr<float>(), patches.data_ptr<float>(),
                               intrinsics.data_ptr<float>(), target.data_ptr<float>(),
                               weight.data_ptr<float>(), lmbda.data_ptr<float>(),
                               ii.data_ptr<int64_t>(), jj.data_ptr<int64_t>(),
                               kk.data_ptr<int64_t>(), E, P, num_poses, num_patches, PPF, t0, t1,
                               iterations, eff_impl ? 1 : 0, ws.data_ptr(), wsb,
                               current_stream()),
               "cuda_ba.forward");
  track_status(ws, poses, E, t0, t1);
  return ws;
}

std::vector<torch::Tensor> ba_forward(torch::Tensor poses, torch::Tensor patches,
                                      torch::Tensor intrinsics, torch::Tensor target,
                                      torch::Tensor weight, torch::Tensor lmbda, torch::Tensor ii,
                                      torch::Tensor jj, torch::Tensor kk, int PPF, int t0, int t1,
                                      int iterations, bool eff_impl) {
  ba_forward_ws(poses, patches, intrinsics, target, weight, lmbda, ii, jj, kk, PPF, t0, t1,
                iterations, eff_impl);
  return {};
}

// Split call (dpvo_ba_plan / dpvo_ba_forward_planned): plan(...) -> workspace,
// reads ii / jj / kk only (may run on a side stream concurrently with A-CORR);
// forward_planned(ws, ...) runs the iterations.  Same results as forward().
bool ba_plan_supported(int E, int t0, int t1, int P) { return dpvo_ba_plan_supported(E, t0, t1, P); }

torch::Tensor ba_plan(torch::Tensor ii, torch::Tensor jj, torch::Tensor kk, int64_t num_patches,
                      int64_t num_poses, int t0, int t1) {
  ii = idx64(ii, "ii");
  jj = idx64(jj, "jj");
  kk = idx64(kk, "kk");
  const c10::hip::OptionalHIPGuardMasqueradingAsCUDA guard(ii.device());
  const int E = ii.numel();
  TORCH_CHECK(jj.numel() == E && kk.numel() == E, "ii, jj, kk must have equal length");
  const size_t wsb = dpvo_ba_workspace_bytes(E, t0, t1);
  auto ws = torch::empty({(int64_t)wsb}, ii.options().dtype(torch::kUInt8));
  check_status(dpvo_ba_plan(ii.data_ptr<int64_t>(), jj.data_ptr<int64_t>(), kk.data_ptr<int64_t>(),
                            E, (int)num_patches, (int)num_poses, t0, t1, ws.data_ptr(), wsb,
                            current_stream()),
               "cuda_ba.plan");
  return ws;
}

std::vector<int64_t> ba_plan_offsets(int64_t E, int t0, int t1) {
  std::vector<int64_t> o(5);
  check_status(dpvo_ba_plan_offsets((int)E, t0, t1, o.data()), "cuda_ba.plan_offsets");
  return o;
}

void ba_forward_planned(torch::Tensor ws, torch::Tensor poses, torch::Tensor patches,
                        torch::Tensor intrinsics, torch::Tensor target, torch::Tensor weight,
                        torch::Tensor lmbda, torch::Tensor ii, torch::Tensor jj, torch::Tensor kk,
                        int t0, int t1, int iterations) {
  check_device(poses, "poses");
  check_device(patches, "patches");
  TORCH_CHECK(poses.scalar_type() == torch::kFloat32 && patches.scalar_type() == torch::kFloat32,
              "poses / patches must be float32");
  TORCH_CHECK(poses.is_contiguous() && patches.is_contiguous(),
              "poses and patches must be contiguous (updated in place)");
  const c10::hip::OptionalHIPGuardMasqueradingAsCUDA guard(poses.device());
  const int P = patches.size(-1);
  const int num_poses = poses.numel() / 7;
  const int num_patches = patches.numel() / (3 * P * P);
  intrinsics = f32_contig(intrinsics, "intrinsics");
  target = f32_contig(target, "target");
  weight = f32_contig(weight, "weight");
  lmbda = f32_contig(lmbda, "lmbda");
  ii = idx64(ii, "ii");
  jj = idx64(jj, "jj");
  kk = idx64(kk, "kk");
  const int E = ii.numel();
  TORCH_CHECK(target.numel() >= 2 * E && weight.numel() >= 2 * E, "target/weight must be [.., E, 2]");
  if (E == 0 || iterations <= 0) return;
  poll_status(poses);
  check_status(dpvo_ba_forward_planned(poses.data_ptr<float>(), patches.data_ptr<float>(),
                                       intrinsics.data_ptr<float>(), target.data_ptr<float>(),
                                       weight.data_ptr<float>(), lmbda.data_ptr<float>(),
                                       ii.data_ptr<int64_t>(), jj.data_ptr<int64_t>(),
                                       kk.data_ptr<int64_t>(), E, P, num_poses, num_patches, t0,
                                       t1, iterations, ws.data_ptr(), ws.numel(), current_stream()),
               "cuda_ba.forward_planned");
  track_status(ws, poses, E, t0, t1);
}

// Same call; returns the 2432 phase marks (100 MHz ticks: [0, 128) phases; window kernel
// [128 + 256 it + g] / [640 + 256 it + g] per-workgroup assembled / partials seen, [1152 + g]
// setup done, [1408 + g] iteration 0 assembled before its reduction) followed by the
// multi-kernel path's per-workgroup marks.
torch::Tensor ba_forward_marks(torch::Tensor poses, torch::Tensor patches,
                               torch::Tensor intrinsics, torch::Tensor target, torch::Tensor weight,
                               torch::Tensor lmbda, torch::Tensor ii, torch::Tensor jj,
                               torch::Tensor kk, int PPF, int t0, int t1, int iterations,
                               bool eff_impl) {
  check_status(dpvo_ba_set_marks(1), "cuda_ba.forward_marks");
  torch::Tensor ws;
  try {
    ws = ba_forward_ws(poses, patches, intrinsics, target, weight, lmbda, ii, jj, kk, PPF, t0, t1,
                       iterations, eff_impl);
  } catch (...) {
    dpvo_ba_set_marks(0);
    throw;
  }
  check_status(dpvo_ba_set_marks(0), "cuda_ba.forward_marks");
  auto out = torch::zeros({2432}, poses.options().dtype(torch::kInt64));
  if (!ws.defined()) return out;
  check_status(dpvo_ba_phase_marks(ws.data_ptr(), ii.numel(), t0, t1, out.data_ptr<int64_t>(),
                                   current_stream()),
               "cuda_ba.forward_marks");
  const int N = t1 - t0, E = ii.numel();
  const int64_t grid = N * (N + 1) / 2;
  auto wg = torch::zeros({2 * grid}, out.options());
  check_status(dpvo_ba_workgroup_marks(ws.data_ptr(), E, t0, t1, wg.data_ptr<int64_t>(),
                                       current_stream()),
               "cuda_ba.forward_marks");
  return torch::cat({out, wg});
}

// The marks a workspace holds (after launches made with set_marks(true)).
torch::Tensor ba_workspace_marks(torch::Tensor ws, int64_t E, int t0, int t1) {
  check_device(ws, "ws");
  TORCH_CHECK(E >= 0 && t1 > t0, "cuda_ba.workspace_marks: bad E / window");
  TORCH_CHECK((size_t)ws.nbytes() >= dpvo_ba_workspace_bytes((int)E, t0, t1),
              "cuda_ba.workspace_marks: ws is not a BA workspace planned for (E, t0, t1)");
  auto out = torch::zeros({2432}, ws.options().dtype(torch::kInt64));
  check_status(dpvo_ba_phase_marks(ws.data_ptr(), (int)E, t0, t1, out.data_ptr<int64_t>(),
                                   current_stream()),
               "cuda_ba.workspace_marks");
  return out;
}

// Same call; returns the pose step dX [N, 6] (fp64) of the last iteration
// (ba_cuda.cu:561-562) -- the parity tests' view of the solve.
torch::Tensor ba_forward_dx(torch::Tensor poses, torch::Tensor patches, torch::Tensor intrinsics,
                            torch::Tensor target, torch::Tensor weight, torch::Tensor lmbda,
                            torch::Tensor ii, torch::Tensor jj, torch::Tensor kk, int PPF, int t0,
                            int t1, int iterations, bool eff_impl) {
  auto ws = ba_forward_ws(poses, patches, intrinsics, target, weight, lmbda, ii, jj, kk, PPF, t0,
                          t1, iterations, eff_impl);
  const int N = t1 > t0 ? t1 - t0 : 0;
  auto out = torch::zeros({N, 6}, poses.options().dtype(torch::kFloat64));
  if (!ws.defined() || N == 0) return out;
  check_status(dpvo_ba_last_dx(ws.data_ptr(), ii.numel(), t0, t1, out.data_ptr<double>(),
                               current_stream()),
               "cuda_ba.forward_dx");
  return out;
}

// dX [N, 6] of the last iteration of forward_planned(_dev) on workspace ws
torch::Tensor ba_last_dx(torch::Tensor ws, int64_t E, int t0, int t1) {
  const int N = t1 > t0 ? t1 - t0 : 0;
  auto out = torch::zeros({N, 6}, ws.options().dtype(torch::kFloat64));
  if (N == 0) return out;
  check_status(dpvo_ba_last_dx(ws.data_ptr(), (int)E, t0, t1, out.data_ptr<double>(),
                               current_stream()),
               "cuda_ba.last_dx");
  return out;
}

// ba.cpp:47-53 -> cuda_reproject (ba_cuda.cu:585-616)
torch::Tensor ba_reproject(torch::Tensor poses, torch::Tensor patches, torch::Tensor intrinsics,
                           torch::Tensor ii, torch::Tensor jj, torch::Tensor kk) {
  poses = f32_contig(poses, "poses");
  patches = f32_contig(patches, "patches");
  intrinsics = f32_contig(intrinsics, "intrinsics");
  const c10::hip::OptionalHIPGuardMasqueradingAsCUDA guard(poses.device());
  ii = idx64(ii, "ii");
  jj = idx64(jj, "jj");
  kk = idx64(kk, "kk");
  const int P = patches.size(-1);
  const int E = ii.numel();
  auto coords = torch::empty({E, 2, P, P}, poses.options());
  check_status(dpvo_reproject(poses.data_ptr<float>(), patches.data_ptr<float>(),
                              intrinsics.data_ptr<float>(), ii.data_ptr<int64_t>(),
                              jj.data_ptr<int64_t>(), kk.data_ptr<int64_t>(), E, P,
                              poses.numel() / 7, patches.numel() / (3 * P * P),
                              coords.data_ptr<float>(), current_stream()),
               "cuda_ba.reproject");
  return coords.view({1, E, 2, P, P});
}

// reproject + the A-CORR edge order (edges grouped by target frame) in one launch
std::vector<torch::Tensor> ba_reproject_ordered(torch::Tensor poses, torch::Tensor patches,
                                                torch::Tensor intrinsics, torch::Tensor ii,
                                                torch::Tensor jj, torch::Tensor kk, int N2) {
  poses = f32_contig(poses, "poses");
  patches = f32_contig(patches, "patches");
  intrinsics = f32_contig(intrinsics, "intrinsics");
  const c10::hip::OptionalHIPGuardMasqueradingAsCUDA guard(poses.device());
  ii = idx64(ii, "ii");
  jj = idx64(jj, "jj");
  kk = idx64(kk, "kk");
  const int P = patches.size(-1);
  const int E = ii.numel();
  auto coords = torch::empty({E, 2, P, P}, poses.options());
  auto order = torch::empty({E}, poses.options().dtype(torch::kInt32));
  check_status(dpvo_reproject_ordered(poses.data_ptr<float>(), patches.data_ptr<float>(),
                                      intrinsics.data_ptr<float>(), ii.data_ptr<int64_t>(),
                                      jj.data_ptr<int64_t>(), kk.data_ptr<int64_t>(), E, P,
                                      poses.numel() / 7, patches.numel() / (3 * P * P), N2,
                                      coords.data_ptr<float>(), order.data_ptr<int32_t>(),
                                      current_stream()),
               "cuda_ba.reproject_ordered");
  return {coords.view({1, E, 2, P, P}), order};
}

// reproject + edge order + BA plan (workspace for forward_planned) in one launch
std::vector<torch::Tensor> ba_reproject_ordered_plan(torch::Tensor poses, torch::Tensor patches,
                                                     torch::Tensor intrinsics, torch::Tensor ii,
                                                     torch::Tensor jj, torch::Tensor kk, int N2,
                                                     int t0, int t1) {
  poses = f32_contig(poses, "poses");
  patches = f32_contig(patches, "patches");
  intrinsics = f32_contig(intrinsics, "intrinsics");
  const c10::hip::OptionalHIPGuardMasqueradingAsCUDA guard(poses.device());
  ii = idx64(ii, "ii");
  jj = idx64(jj, "jj");
  kk = idx64(kk, "kk");
  const int P = patches.size(-1);
  const int E = ii.numel();
  TORCH_CHECK(jj.numel() == E && kk.numel() == E, "ii, jj, kk must have equal length");
  auto coords = torch::empty({E, 2, P, P}, poses.options());
  auto order = torch::empty({E}, poses.options().dtype(torch::kInt32));
  const size_t wsb = dpvo_ba_workspace_bytes(E, t0, t1);
  auto ws = torch::empty({(int64_t)wsb}, poses.options().dtype(torch::kUInt8));
  check_status(dpvo_reproject_ordered_plan(
                   poses.data_ptr<float>(), patches.data_ptr<float>(), intrinsics.data_ptr<float>(),
                   ii.data_ptr<int64_t>(), jj.data_ptr<int64_t>(), kk.data_ptr<int64_t>(), E, P,
                   poses.numel() / 7, patches.numel() / (3 * P * P), N2, coords.data_ptr<float>(),
                   order.data_ptr<int32_t>(), t0, t1, ws.data_ptr(), wsb, current_stream()),
               "cuda_ba.reproject_ordered_plan");
  return {coords.view({1, E, 2, P, P}), order, ws};
}

// ... plus the new frame's pyramid insertion in the same launch (src [C, H, W]
// NCHW, dst[l] the channels-last [C, H/s, W/s] slot view of level l)
std::vector<torch::Tensor> ba_reproject_ordered_plan_insert(
    torch::Tensor poses, torch::Tensor patches, torch::Tensor intrinsics, torch::Tensor ii,
    torch::Tensor jj, torch::Tensor kk, int N2, int t0, int t1, torch::Tensor src,
    std::vector<torch::Tensor> dst, std::vector<int64_t> scales) {
  poses = f32_contig(poses, "poses");
  patches = f32_contig(patches, "patches");
  intrinsics = f32_contig(intrinsics, "intrinsics");
  const c10::hip::OptionalHIPGuardMasqueradingAsCUDA guard(poses.device());
  ii = idx64(ii, "ii");
  jj = idx64(jj, "jj");
  kk = idx64(kk, "kk");
  check_device(src, "src");
  TORCH_CHECK(src.dim() == 3, "src must be [C, H, W]");
  TORCH_CHECK(src.scalar_type() == torch::kFloat32 || src.scalar_type() == torch::kFloat16,
              "src must be float32 or float16");
  TORCH_CHECK(dst.size() == scales.size() && !dst.empty(), "one scale per destination level");
  src = src.contiguous();
  const int C = src.size(0), H = src.size(1), W = src.size(2);
  std::vector<void*> ptrs;
  std::vector<int> sc;
  for (size_t l = 0; l < dst.size(); l++) {
    const torch::Tensor& d = dst[l];
    check_device(d, "dst");
    const int s = (int)scales[l];
    TORCH_CHECK(d.scalar_type() == src.scalar_type() && d.dim() == 3 && d.size(0) == C && s > 0 &&
                    d.size(1) == H / s && d.size(2) == W / s,
                "dst level ", l, " must be [C, H/s, W/s] of src's dtype");
    TORCH_CHECK(d.stride(0) == 1 && d.stride(2) == C && d.stride(1) == (int64_t)C * d.size(2),
                "dst level ", l, " must be channels-last");
    ptrs.push_back(d.data_ptr());
    sc.push_back(s);
  }
  const int P = patches.size(-1);
  const int E = ii.numel();
  TORCH_CHECK(jj.numel() == E && kk.numel() == E, "ii, jj, kk must have equal length");
  auto coords = torch::empty({E, 2, P, P}, poses.options());
  auto order = torch::empty({E}, poses.options().dtype(torch::kInt32));
  const size_t wsb = dpvo_ba_workspace_bytes(E, t0, t1);
  auto ws = torch::empty({(int64_t)wsb}, poses.options().dtype(torch::kUInt8));
  check_status(dpvo_reproject_ordered_plan_insert(
                   poses.data_ptr<float>(), patches.data_ptr<float>(), intrinsics.data_ptr<float>(),
                   ii.data_ptr<int64_t>(), jj.data_ptr<int64_t>(), kk.data_ptr<int64_t>(), E, P,
                   poses.numel() / 7, patches.numel() / (3 * P * P), N2, coords.data_ptr<float>(),
                   order.data_ptr<int32_t>(), t0, t1, ws.data_ptr(), wsb, src.data_ptr(),
                   ptrs.data(), sc.data(), (int)ptrs.size(), C, H, W, dtype_code(src),
                   current_stream()),
               "cuda_ba.reproject_ordered_plan_insert");
  return {coords.view({1, E, 2, P, P}), order, ws};
}

// Device-t0 variants (graph-replayed DPVO updates: the window start moves
// every frame while shapes stay fixed): t0_dev is an int32 device scalar, N =
// t1 - t0 the (fixed) number of free poses.
static const int32_t* dev_scalar(const torch::Tensor& t, const char* name) {
  check_device(t, name);
  TORCH_CHECK(t.scalar_type() == torch::kInt32 && t.numel() >= 1 && t.is_contiguous(), name,
              " must be a contiguous int32 device tensor");
  return t.data_ptr<int32_t>();
}

std::vector<torch::Tensor> ba_reproject_ordered_plan_dev(torch::Tensor poses, torch::Tensor patches,
                                                         torch::Tensor intrinsics, torch::Tensor ii,
                                                         torch::Tensor jj, torch::Tensor kk, int N2,
                                                         torch::Tensor t0_dev, int N) {
  poses = f32_contig(poses, "poses");
  patches = f32_contig(patches, "patches");
  intrinsics = f32_contig(intrinsics, "intrinsics");
  const c10::hip::OptionalHIPGuardMasqueradingAsCUDA guard(poses.device());
  ii = idx64(ii, "ii");
  jj = idx64(jj, "jj");
  kk = idx64(kk, "kk");
  const int P = patches.size(-1);
  const int E = ii.numel();
  TORCH_CHECK(jj.numel() == E && kk.numel() == E, "ii, jj, kk must have equal length");
  auto coords = torch::empty({E, 2, P, P}, poses.options());
  auto order = torch::empty({E}, poses.options().dtype(torch::kInt32));
  const size_t wsb = dpvo_ba_workspace_bytes(E, 0, N);
  auto ws = torch::empty({(int64_t)wsb}, poses.options().dtype(torch::kUInt8));
  check_status(dpvo_reproject_ordered_plan_dev(
                   poses.data_ptr<float>(), patches.data_ptr<float>(), intrinsics.data_ptr<float>(),
                   ii.data_ptr<int64_t>(), jj.data_ptr<int64_t>(), kk.data_ptr<int64_t>(), E, P,
                   poses.numel() / 7, patches.numel() / (3 * P * P), N2, coords.data_ptr<float>(),
                   order.data_ptr<int32_t>(), dev_scalar(t0_dev, "t0_dev"), N, ws.data_ptr(), wsb,
                   current_stream()),
               "cuda_ba.reproject_ordered_plan_dev");
  return {coords.view({1, E, 2, P, P}), order, ws};
}

void ba_forward_planned_dev(torch::Tensor ws, torch::Tensor poses, torch::Tensor patches,
                            torch::Tensor intrinsics, torch::Tensor target, torch::Tensor weight,
                            torch::Tensor lmbda, torch::Tensor ii, torch::Tensor jj,
                            torch::Tensor kk, torch::Tensor t0_dev, int N, int iterations) {
  check_device(poses, "poses");
  check_device(patches, "patches");
  TORCH_CHECK(poses.scalar_type() == torch::kFloat32 && patches.scalar_type() == torch::kFloat32,
              "poses / patches must be float32");
  TORCH_CHECK(poses.is_contiguous() && patches.is_contiguous(),
              "poses and patches must be contiguous (updated in place)");
  const c10::hip::OptionalHIPGuardMasqueradingAsCUDA guard(poses.device());
  const int P = patches.size(-1);
  intrinsics = f32_contig(intrinsics, "intrinsics");
  target = f32_contig(target, "target");
  weight = f32_contig(weight, "weight");
  lmbda = f32_contig(lmbda, "lmbda");
  ii = idx64(ii, "ii");
  jj = idx64(jj, "jj");
  kk = idx64(kk, "kk");
  const int E = ii.numel();
  TORCH_CHECK(jj.numel() == E && kk.numel() == E && target.numel() == 2 * (int64_t)E &&
                  weight.numel() == 2 * (int64_t)E,
              "ii / jj / kk / target / weight sizes disagree");
  check_status(dpvo_ba_forward_planned_dev(
                   poses.data_ptr<float>(), patches.data_ptr<float>(), intrinsics.data_ptr<float>(),
                   target.data_ptr<float>(), weight.data_ptr<float>(), lmbda.data_ptr<float>(),
                   ii.data_ptr<int64_t>(), jj.data_ptr<int64_t>(), kk.data_ptr<int64_t>(), E, P,
                   poses.numel() / 7, patches.numel() / (3 * P * P), dev_scalar(t0_dev, "t0_dev"),
                   N, iterations, ws.data_ptr(), ws.numel(), current_stream()),
               "cuda_ba.forward_planned_dev");
}

// ba.cpp:59-97 (host loop in the reference; here one O(E^2) LDS-tiled kernel)
std::vector<torch::Tensor> ba_neighbors(torch::Tensor ii, torch::Tensor jj) {
  ii = idx64(ii, "ii");
  jj = idx64(jj, "jj");
  const c10::hip::OptionalHIPGuardMasqueradingAsCUDA guard(ii.device());
  const int E = ii.numel();
  auto ix = torch::empty({E}, ii.options());
  auto jx = torch::empty({E}, ii.options());
  check_status(dpvo_neighbors(ii.data_ptr<int64_t>(), jj.data_ptr<int64_t>(), E,
                              ix.data_ptr<int64_t>(), jx.data_ptr<int64_t>(), current_stream()),
               "cuda_ba.neighbors");
  return {ix, jx};
}

// ba.cpp:120-180: Sim3 pose-graph solve of the loop-closure backend
// (optim_utils.py:229).  Like the reference it accepts tensors on any device
// and returns delta on res.device() (ba.cpp:123-129, 170): host inputs (the
// loop-closure worker runs perform_updates on CPU tensors, long_term.py:258)
// are copied to the current HIP device, solved there, and copied back.
// Assembly of A = J^T J (+ damping) and b = -J^T res on the device (pgo.hip,
// fp64 like the reference's Eigen system); the SPD solve of the top-left
// freen*7 block by the device Cholesky in fp64; delta returned as f32 [n, 7]
// with the rows of fixed poses zero (ba.cpp:103-118).  A factorisation that
// fails (NaN / not positive definite) raises RuntimeError instead of
// returning garbage (the reference leaves Eigen's info unchecked).
std::vector<torch::Tensor> ba_solve_system(torch::Tensor J_Ginv_i, torch::Tensor J_Ginv_j,
                                           torch::Tensor ii, torch::Tensor jj, torch::Tensor res,
                                           double ep, double lm, int freen) {
  const torch::Device out_dev = res.device();
  torch::Device dev = out_dev;
  if (!res.is_cuda()) {
    TORCH_CHECK(torch::cuda::is_available(),
                "cuda_ba.solve_system: no HIP device (the MI355X build has no CPU path)");
    dev = torch::Device(torch::kCUDA, c10::hip::current_device());
  }
  const c10::hip::OptionalHIPGuardMasqueradingAsCUDA guard(dev);
  J_Ginv_i = J_Ginv_i.to(dev);
  J_Ginv_j = J_Ginv_j.to(dev);
  ii = ii.to(dev);
  jj = jj.to(dev);
  res = res.to(dev);
  J_Ginv_i = f32_contig(J_Ginv_i, "J_Ginv_i");
  J_Ginv_j = f32_contig(J_Ginv_j, "J_Ginv_j");
  res = f32_contig(res, "res");
  ii = idx64(ii, "ii");
  jj = idx64(jj, "jj");
  const int64_t r = res.size(0);
  TORCH_CHECK(r > 0 && res.numel() == 7 * r, "res must be [r, 7] with r > 0");
  TORCH_CHECK(J_Ginv_i.numel() == 49 * r && J_Ginv_j.numel() == 49 * r,
              "J_Ginv_i / J_Ginv_j must be [r, 7, 7]");
  TORCH_CHECK(ii.numel() == r && jj.numel() == r, "ii / jj must be [r]");
  // The structure (which poses a long edge touches) is host logic, as in the
  // reference (ba.cpp:141-158 builds the triplets on the host): one copy of
  // the indices to the host, which also does the reference's checks.
  const auto iih = ii.cpu(), jjh = jj.cpu();
  const int64_t* ip = iih.data_ptr<int64_t>();
  const int64_t* jp = jjh.data_ptr<int64_t>();
  int64_t n = 0;
  for (int64_t x = 0; x < r; x++) {
    // the reference calls exit(1) on a self edge (ba.cpp:150-151); raise instead
    TORCH_CHECK(ip[x] != jp[x], "cuda_ba.solve_system: edge with ii == jj");
    TORCH_CHECK(ip[x] >= 0 && jp[x] >= 0, "cuda_ba.solve_system: negative pose index");
    n = std::max(n, std::max(ip[x], jp[x]) + 1);
  }
  int64_t nf = freen;  // solve(A, b, freen*7): < 0 (or past the end) -> whole system
  if (nf < 0 || nf > n) nf = n;
  auto delta = torch::zeros({n, 7}, res.options().dtype(torch::kFloat64));
  if (nf > 0) {
    TORCH_CHECK(nf < (1LL << 30), "cuda_ba.solve_system: too many poses");
    int64_t len = 0;
    check_status(dpvo_pgo_plan(ip, jp, (int)r, (int)nf, nullptr, 0, &len), "cuda_ba.solve_system");
    auto planh = torch::empty({len}, torch::kInt64);
    check_status(dpvo_pgo_plan(ip, jp, (int)r, (int)nf, planh.data_ptr<int64_t>(), len, &len),
                 "cuda_ba.solve_system");
    const int64_t* hdr = planh.data_ptr<int64_t>();
    const int64_t m = hdr[3], ws_n = hdr[25], hS = hdr[22], hBB = hdr[23], hDelta = hdr[24];
    auto plan = planh.to(dev, /*non_blocking=*/false);
    auto ws = torch::empty({ws_n}, res.options().dtype(torch::kFloat64));
    auto fail = torch::zeros({1}, res.options().dtype(torch::kInt32));
    check_status(dpvo_pgo_factor(J_Ginv_i.data_ptr<float>(), J_Ginv_j.data_ptr<float>(),
                                 ii.data_ptr<int64_t>(), res.data_ptr<float>(),
                                 plan.data_ptr<int64_t>(), hdr, (float)ep, (float)lm,
                                 ws.data_ptr<double>(), fail.data_ptr<int>(), current_stream()),
                 "cuda_ba.solve_system");
    torch::Tensor xB, info = torch::zeros({1}, res.options().dtype(torch::kInt32));
    if (m > 0) {  // dense SPD solve of the border system (7 m unknowns)
      auto S = ws.narrow(0, hS, 49 * m * m).view({7 * m, 7 * m});
      auto bB = ws.narrow(0, hBB, 7 * m);
      auto chol = at::linalg_cholesky_ex(S);
      info = std::get<1>(chol).to(torch::kInt32).view({1});
      xB = at::cholesky_solve(bB.unsqueeze(1), std::get<0>(chol)).squeeze(1).contiguous();
    }
    check_status(dpvo_pgo_back(plan.data_ptr<int64_t>(), hdr,
                               m > 0 ? xB.data_ptr<double>() : nullptr, ws.data_ptr<double>(),
                               current_stream()),
                 "cuda_ba.solve_system");
    delta.narrow(0, 0, nf).copy_(ws.narrow(0, hDelta, 7 * nf).view({nf, 7}));
    if (m > 0) {
      auto bidx = planh.narrow(0, hdr[7], 3 * m).view({m, 3}).select(1, 0).contiguous().to(dev);
      delta.index_copy_(0, bidx, xB.view({m, 7}));
    }
    // one device->host sync for both failure reports
    const auto st = torch::cat({fail, info}).cpu();
    const int* sv = st.data_ptr<int>();
    TORCH_CHECK(sv[0] == 0 && sv[1] == 0,
                "cuda_ba.solve_system: the damped pose-graph system is not positive definite "
                "(segment pivot failure ", sv[0], ", border Cholesky info ", sv[1],
                "); check for NaN residuals/Jacobians or unconstrained poses with ep = 0");
  }
  return {delta.to(torch::kFloat32).to(out_dev)};
}

// Split F-BA for the edge-sharded multi-GPU path.
torch::Tensor ba_setup(torch::Tensor ii, torch::Tensor jj, torch::Tensor kk, int num_patches,
                       int t0, int t1) {
  ii = idx64(ii, "ii");
  jj = idx64(jj, "jj");
  kk = idx64(kk, "kk");
  const c10::hip::OptionalHIPGuardMasqueradingAsCUDA guard(ii.device());
  const int E = ii.numel();
  const size_t wsb = dpvo_ba_workspace_bytes(E, t0, t1);
  auto ws = torch::empty({(int64_t)wsb}, ii.options().dtype(torch::kUInt8));
  check_status(dpvo_ba_setup(ii.data_ptr<int64_t>(), jj.data_ptr<int64_t>(),
                             kk.data_ptr<int64_t>(), E, num_patches, t0, t1, ws.data_ptr(), wsb,
                             current_stream()),
               "cuda_ba.setup");
  return ws;
}

std::vector<torch::Tensor> ba_build_schur(torch::Tensor ws, torch::Tensor poses,
                                          torch::Tensor patches, torch::Tensor intrinsics,
                                          torch::Tensor target, torch::Tensor weight,
                                          torch::Tensor lmbda, torch::Tensor ii, torch::Tensor jj,
                                          torch::Tensor kk, int t0, int t1) {
  const c10::hip::OptionalHIPGuardMasqueradingAsCUDA guard(poses.device());
  TORCH_CHECK(poses.is_contiguous() && patches.is_contiguous(), "poses/patches contiguous");
  intrinsics = f32_contig(intrinsics, "intrinsics");
  target = f32_contig(target, "target");
  weight = f32_contig(weight, "weight");
  lmbda = f32_contig(lmbda, "lmbda");
  ii = idx64(ii, "ii");
  jj = idx64(jj, "jj");
  kk = idx64(kk, "kk");
  const int N = t1 - t0, E = ii.numel(), P = patches.size(-1);
  auto S = torch::zeros({N * (N + 1) / 2, 6, 6}, poses.options().dtype(torch::kFloat64));
  auto y = torch::zeros({6 * N}, poses.options().dtype(torch::kFloat64));
  check_status(dpvo_ba_build_schur(poses.data_ptr<float>(), patches.data_ptr<float>(),
                                   intrinsics.data_ptr<float>(), target.data_ptr<float>(),
                                   weight.data_ptr<float>(), lmbda.data_ptr<float>(),
                                   ii.data_ptr<int64_t>(), jj.data_ptr<int64_t>(),
                                   kk.data_ptr<int64_t>(), E, P, poses.numel() / 7, t0, t1,
                                   ws.data_ptr(), S.data_ptr<double>(), y.data_ptr<double>(),
                                   current_stream()),
               "cuda_ba.build_schur");
  return {S, y};
}

torch::Tensor ba_solve_update(torch::Tensor ws, torch::Tensor poses, torch::Tensor patches,
                              torch::Tensor S, torch::Tensor y, int E, int t0, int t1) {
  const c10::hip::OptionalHIPGuardMasqueradingAsCUDA guard(poses.device());
  TORCH_CHECK(poses.is_contiguous() && patches.is_contiguous(), "poses/patches contiguous");
  S = S.contiguous();
  y = y.contiguous();
  TORCH_CHECK(S.scalar_type() == torch::kFloat64 && y.scalar_type() == torch::kFloat64,
              "S / y must be float64");
  const int N = t1 - t0, P = patches.size(-1);
  auto dX = torch::zeros({N > 0 ? N : 0, 6}, poses.options().dtype(torch::kFloat64));
  check_status(dpvo_ba_solve_update(poses.data_ptr<float>(), patches.data_ptr<float>(),
                                    S.data_ptr<double>(), y.data_ptr<double>(), E, P,
                                    poses.numel() / 7, t0, t1, ws.data_ptr(),
                                    N > 0 ? dX.data_ptr<double>() : nullptr, current_stream()),
               "cuda_ba.solve_update");
  return dX;
}

torch::Tensor ba_last_status(torch::Tensor ws, int E, int t0, int t1) {
  auto out = torch::zeros({1}, ws.options().dtype(torch::kInt32));
  check_status(dpvo_ba_last_status(ws.data_ptr(), E, t0, t1, out.data_ptr<int>(),
                                   current_stream()),
               "cuda_ba.last_status");
  return out;
}

// Large-graph F-BA split for the edge-sharded driver (dpvo_amd/fastba/sharded.py):
// setup -> [build -> all_reduce(packed) -> solve_update] x iterations.
torch::Tensor gba_setup(torch::Tensor ii, torch::Tensor jj, torch::Tensor kk, int num_patches,
                        int PPF, int t0, int t1, int own_lo, int own_hi) {
  ii = idx64(ii, "ii");
  jj = idx64(jj, "jj");
  kk = idx64(kk, "kk");
  const c10::hip::OptionalHIPGuardMasqueradingAsCUDA guard(ii.device());
  const int E = ii.numel();
  TORCH_CHECK(E > 0, "gba_setup: empty graph");
  const size_t wsb = dpvo_gba_workspace_bytes(E, t0, t1);
  auto ws = torch::empty({(int64_t)wsb}, ii.options().dtype(torch::kUInt8));
  check_status(dpvo_gba_setup(ii.data_ptr<int64_t>(), jj.data_ptr<int64_t>(),
                              kk.data_ptr<int64_t>(), E, num_patches, PPF, t0, t1, own_lo, own_hi,
                              ws.data_ptr(), wsb, current_stream()),
               "cuda_ba.gba_setup");
  return ws;
}

void gba_build(torch::Tensor ws, torch::Tensor poses, torch::Tensor patches,
               torch::Tensor intrinsics, torch::Tensor target, torch::Tensor weight,
               torch::Tensor lmbda, torch::Tensor ii, torch::Tensor jj, int t0, int t1) {
  const c10::hip::OptionalHIPGuardMasqueradingAsCUDA guard(poses.device());
  TORCH_CHECK(poses.is_contiguous() && patches.is_contiguous(), "poses/patches contiguous");
  poses = f32_contig(poses, "poses");
  patches = f32_contig(patches, "patches");
  intrinsics = f32_contig(intrinsics, "intrinsics");
  target = f32_contig(target, "target");
  weight = f32_contig(weight, "weight");
  lmbda = f32_contig(lmbda, "lmbda");
  ii = idx64(ii, "ii");
  jj = idx64(jj, "jj");
  const int E = ii.numel(), P = patches.size(-1);
  TORCH_CHECK(ws.numel() >= (int64_t)dpvo_gba_workspace_bytes(E, t0, t1), "workspace too small");
  check_status(dpvo_gba_build(poses.data_ptr<float>(), patches.data_ptr<float>(),
                              intrinsics.data_ptr<float>(), target.data_ptr<float>(),
                              weight.data_ptr<float>(), lmbda.data_ptr<float>(),
                              ii.data_ptr<int64_t>(), jj.data_ptr<int64_t>(), E, P,
                              poses.numel() / 7, t0, t1, ws.data_ptr(), current_stream()),
               "cuda_ba.gba_build");
}

// the packed [y (6N) | S blocks (nblk x 36)] fp64 system inside the workspace
torch::Tensor gba_packed(torch::Tensor ws, int E, int t0, int t1, int64_t nblk) {
  const int64_t N = t1 > t0 ? t1 - t0 : 0;
  const int64_t off = (int64_t)dpvo_gba_packed_offset(E, t0, t1);
  const int64_t n = 6 * N + 36 * nblk;
  TORCH_CHECK(off % 8 == 0 && off + 8 * n <= ws.numel(), "gba_packed: bad extent");
  return ws.narrow(0, off, 8 * n).view(torch::kFloat64);
}

void gba_solve_update(torch::Tensor ws, torch::Tensor poses, torch::Tensor patches, int E, int t0,
                      int t1) {
  const c10::hip::OptionalHIPGuardMasqueradingAsCUDA guard(poses.device());
  TORCH_CHECK(poses.is_contiguous() && patches.is_contiguous(), "poses/patches contiguous");
  check_status(dpvo_gba_solve_update(poses.data_ptr<float>(), patches.data_ptr<float>(), E,
                                     patches.size(-1), t0, t1, ws.data_ptr(), current_stream()),
               "cuda_ba.gba_solve_update");
}

torch::Tensor gba_info(torch::Tensor ws, int E, int t0, int t1) {
  auto out = torch::zeros({8}, ws.options().dtype(torch::kInt32));
  check_status(dpvo_gba_info(ws.data_ptr(), E, t0, t1, out.data_ptr<int>(), current_stream()),
               "cuda_ba.gba_info");
  return out;
}

// PatchGraph bookkeeping on the device (dpvo.py:480-568): no host sync.
static float* opt_f32(const torch::Tensor& t) {
  return t.defined() && t.numel() ? t.data_ptr<float>() : nullptr;
}

void pg_append(torch::Tensor ix, torch::Tensor kk_new, torch::Tensor jj_new, torch::Tensor ii,
               torch::Tensor jj, torch::Tensor kk, torch::Tensor net, torch::Tensor counts) {
  ix = idx64(ix, "ix");
  kk_new = idx64(kk_new, "kk");
  jj_new = idx64(jj_new, "jj");
  TORCH_CHECK(ii.is_contiguous() && jj.is_contiguous() && kk.is_contiguous() &&
              counts.is_contiguous() && counts.scalar_type() == torch::kInt32,
              "pg buffers must be contiguous, counts int32");
  const c10::hip::OptionalHIPGuardMasqueradingAsCUDA guard(ii.device());
  const int max_edges = ii.numel();
  const int DIM = net.defined() && net.numel() ? (int)(net.numel() / max_edges) : 0;
  check_status(dpvo_pg_append(ix.data_ptr<int64_t>(), kk_new.data_ptr<int64_t>(),
                              jj_new.data_ptr<int64_t>(), kk_new.numel(), ii.data_ptr<int64_t>(),
                              jj.data_ptr<int64_t>(), kk.data_ptr<int64_t>(), opt_f32(net), DIM,
                              counts.data_ptr<int>(), max_edges, current_stream()),
               "cuda_ba.pg_append");
}

void pg_remove(c10::optional<torch::Tensor> mask, c10::optional<torch::Tensor> ix, int64_t thresh,
               int64_t lc_min, bool store, std::vector<torch::Tensor> act,
               std::vector<torch::Tensor> back, std::vector<torch::Tensor> inac,
               torch::Tensor counts, torch::Tensor pos) {
  TORCH_CHECK(act.size() == 6 && back.size() == 6 && inac.size() == 5,
              "act/back: [ii, jj, kk, net, weight, target]; inac: [ii, jj, kk, weight, target]");
  const c10::hip::OptionalHIPGuardMasqueradingAsCUDA guard(counts.device());
  const int max_edges = act[0].numel();
  const int DIM = act[3].defined() && act[3].numel() ? (int)(act[3].numel() / max_edges) : 0;
  const uint8_t* mp = nullptr;
  torch::Tensor m8;
  if (mask && mask->defined()) {
    m8 = mask->to(torch::kUInt8).contiguous();
    check_device(m8, "mask");
    mp = m8.data_ptr<uint8_t>();
  }
  const int64_t* ixp = (ix && ix->defined()) ? idx64(*ix, "ix").data_ptr<int64_t>() : nullptr;
  auto L = [](const torch::Tensor& t) { return t.data_ptr<int64_t>(); };
  check_status(dpvo_pg_remove(mp, ixp, thresh, lc_min, store ? 1 : 0, L(act[0]), L(act[1]),
                              L(act[2]), opt_f32(act[3]), act[4].data_ptr<float>(),
                              act[5].data_ptr<float>(), L(back[0]), L(back[1]), L(back[2]),
                              opt_f32(back[3]), back[4].data_ptr<float>(), back[5].data_ptr<float>(),
                              L(inac[0]), L(inac[1]), L(inac[2]), inac[3].data_ptr<float>(),
                              inac[4].data_ptr<float>(), DIM, counts.data_ptr<int>(),
                              pos.data_ptr<int>(), max_edges, current_stream()),
               "cuda_ba.pg_remove");
}

void pg_remove_window_dev(torch::Tensor ix, torch::Tensor n_dev, int64_t thresh_off,
                         int64_t lc_off, bool lc_on, bool store, std::vector<torch::Tensor> act,
                         std::vector<torch::Tensor> back, std::vector<torch::Tensor> inac,
                         torch::Tensor counts, torch::Tensor pos) {
  TORCH_CHECK(act.size() == 6 && back.size() == 6 && inac.size() == 5,
              "act/back: [ii, jj, kk, net, weight, target]; inac: [ii, jj, kk, weight, target]");
  const c10::hip::OptionalHIPGuardMasqueradingAsCUDA guard(counts.device());
  const int max_edges = act[0].numel();
  const int DIM = act[3].defined() && act[3].numel() ? (int)(act[3].numel() / max_edges) : 0;
  ix = idx64(ix, "ix");
  auto L = [](const torch::Tensor& t) { return t.data_ptr<int64_t>(); };
  check_status(dpvo_pg_remove_window_dev(
                   ix.data_ptr<int64_t>(), dev_scalar(n_dev, "n_dev"), thresh_off, lc_off,
                   lc_on ? 1 : 0, store ? 1 : 0, L(act[0]), L(act[1]), L(act[2]), opt_f32(act[3]),
                   act[4].data_ptr<float>(), act[5].data_ptr<float>(), L(back[0]), L(back[1]),
                   L(back[2]), opt_f32(back[3]), back[4].data_ptr<float>(),
                   back[5].data_ptr<float>(), L(inac[0]), L(inac[1]), L(inac[2]),
                   inac[3].data_ptr<float>(), inac[4].data_ptr<float>(), DIM,
                   counts.data_ptr<int>(), pos.data_ptr<int>(), max_edges, current_stream()),
               "cuda_ba.pg_remove_window_dev");
}

void pg_append_dev(torch::Tensor ix, torch::Tensor kk_new, torch::Tensor jj_new,
                   torch::Tensor n_dev, torch::Tensor ii, torch::Tensor jj, torch::Tensor kk,
                   torch::Tensor net, torch::Tensor counts) {
  ix = idx64(ix, "ix");
  kk_new = idx64(kk_new, "kk");
  jj_new = idx64(jj_new, "jj");
  TORCH_CHECK(kk_new.numel() == jj_new.numel(), "kk / jj sizes differ");
  TORCH_CHECK(ii.is_contiguous() && jj.is_contiguous() && kk.is_contiguous() &&
              counts.is_contiguous() && counts.scalar_type() == torch::kInt32,
              "pg buffers must be contiguous, counts int32");
  const c10::hip::OptionalHIPGuardMasqueradingAsCUDA guard(ii.device());
  const int max_edges = ii.numel();
  const int DIM = net.defined() && net.numel() ? (int)(net.numel() / max_edges) : 0;
  check_status(dpvo_pg_append_dev(ix.data_ptr<int64_t>(), kk_new.data_ptr<int64_t>(),
                                  jj_new.data_ptr<int64_t>(), dev_scalar(n_dev, "n_dev"),
                                  (int)kk_new.numel(), ii.data_ptr<int64_t>(),
                                  jj.data_ptr<int64_t>(), kk.data_ptr<int64_t>(), opt_f32(net),
                                  DIM, counts.data_ptr<int>(), max_edges, current_stream()),
               "cuda_ba.pg_append_dev");
}

void pg_remove_frame_dev(torch::Tensor kf, std::vector<torch::Tensor> act,
                         std::vector<torch::Tensor> back, torch::Tensor counts, torch::Tensor pos) {
  TORCH_CHECK(act.size() == 6 && back.size() == 6, "act/back: [ii, jj, kk, net, weight, target]");
  const c10::hip::OptionalHIPGuardMasqueradingAsCUDA guard(counts.device());
  const int max_edges = act[0].numel();
  const int DIM = act[3].defined() && act[3].numel() ? (int)(act[3].numel() / max_edges) : 0;
  auto L = [](const torch::Tensor& t) { return t.data_ptr<int64_t>(); };
  check_status(dpvo_pg_remove_frame_dev(
                   dev_scalar(kf, "kf"), L(act[0]), L(act[1]), L(act[2]), opt_f32(act[3]),
                   act[4].data_ptr<float>(), act[5].data_ptr<float>(), L(back[0]), L(back[1]),
                   L(back[2]), opt_f32(back[3]), back[4].data_ptr<float>(),
                   back[5].data_ptr<float>(), DIM, counts.data_ptr<int>(), pos.data_ptr<int>(),
                   max_edges, current_stream()),
               "cuda_ba.pg_remove_frame_dev");
}

// DPVO.keyframe decision (dpvo.py:586-624): kf = {drop, k}, mag = both motionmags
void kf_motion(torch::Tensor ii, torch::Tensor jj, torch::Tensor kk, torch::Tensor counts,
               torch::Tensor poses, torch::Tensor patches, torch::Tensor intrinsics,
               torch::Tensor st, int64_t keyframe_index, double keyframe_thresh, torch::Tensor kf,
               torch::Tensor mag) {
  const c10::hip::OptionalHIPGuardMasqueradingAsCUDA guard(poses.device());
  TORCH_CHECK(poses.scalar_type() == torch::kFloat32 && patches.scalar_type() == torch::kFloat32 &&
                  intrinsics.scalar_type() == torch::kFloat32 && poses.is_contiguous() &&
                  patches.is_contiguous() && intrinsics.is_contiguous(),
              "poses / patches / intrinsics: contiguous float32");
  TORCH_CHECK(mag.scalar_type() == torch::kFloat32 && mag.numel() >= 2 && kf.numel() >= 2,
              "kf int32[2], mag float32[2]");
  auto L = [](const torch::Tensor& t) { return t.data_ptr<int64_t>(); };
  check_status(dpvo_kf_motion(L(idx64(ii, "ii")), L(idx64(jj, "jj")), L(idx64(kk, "kk")),
                              dev_scalar(counts, "counts"), poses.data_ptr<float>(),
                              patches.data_ptr<float>(), intrinsics.data_ptr<float>(),
                              (int)patches.size(-1), dev_scalar(st, "st"), (int)keyframe_index,
                              keyframe_thresh, const_cast<int32_t*>(dev_scalar(kf, "kf")),
                              mag.data_ptr<float>(), current_stream()),
               "cuda_ba.kf_motion");
}

// the rest of the frame drop (dpvo.py:626-673); frames: per-frame arrays whose
// leading dim is the frame (ring 0) or a ring slot (ring > 0)
void kf_shift(torch::Tensor kf, int64_t M, torch::Tensor st, torch::Tensor ii, torch::Tensor jj,
              torch::Tensor kk, torch::Tensor counts, std::vector<torch::Tensor> frames,
              std::vector<int64_t> rings, c10::optional<torch::Tensor> poses,
              c10::optional<torch::Tensor> tstamps, c10::optional<torch::Tensor> delta_log,
              c10::optional<torch::Tensor> delta_tstamps, c10::optional<torch::Tensor> delta_count) {
  TORCH_CHECK(frames.size() == rings.size(), "one ring size per frame array");
  const c10::hip::OptionalHIPGuardMasqueradingAsCUDA guard(counts.device());
  std::vector<void*> ptrs;
  std::vector<int64_t> bytes;
  std::vector<int32_t> ring;
  for (size_t a = 0; a < frames.size(); a++) {
    check_device(frames[a], "frame array");
    TORCH_CHECK(frames[a].is_contiguous() && frames[a].dim() >= 1, "frame arrays contiguous");
    ptrs.push_back(frames[a].data_ptr());
    bytes.push_back(frames[a].numel() / frames[a].size(0) * frames[a].element_size());
    ring.push_back((int32_t)rings[a]);
  }
  auto L = [](const torch::Tensor& t) { return t.data_ptr<int64_t>(); };
  const bool log = delta_log && delta_log->defined();
  float* dl = nullptr;
  int64_t* dt = nullptr;
  int32_t* dc = nullptr;
  const float* pp = nullptr;
  const int64_t* ts = nullptr;
  int cap = 0;
  if (log) {
    TORCH_CHECK(poses && tstamps && delta_tstamps && delta_count, "delta log needs all buffers");
    // the kernel ORs its delta-log overflow bit into counts[2] (keyframe.hip
    // kf_delta_kernel): counts must hold the error word too
    TORCH_CHECK(counts.numel() >= 3, "kf_shift with a delta log: counts needs >= 3 int32 words "
                                     "(n, m, errors)");
    dl = delta_log->data_ptr<float>();
    dt = delta_tstamps->data_ptr<int64_t>();
    dc = const_cast<int32_t*>(dev_scalar(*delta_count, "delta_count"));
    pp = poses->data_ptr<float>();
    ts = tstamps->data_ptr<int64_t>();
    cap = (int)(delta_log->numel() / 7);
  }
  check_status(dpvo_kf_shift(dev_scalar(kf, "kf"), (int)M, const_cast<int32_t*>(dev_scalar(st, "st")),
                             L(ii), L(jj), L(kk), const_cast<int32_t*>(dev_scalar(counts, "counts")),
                             (int)ii.numel(),
                             ptrs.data(), bytes.data(), ring.data(), (int)ptrs.size(), pp, ts, dl,
                             dt, dc, cap, current_stream()),
               "cuda_ba.kf_shift");
}

// CholeskySolver's device solve (dpvo/ba.py:13-38 -> torch.linalg.cholesky_ex +
// cholesky_solve): batched over the leading dims, fp32 / fp64
static void spd_shapes(const torch::Tensor& H, const torch::Tensor& B, int64_t& batch, int& n,
                       int& k) {
  check_device(H, "H");
  check_device(B, "B");
  TORCH_CHECK(H.dim() >= 2 && H.size(-1) == H.size(-2), "H must be [..., n, n]");
  TORCH_CHECK(B.dim() == H.dim() && B.size(-2) == H.size(-1), "B must be [..., n, k]");
  TORCH_CHECK(H.scalar_type() == B.scalar_type() &&
                  (H.scalar_type() == torch::kFloat32 || H.scalar_type() == torch::kFloat64),
              "H / B: float32 or float64, one dtype");
  for (int64_t d = 0; d + 2 < H.dim(); d++)
    TORCH_CHECK(H.size(d) == B.size(d), "H / B batch dims differ");
  n = (int)H.size(-1);
  k = (int)B.size(-1);
  batch = n ? H.numel() / ((int64_t)n * n) : 0;
}

std::vector<torch::Tensor> spd_solve(torch::Tensor H, torch::Tensor B) {
  int64_t batch;
  int n, k;
  spd_shapes(H, B, batch, n, k);
  const c10::hip::OptionalHIPGuardMasqueradingAsCUDA guard(H.device());
  H = H.contiguous();
  B = B.contiguous();
  auto L = torch::empty_like(H);
  auto X = torch::empty_like(B);
  std::vector<int64_t> bs(H.sizes().begin(), H.sizes().end() - 2);
  auto info = torch::zeros(bs, H.options().dtype(torch::kInt32));
  check_status(dpvo_spd_solve(H.data_ptr(), B.data_ptr(), L.data_ptr(), X.data_ptr(),
                              info.data_ptr<int32_t>(), (int)batch, n, k, 1, dtype_code(H),
                              current_stream()),
               "cuda_ba.spd_solve");
  return {X, L, info};
}

torch::Tensor spd_solve_factored(torch::Tensor L, torch::Tensor B) {
  int64_t batch;
  int n, k;
  spd_shapes(L, B, batch, n, k);
  const c10::hip::OptionalHIPGuardMasqueradingAsCUDA guard(L.device());
  L = L.contiguous();
  B = B.contiguous();
  auto X = torch::empty_like(B);
  check_status(dpvo_spd_solve(L.data_ptr(), B.data_ptr(), nullptr, X.data_ptr(), nullptr,
                              (int)batch, n, k, 0, dtype_code(L), current_stream()),
               "cuda_ba.spd_solve_factored");
  return X;
}

// PatchGraph.edges_loop (patchgraph.py:65-91) gated as dpvo.py:984-988
void edges_loop(torch::Tensor poses, torch::Tensor patches, torch::Tensor intrinsics,
                torch::Tensor ix, int64_t M, torch::Tensor st, int64_t n_cap,
                c10::optional<torch::Tensor> last_global_ba, int64_t removal_window,
                int64_t max_edge_age, int64_t global_opt_freq, int64_t keyframe_index,
                double backend_thresh, int64_t max_num_edges, int64_t nms, torch::Tensor work,
                torch::Tensor out_kk, torch::Tensor out_jj, torch::Tensor out_n,
                c10::optional<torch::Tensor> errors) {
  const c10::hip::OptionalHIPGuardMasqueradingAsCUDA guard(poses.device());
  int32_t* err = (errors && errors->defined())
                     ? const_cast<int32_t*>(dev_scalar(*errors, "errors"))
                     : nullptr;
  TORCH_CHECK(work.scalar_type() == torch::kFloat32 &&
                  work.numel() >= (int64_t)dpvo_edges_loop_work_floats(),
              "work: float32[edges_loop_work_floats()]");
  TORCH_CHECK(M > 0 && patches.numel() % (M * 3 * patches.size(-1) * patches.size(-1)) == 0,
              "patches: [N * M, 3, P, P]");
  TORCH_CHECK(out_kk.numel() >= max_num_edges * M && out_jj.numel() >= max_num_edges * M,
              "out_kk / out_jj: max_num_edges x M");
  int32_t* lb = (last_global_ba && last_global_ba->defined())
                    ? const_cast<int32_t*>(dev_scalar(*last_global_ba, "last_global_ba"))
                    : nullptr;
  check_status(dpvo_edges_loop(poses.data_ptr<float>(), patches.data_ptr<float>(),
                               intrinsics.data_ptr<float>(), idx64(ix, "ix").data_ptr<int64_t>(),
                               (int)patches.size(-1), (int)M, dev_scalar(st, "st"), (int)n_cap, lb,
                               (int)removal_window, (int)max_edge_age, (int)global_opt_freq,
                               (int)keyframe_index, (float)backend_thresh, (int)max_num_edges,
                               (int)nms, work.data_ptr<float>(), out_kk.data_ptr<int64_t>(),
                               out_jj.data_ptr<int64_t>(),
                               const_cast<int32_t*>(dev_scalar(out_n, "out_n")), err,
                               current_stream()),
               "cuda_ba.edges_loop");
}

PYBIND11_MODULE(TORCH_EXTENSION_NAME, m) {
  m.def("forward", &ba_forward, "BA forward operator");
  m.def("neighbors", &ba_neighbors, "temporal neighboor indicies");
  m.def("reproject", &ba_reproject, "temporal neighboor indicies");
  m.def("solve_system", &ba_solve_system, "Sim3 pose-graph solve (ba.cpp:120-180)");
  // additions: split BA for the sharded multi-GPU path
  m.def("setup", &ba_setup, "BA graph setup -> workspace");
  m.def("build_schur", &ba_build_schur, "linearize + Schur complement (S_lower, y)");
  m.def("solve_update", &ba_solve_update, "Cholesky solve + pose/patch retraction");
  m.def("last_status", &ba_last_status, "status word of the last BA on a workspace");
  m.def("max_free_poses", &dpvo_ba_max_free_poses);
  m.def("pg_append", &pg_append, "PatchGraph.append_factors on the device (dpvo.py:480-521)");
  m.def("pg_remove", &pg_remove, "PatchGraph.remove_factors on the device (dpvo.py:523-568)");
  m.def("plan_supported", &ba_plan_supported, "window path available for (E, t0, t1, P)");
  m.def("plan", &ba_plan, "group the edges by patch (reads ii/jj/kk only) -> workspace");
  m.def("plan_offsets", &ba_plan_offsets,
        "byte offsets of epos, poff, pmask, pkk, meta inside a plan workspace");
  m.def("forward_planned", &ba_forward_planned, "BA iterations on a planned workspace");
  m.def("check_status", &ba_check_status,
        "sync on the BA status of every forward so far on the device of `like`; raises "
        "RuntimeError on fatal bits (2 bad kk, 4/8 large-graph limits, 16 timeout); returns "
        "the OR of all bits (1 = a Cholesky failure gave a zero step) and resets it");
  m.def("gba_setup", &gba_setup, "large-graph BA setup (ownership own_lo <= kk/PPF < own_hi)");
  m.def("gba_build", &gba_build, "large-graph BA: linearise owned patches -> packed (y, S)");
  m.def("gba_packed", &gba_packed, "view of the packed fp64 [y | S blocks] system");
  m.def("gba_solve_update", &gba_solve_update, "large-graph BA: solve + retraction");
  m.def("gba_info", &gba_info, "status, nuniq, nitems, nblk, nI, nB, g, nsb (device int32[8])");
  m.def("forward_marks", &ba_forward_marks, "forward + per-phase wall-clock marks");
  m.def("set_marks", [](bool on) { check_status(dpvo_ba_set_marks(on ? 1 : 0), "set_marks"); },
        "stamp wall-clock marks into the BA workspace (instrumentation)");
  m.def("workspace_marks", &ba_workspace_marks,
        "the 2432 marks of a workspace ([1664 + 2b] / [1665 + 2b]: fused launch workgroup b)");
  m.def("forward_dx", &ba_forward_dx, "forward; returns the last iteration's dX [N, 6] (fp64)");
  m.def("last_dx", &ba_last_dx, "dX [N, 6] of the last iteration of a planned forward on ws");
  m.def("reproject_ordered_plan", &ba_reproject_ordered_plan,
        "reproject + A-CORR edge order + BA plan (workspace for forward_planned), one launch");
  m.def("reproject_ordered_plan_dev", &ba_reproject_ordered_plan_dev,
        "reproject_ordered_plan with the window start t0 read from an int32 device scalar");
  m.def("forward_planned_dev", &ba_forward_planned_dev,
        "forward_planned with t0 read from an int32 device scalar (graph replay)");
  m.def("pg_remove_window_dev", &pg_remove_window_dev,
        "DPVO.keyframe window removal with thresholds relative to a device frame count");
  m.def("pg_append_dev", &pg_append_dev, "append_factors with a device edge count");
  m.def("pg_remove_frame_dev", &pg_remove_frame_dev,
        "DPVO.keyframe frame-drop removal predicated on the device decision kf");
  m.def("kf_motion", &kf_motion, "DPVO.keyframe motion magnitude + decision (dpvo.py:586-624)");
  m.def("kf_shift", &kf_shift, "DPVO.keyframe frame drop: delta log, edge / frame shift, counters",
        py::arg("kf"), py::arg("M"), py::arg("st"), py::arg("ii"), py::arg("jj"), py::arg("kk"),
        py::arg("counts"), py::arg("frames"), py::arg("rings"), py::arg("poses") = py::none(),
        py::arg("tstamps") = py::none(), py::arg("delta_log") = py::none(),
        py::arg("delta_tstamps") = py::none(), py::arg("delta_count") = py::none());
  m.def("edges_loop", &edges_loop, "PatchGraph.edges_loop (patchgraph.py:65-91), device count");
  m.def("edges_loop_work_floats", []() { return (int64_t)dpvo_edges_loop_work_floats(); });
  m.def("reproject_ordered_plan_insert", &ba_reproject_ordered_plan_insert,
        "reproject + edge order + BA plan + the new frame's pyramid insertion, one launch");
  m.def("reproject_ordered", &ba_reproject_ordered,
        "reproject + edge order by target frame (for cuda_corr.forward_levels(order=))");
  m.def("select_path", [](int mode) { check_status(dpvo_ba_select_path(mode), "select_path"); },
        "F-BA implementation: 0 auto, 2 multi-kernel, 4 large-graph, 5 window");
  m.def("spd_solve", &spd_solve,
        "batched SPD factor + solve (CholeskySolver, dpvo/ba.py:13-38): H [..., n, n] (lower "
        "triangle read), B [..., n, k] -> [X, L (lower factor), info (first failed column, 0 = ok)]");
  m.def("spd_solve_factored", &spd_solve_factored,
        "X = (L L^T)^-1 B for a lower factor L from spd_solve (the backward's cholesky_solve)");
  m.attr("native_library") = dpvo_version();
}
