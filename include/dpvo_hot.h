/*
 * dpvo_hot.h -- C ABI of the MI355X (gfx950) DPVO hot path.
 *
 * Every entry point takes plain device pointers, sizes and an opaque HIP
 * stream (`void*`, hipStream_t; NULL = legacy default stream), launches
 * hand-written HIP kernels on that stream and returns a dpvo_status.  No
 * entry point allocates device memory, synchronises or copies to the host,
 * so each call is hipGraph-capturable; scratch memory is passed in as a
 * caller-owned workspace sized by the matching *_workspace_bytes().
 *
 * Each function names the reference interface it replaces (paths relative to
 * /root/reference, cuteboyqq/DPVO).  The Python extension modules cuda_corr,
 * cuda_ba and lietorch_backends (dpvo_amd/csrc/ext_*.cpp) bind exactly these.
 *
 * Layouts (row-major, contiguous):
 *   fmap1   [B, N1, C, H, W]    gmap patch features (H = W = p)
 *   fmap2   [B, N2, C, H2, W2]  one pyramid level of frame features
 *   coords  [B, M, 2, H, W]     float32 (x, y) per patch pixel, this level
 *   ii, jj  [M]                 int64 patch / frame index per edge
 *   corr    [B, M, 2R+1, 2R+1, H, W]  axis 2 = x offset, axis 3 = y offset
 *   poses   [*, 7]  float32 (tx, ty, tz, qx, qy, qz, qw)
 *   patches [*, 3, P, P] float32 (x, y, inverse depth)
 */
#ifndef DPVO_HOT_H
#define DPVO_HOT_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef enum {
  DPVO_OK = 0,
  DPVO_ERR_INVALID = 1,     /* bad argument (shape, dtype, null pointer)      */
  DPVO_ERR_LAUNCH = 2,      /* hipLaunchKernel / hipGetLastError failure       */
  DPVO_ERR_UNSUPPORTED = 3, /* configuration outside what this build handles   */
  DPVO_ERR_WORKSPACE = 4    /* workspace smaller than *_workspace_bytes()      */
} dpvo_status;

typedef enum { DPVO_F32 = 0, DPVO_F16 = 1, DPVO_F64 = 2 } dpvo_dtype;

/* Human-readable text for a status code (static storage). */
const char* dpvo_status_string(int status);
/* Build identification, e.g. "dpvo_hot gfx950 <git>". */
const char* dpvo_version(void);

/* ---------------------------------------------------------------- altcorr */

/* A-CORR.  Replaces cuda_corr.forward (dpvo/altcorr/correlation.cpp:57,
   correlation_kernel.cu:232-272 + corr_forward_kernel :82-175).
   out[B,M,2R+1,2R+1,H,W] in fmap dtype; accumulation is always fp32 (f64 for
   DPVO_F64).  Requires H*W <= 16, R <= 7. */
int dpvo_corr_forward(const void* fmap1, const void* fmap2, const float* coords,
                      const int64_t* ii, const int64_t* jj, int B, int M, int C, int H, int W,
                      int N1, int N2, int H2, int W2, int radius, int dtype, void* out,
                      void* stream);

/* A-CORR, all pyramid levels of one DPVO update in one launch (the fused form
   of the two/four per-level calls at dpvo/dpvo.py:462-465).  fmap2[l] is
   [B, N2, C, H2[l], W2[l]]; coords are level-1 coordinates and are divided by
   scale[l] in-kernel (dpvo.py:462-463 passes coords / 1 and coords / 4).
   out is [B, M, 2R+1, 2R+1, H, W, L] float = DPVO's torch.stack(..., -1). */
int dpvo_corr_forward_levels(const void* fmap1, const void* const* fmap2, const int* H2,
                             const int* W2, const float* scale, int L, const float* coords,
                             const int64_t* ii, const int64_t* jj, int B, int M, int C, int H,
                             int W, int N1, int N2, int radius, int dtype, float* out,
                             void* stream);

/* A-CORR, all levels, channels-last pyramid (no reference counterpart: the
   layout is this build's; semantics identical to dpvo_corr_forward_levels).
   fmap2[l] is [B,N2,H2[l],W2[l],C] (a [B,N2,C,H,W] tensor in channels-last
   memory), fp32, C == 128, L <= 4, H*W <= 16, (2R+1)^2*H*W <= 512.
   Returns DPVO_ERR_UNSUPPORTED outside that envelope (callers fall back to
   dpvo_corr_forward_levels on NCHW data). */
int dpvo_corr_forward_levels_nhwc(const void* fmap1, const void* const* fmap2, const int* H2,
                                  const int* W2, const float* scale, int L, const float* coords,
                                  const int64_t* ii, const int64_t* jj, int B, int M, int C,
                                  int H, int W, int N1, int N2, int radius, int dtype, float* out,
                                  void* stream);
/* The same with an edge order (B == 1): order[p] = edge processed at position
   p, as written by dpvo_reproject_ordered (edges grouped by target frame).
   Workgroups are mapped to XCDs so that each XCD processes one contiguous
   eighth of that order: a target frame's pyramid levels stay in one XCD's L2.
   Results are identical to the unordered call (order == NULL). */
int dpvo_corr_forward_levels_nhwc_ordered(const void* fmap1, const void* const* fmap2,
                                          const int* H2, const int* W2, const float* scale, int L,
                                          const float* coords, const int64_t* ii,
                                          const int64_t* jj, const int32_t* order, int B, int M,
                                          int C, int H, int W, int N1, int N2, int radius,
                                          int dtype, float* out, void* stream);
/* Feature maps [count,C,H,W] -> channels-last [count,H,W,C] (the per-frame
   cost of keeping a channels-last pyramid; dtype F32 or F16). */
int dpvo_feature_to_nhwc(const void* src, void* dst, int count, int C, int H, int W, int dtype,
                         void* stream);

/* Frame insertion of a channels-last pyramid (the ring-buffer writes of
   dpvo.py __call__: fmap -> level 1, avg_pool2d(fmap, s, s) -> level s,
   net.py:411 / dpvo.py:462-463) in one launch.  src: one NCHW level-1 frame
   [C, H, W] fp32; dst[l]: the channels-last slot [H/s, W/s, C] of level l,
   scale[l] in {1, 2, 4, 8}.  Pooling sums row-major in fp32 and divides by
   s^2 (torch avg_pool2d order: bit-identical). */
int dpvo_feature_pyramid_insert(const void* src, void* const* dst, const int* scale, int L, int C,
                                int H, int W, int dtype, void* stream);
/* Ring variant of dpvo_feature_pyramid_insert for graph-replayed frames: dst0[l]
   is slot 0 of level l's ring, slots slot_bytes[l] apart; the slot written is
   *slot_dev % mem, read on the device (replaces the host slot of dpvo.py's
   fmap1_/fmap2_ ring writes). */
int dpvo_feature_pyramid_insert_ring(const void* src, void* const* dst0, const int64_t* slot_bytes,
                                     const int* scale, int L, int C, int H, int W, int mem,
                                     const int32_t* slot_dev, int dtype, void* stream);

/* A-CORR-BWD.  Replaces cuda_corr.backward (correlation.cpp:58,
   correlation_kernel.cu:275-325 + corr_backward_kernel :178-229).
   grad [B,M,2R+1,2R+1,H,W] float32.  fmap1_grad / fmap2_grad are ZEROED by
   this call and then accumulated (fp32 atomics, like the reference). */
int dpvo_corr_backward(const void* fmap1, const void* fmap2, const float* coords,
                       const int64_t* ii, const int64_t* jj, const float* grad, int B, int M,
                       int C, int H, int W, int N1, int N2, int H2, int W2, int radius, int dtype,
                       void* fmap1_grad, void* fmap2_grad, void* stream);

/* A-PATCH.  Replaces cuda_corr.patchify_forward (correlation.cpp:60,
   correlation_kernel.cu:327-346 + patchify_forward_kernel :16-47).
   net [B,C,H,W], coords [B,M,2] float32 -> out [B,M,C,D,D], D = 2R+2.
   clamp=0: zero fill outside the map (CUDA semantics); clamp=1: clamp to the
   border (the fork's runtime patchify_forward_kernel_python,
   correlation_kernel.py:181-224). */
int dpvo_patchify_forward(const void* net, const float* coords, int B, int C, int H, int W, int M,
                          int radius, int clamp, int dtype, void* out, void* stream);

/* A-PATCH-BWD.  Replaces cuda_corr.patchify_backward (correlation.cpp:61,
   correlation_kernel.cu:349-372 + patchify_backward_kernel :49-80).
   net_grad [B,C,H,W] is zeroed by this call, then scatter-added. */
int dpvo_patchify_backward(const void* grad, const float* coords, int B, int C, int H, int W,
                           int M, int radius, int clamp, int dtype, void* net_grad, void* stream);

/* ---------------------------------------------------------------- fastba */

/* Workspace for dpvo_ba_forward / the split BA entry points. */
size_t dpvo_ba_workspace_bytes(int E, int t0, int t1);

/* Instrumentation / testing: which F-BA implementation dpvo_ba_forward uses.
   0 = auto: the window kernel (ba_window.hip: plan kernel + one persistent
   workgroup per share of a lower 6x6 block of S, dense solve in every
   workgroup) for E <= 10240 edges and N <= 16 free poses, the multi-kernel
   path (ba.hip) for E <= 16384 and N <= 20, the large-graph path
   (ba_large.hip) beyond; 2 = the multi-kernel path; 4 = always the
   large-graph path; 5 = same as 0.  1 and 3 (the round-1 single-workgroup
   and per-block kernels) were removed: DPVO_ERR_INVALID.  Process-wide; call
   before sizing the workspace. */
int dpvo_ba_select_path(int mode);

/* Sim3 pose-graph normal equations.  Replaces the host assembly of
   cuda_ba.solve_system (dpvo/fastba/ba.cpp:120-165): J_Ginv_i / J_Ginv_j
   [r, 7, 7] f32, ii / jj [r] int64 (ii != jj, < n), res [r, 7] f32 ->
   dense A [7n, 7n] = J^T J with diag(A) += diag(A)*lm + ep, and
   b [7n] = -J^T res, both fp64 (device memory, zeroed here).  The Cholesky
   solve of the top-left freen*7 block runs in the caller (ba.cpp:103-118). */
int dpvo_pgo_assemble(const float* J_Ginv_i, const float* J_Ginv_j, const int64_t* ii,
                      const int64_t* jj, const float* res, int r, int n, float ep, float lm,
                      double* A, double* b, void* stream);

/* Structured sparse solve of the same system (the default path of
   cuda_ba.solve_system, replacing Eigen SimplicialCholesky, ba.cpp:99-180).
   Poses touched by a long edge (|i - j| > 1) form a dense "border"; the other
   free poses form chain segments that are block-tridiagonal.
   dpvo_pgo_plan (HOST arrays ii / jj [r]; nf = number of free poses, i.e.
   the reference's freen, or n): call with plan == NULL to get the length in
   int64 words, then again to fill it.  The plan's first 32 words are its
   header (counts, table offsets, workspace offsets in doubles; word 25 = the
   workspace length, 3 = m border poses, 22 / 23 = offsets of the dense border
   matrix [7m, 7m] and its right-hand side, 24 = the [nf, 7] step; the border
   table at word 7 holds (pose, left segment, right segment) triples).
   dpvo_pgo_factor (device plan, host copy of the header `hdr`): zeroes the
   workspace, assembles every 7x7 block (edges summed in ascending order:
   deterministic), factors the segments and folds their Schur terms into the
   border system; *fail (device int) = 1 if a segment pivot is not positive.
   The caller solves the border system (dense SPD) into xB [m, 7];
   dpvo_pgo_back back-substitutes the segments. */
int dpvo_pgo_plan(const int64_t* ii, const int64_t* jj, int r, int nf, int64_t* plan,
                  int64_t plan_cap, int64_t* plan_len);
int dpvo_pgo_factor(const float* J_Ginv_i, const float* J_Ginv_j, const int64_t* ii,
                    const float* res, const int64_t* plan, const int64_t* hdr, float ep, float lm,
                    double* ws, int* fail, void* stream);
int dpvo_pgo_back(const int64_t* plan, const int64_t* hdr, const double* xB, double* ws,
                  void* stream);

/* Largest number of free poses (t1 - t0) dpvo_ba_forward handles. */
int dpvo_ba_max_free_poses(void);

/* F-BA.  Replaces cuda_ba.forward (dpvo/fastba/ba.cpp:32-45 -> cuda_ba,
   ba_cuda.cu:433-582; fastba.BA, dpvo/fastba/ba.py:7-8).  Runs `iterations`
   Gauss-Newton/Schur steps and updates poses[t0:t1] and the inverse depth of
   every patch kk[*] IN PLACE.  lmbda is a device pointer to one float.
   eff_impl / PPF select the reference's block-sparse E (block_e.cu); this
   implementation is block-sparse for every call and accepts both values.
   Reductions and the Cholesky solve are fp64, deterministic (no float
   atomics).  A failed factorisation yields dX = 0 and status flag bit 1 in
   ws-reported diagnostics (dpvo_ba_last_status). */
int dpvo_ba_forward(float* poses, float* patches, const float* intrinsics, const float* target,
                    const float* weight, const float* lmbda, const int64_t* ii, const int64_t* jj,
                    const int64_t* kk, int E, int P, int num_poses, int num_patches, int PPF,
                    int t0, int t1, int iterations, int eff_impl, void* workspace,
                    size_t workspace_bytes, void* stream);

/* Split form of dpvo_ba_forward used by the edge-sharded multi-GPU BA
   (SURVEY 8e): setup once per call, then per iteration build the local Schur
   system, all-reduce (S, y) across ranks, and solve+update.
   S_lower: [N(N+1)/2][6][6] double (block (a,b), a >= b, row-major blocks in
   order a*(a+1)/2 + b); y: [6N] double. */
int dpvo_ba_setup(const int64_t* ii, const int64_t* jj, const int64_t* kk, int E, int num_patches,
                  int t0, int t1, void* workspace, size_t workspace_bytes, void* stream);
int dpvo_ba_build_schur(const float* poses, const float* patches, const float* intrinsics,
                        const float* target, const float* weight, const float* lmbda,
                        const int64_t* ii, const int64_t* jj, const int64_t* kk, int E, int P,
                        int num_poses, int t0, int t1, void* workspace, double* S_lower,
                        double* y, void* stream);
int dpvo_ba_solve_update(float* poses, float* patches, const double* S_lower, const double* y,
                         int E, int P, int num_poses, int t0, int t1, void* workspace,
                         double* dX_out, void* stream);
/* Status word of the last BA call on this workspace, copied to the DEVICE int
   `out`: bit 0 = Cholesky failed in the last solve (dX was set to 0),
   bit 1 = some kk outside [0, num_patches) (clamped). */
int dpvo_ba_last_status(const void* workspace, int E, int t0, int t1, int* out, void* stream);
/* Split F-BA for a caller that knows the edge list before the update (DPVO
   fixes the patch graph before reproject / corr, dpvo.py:775-824).
   dpvo_ba_plan groups the edges by patch -- it reads ii / jj / kk only, so it
   can run on a side stream concurrently with A-CORR -- and
   dpvo_ba_forward_planned runs the iterations on that workspace (same
   workspace size as dpvo_ba_forward; identical results).  Only for shapes
   dpvo_ba_plan_supported() accepts (the window path: E <= 10240, N <= 16,
   P * P <= 64); otherwise call dpvo_ba_forward. */
int dpvo_ba_plan_supported(int E, int t0, int t1, int P);
/* Byte offsets, inside a dpvo_ba_plan workspace, of the plan arrays:
   out[0] epos int32[E] (edge at sorted position p, grouped by patch, ascending
   edge index inside a patch), out[1] poff int32[E+1] (first position of patch
   u), out[2] pmask uint32[E] (free-pose bits of patch u), out[3] pkk int32[E]
   (kk of patch u, ascending), out[4] meta int32[8] (nuniq, fixed-pose minimum,
   status).  For tests and tools; no reference counterpart. */
int dpvo_ba_plan_offsets(int E, int t0, int t1, int64_t* out);
int dpvo_ba_plan(const int64_t* ii, const int64_t* jj, const int64_t* kk, int E, int num_patches,
                 int num_poses, int t0, int t1, void* workspace, size_t workspace_bytes,
                 void* stream);
int dpvo_ba_forward_planned(float* poses, float* patches, const float* intrinsics,
                            const float* target, const float* weight, const float* lmbda,
                            const int64_t* ii, const int64_t* jj, const int64_t* kk, int E, int P,
                            int num_poses, int num_patches, int t0, int t1, int iterations,
                            void* workspace, size_t workspace_bytes, void* stream);

/* OR the status word of the last dpvo_ba_forward on this workspace (any
   path: window kernels or the large-graph solver) into the DEVICE int `acc`
   (sticky; the caller resets it).  Bits: 1 Cholesky failed (dX = 0, as
   dpvo/ba.py:17-21), 2 kk outside [0, num_patches) (clamped), 4 a patch
   touches more free poses than the large-graph solver handles, 8 too many
   border poses (large graph), 16 a cross-workgroup wait timed out, 32 a
   window graph too large for the per-workgroup LDS plan.  Bits 2..32 mean the step was not the reference's and the extension raises.
   Graph-capturable (one tiny kernel, no host sync). */
int dpvo_ba_status_accumulate(const void* workspace, int E, int t0, int t1, int* acc,
                              void* stream);
/* Register `acc` (device int) as the current device's status sink: the
   window-path kernels OR their status into it directly (no extra launch per
   call); dpvo_ba_status_accumulate is then a no-op for that path. */
int dpvo_ba_set_status_sink(int* acc);
/* Instrumentation (no reference counterpart): the marks the last
   dpvo_ba_forward on this workspace stamped -- wall clock (100 MHz): [0]
   start, [1] setup, then linearize, patch, schur, solve, update per iteration;
   shader clock: [38] start, [39] end; [40..] finer stamps inside the setup
   and the first solve -- copied to the DEVICE array `out`. */
int dpvo_ba_phase_marks(const void* workspace, int E, int t0, int t1, int64_t* out, void* stream);
/* Instrumentation: start / end wall-clock stamps of every workgroup of the
   last Schur launch, [2 x N(N+1)/2] int64 to DEVICE `out`. */
int dpvo_ba_workgroup_marks(const void* workspace, int E, int t0, int t1, int64_t* out,
                            void* stream);
/* Instrumentation: when `on` is nonzero the BA kernels of later calls on this
   process stamp the phase marks above (off by default: the product calls
   store no marks). */
int dpvo_ba_set_marks(int on);
/* Diagnostics (no reference counterpart; the parity tests' view of the
   reference's dX = chol_solve(S, y), ba_cuda.cu:561-562): the pose step dX
   [6N] (fp64, pose t0 + i at [6 i .. 6 i + 5]) of the LAST iteration of the
   last dpvo_ba_forward / dpvo_ba_forward_planned on this workspace, any
   path, copied to the DEVICE array `out`. */
int dpvo_ba_last_dx(const void* workspace, int E, int t0, int t1, double* out, void* stream);

/* F-BA on large graphs (ba_large.hip): DPVO's global BA (dpvo.py:695-715 ->
   fastba.BA(..., eff_impl=True), block_e.cu:43-300) and the edge-sharded
   multi-GPU form.  dpvo_ba_forward dispatches here by itself;
   the split entry points serve the sharded driver:
     setup   once per call: patch grouping, block-sparse pattern of S and the
             band / border analysis.  Rank ownership: a patch belongs to this
             rank iff own_lo <= kk / PPF < own_hi (its source frame); only
             owned patches (and their edges) are linearised and summed.
     build   per iteration: linearise the owned edges and write this rank's
             part of the packed system [y (6N doubles) | S lower 6x6 blocks
             (nblk x 36 doubles)] at workspace + dpvo_gba_packed_offset().
             (all_reduce(SUM) of the first 6N + 36 nblk doubles goes here.)
     solve_update  damp, solve S dX = y (block cyclic reduction + border
             Schur complement, fp64), retract poses t0..t1-1 and the inverse
             depth of every OWNED patch.
   info copies 8 ints to DEVICE `out`: status (bit 0 factorisation failed ->
   dX = 0, bit 1 kk clamped, bit 2 a patch touches > 24 free poses, bit 3
   more than 64 poses couple further back than 16 poses -> dX = 0), unique
   patches, items, nblk, interior poses, border poses, superblock poses g,
   superblocks.  N <= dpvo_gba_max_free_poses(), E <= 2^22. */
size_t dpvo_gba_workspace_bytes(int E, int t0, int t1);
int dpvo_gba_max_free_poses(void);
size_t dpvo_gba_packed_offset(int E, int t0, int t1);
int dpvo_gba_setup(const int64_t* ii, const int64_t* jj, const int64_t* kk, int E, int num_patches,
                   int PPF, int t0, int t1, int own_lo, int own_hi, void* workspace,
                   size_t workspace_bytes, void* stream);
int dpvo_gba_build(const float* poses, const float* patches, const float* intrinsics,
                   const float* target, const float* weight, const float* lmbda, const int64_t* ii,
                   const int64_t* jj, int E, int P, int num_poses, int t0, int t1,
                   void* workspace, void* stream);
int dpvo_gba_solve_update(float* poses, float* patches, int E, int P, int t0, int t1,
                          void* workspace, void* stream);
int dpvo_gba_info(const void* workspace, int E, int t0, int t1, int* out, void* stream);

/* F-REPROJ.  Replaces cuda_ba.reproject (ba.cpp:47-53 -> cuda_reproject,
   ba_cuda.cu:585-616 + reproject :379-429).  coords [E,2,P,P]. */
int dpvo_reproject(const float* poses, const float* patches, const float* intrinsics,
                   const int64_t* ii, const int64_t* jj, const int64_t* kk, int E, int P,
                   int num_poses, int num_patches, float* coords, void* stream);

/* dpvo_reproject plus, in the same launch (one extra workgroup), the A-CORR
   edge order: order[0..E) = edges grouped by target frame jj (jj in [0, N2);
   keys outside share the last group).  Feeds
   dpvo_corr_forward_levels_nhwc_ordered. */
int dpvo_reproject_ordered(const float* poses, const float* patches, const float* intrinsics,
                           const int64_t* ii, const int64_t* jj, const int64_t* kk, int E, int P,
                           int num_poses, int num_patches, int N2, float* coords, int32_t* order,
                           void* stream);

/* dpvo_reproject_ordered plus dpvo_ba_plan(ii, jj, kk, .., t0, t1, workspace)
   in the same launch: the start of a DPVO update (dpvo.py:775-824 reprojects,
   then runs BA on the same edges), so the edge grouping the window BA needs
   runs beside the reprojection instead of as its own launch.  workspace is
   then passed to dpvo_ba_forward_planned.  Same outputs, bit for bit, as the
   two separate calls; DPVO_ERR_UNSUPPORTED where dpvo_ba_plan_supported is 0. */
int dpvo_reproject_ordered_plan(const float* poses, const float* patches,
                                const float* intrinsics, const int64_t* ii, const int64_t* jj,
                                const int64_t* kk, int E, int P, int num_poses, int num_patches,
                                int N2, float* coords, int32_t* order, int t0, int t1,
                                void* workspace, size_t workspace_bytes, void* stream);
/* dpvo_reproject_ordered_plan plus, in the same launch, the insertion of the
   update's new frame into the channels-last pyramid (dpvo_feature_pyramid_insert's
   arguments: src [C, H, W] NCHW level-1 frame, dst[l] the channels-last slot of
   level l, scale[l] in {1, 2, 4, 8}, dtype F32 / F16).  The insertion tiles run
   on the CUs the reprojection and the single-workgroup plan leave idle (DPVO
   inserts the frame in __call__ just before update(); nothing in this launch
   reads the slot it writes).  Outputs bit-identical to the separate calls. */
int dpvo_reproject_ordered_plan_insert(const float* poses, const float* patches,
                                       const float* intrinsics, const int64_t* ii,
                                       const int64_t* jj, const int64_t* kk, int E, int P,
                                       int num_poses, int num_patches, int N2, float* coords,
                                       int32_t* order, int t0, int t1, void* workspace,
                                       size_t workspace_bytes, const void* src, void* const* dst,
                                       const int* scale, int L, int C, int H, int W, int dtype,
                                       void* stream);
/* Device-scalar variants for graph-replayed DPVO updates (the window start t0
   moves every frame, shapes stay fixed): t0 is read from the int32 device
   scalar *t0_dev, N = t1 - t0 is given.  Same results as the host-t0 calls. */
int dpvo_reproject_ordered_plan_dev(const float* poses, const float* patches,
                                    const float* intrinsics, const int64_t* ii, const int64_t* jj,
                                    const int64_t* kk, int E, int P, int num_poses,
                                    int num_patches, int N2, float* coords, int32_t* order,
                                    const int32_t* t0_dev, int N, void* workspace,
                                    size_t workspace_bytes, void* stream);
int dpvo_ba_forward_planned_dev(float* poses, float* patches, const float* intrinsics,
                                const float* target, const float* weight, const float* lmbda,
                                const int64_t* ii, const int64_t* jj, const int64_t* kk, int E,
                                int P, int num_poses, int num_patches, const int32_t* t0_dev,
                                int N, int iterations, void* workspace, size_t workspace_bytes,
                                void* stream);

/* F-NBR.  Replaces cuda_ba.neighbors (ba.cpp:59-97).  Groups edges by ii,
   stable-sorts each group by jj; ix = previous edge, jx = next edge, -1 at
   the ends.  Single-workgroup LDS sort: E <= dpvo_neighbors_max_edges(). */
int dpvo_neighbors_max_edges(void);
int dpvo_neighbors(const int64_t* ii, const int64_t* jj, int E, int64_t* ix, int64_t* jx,
                   void* stream);

/* ---------------------------------------------------------------- lietorch */

/* L-SE3.  Replaces lietorch_backends.{expm, logm, inv, mul, adj, adjT, act,
   act4, as_matrix, projector, Jinv} (dpvo/lietorch/src/lietorch.cpp:18-283,
   lietorch_gpu.cu:20-601).  group: 1 = SO3, 3 = SE3 (dispatch.h:24-45).
   dtype DPVO_F32 / DPVO_F64.  n elements, each row contiguous:
     op 0 exp   : X=a[K]          -> out[N]
     op 1 log   : X[N]            -> out[K]
     op 2 inv   : X[N]            -> out[N]
     op 3 mul   : X[N], Y[N]      -> out[N]
     op 4 adj   : X[N], Y=a[K]    -> out[K]
     op 5 adjT  : X[N], Y=a[K]    -> out[K]
     op 6 act   : X[N], Y=p[3]    -> out[3]
     op 7 act4  : X[N], Y=p[4]    -> out[4]
     op 8 matrix: X[N]            -> out[4x4]
     op 9 proj  : X[N]            -> out[NxN]
     op 10 Jinv : X[N], Y=a[K]    -> out[K]
   Quaternions are normalised on load (so3.h:95-97). */
int dpvo_lie_forward(int group, int op, int dtype, int n, const void* X, const void* Y, void* out,
                     void* stream);

/* Backward of ops 0-7 (lietorch_gpu.cu:32-256); gradient rows of group
   elements are N-strided with the tangent gradient in the first K entries
   (the reference convention).  out0 = dX (or da for exp), out1 = dY/da/dp. */
int dpvo_lie_backward(int group, int op, int dtype, int n, const void* grad, const void* X,
                      const void* Y, void* out0, void* out1, void* stream);

/* PatchGraph edge bookkeeping on the device (dpvo/dpvo.py:480-568,
   dpvo/patchgraph.py:11-63), static MAX_EDGES buffers, counts in the device
   int array `counts`: [0] num_edges, [1] num_edges_inac, [2] error flags
   (1 append overflow -> edges not added; 2 inactive store full -> removed
   edges not stored, like the reference's warning), [3..4] scratch.  No host
   synchronisation.
   dpvo_pg_append replaces append_factors(ii=kk_new, jj=jj_new): edges at
   [num, num + n), ii = ix[kk], net rows zeroed (net may be null).
   dpvo_pg_remove replaces remove_factors(mask, store): mask (uint8, 1 =
   remove, length >= num) or, when mask is null, the DPVO window rule
   ix[kk] < thresh (dpvo.py:684) sparing loop-closure edges with
   jj - ii > 30 and jj > lc_min when lc_min >= 0 (:685-688).  Kept edges are
   compacted in order into the *_b ("back") buffers -- the caller swaps
   them with the active set -- and removed ones appended in order to the
   inactive store when `store`.  pos: int scratch [max_edges]. */
int dpvo_pg_append(const int64_t* ix, const int64_t* kk_new, const int64_t* jj_new, int n,
                   int64_t* ii, int64_t* jj, int64_t* kk, float* net, int DIM, int* counts,
                   int max_edges, void* stream);
int dpvo_pg_remove(const uint8_t* mask, const int64_t* ix, int64_t thresh, int64_t lc_min,
                   int store, int64_t* ii, int64_t* jj, int64_t* kk, float* net, float* weight,
                   float* target, int64_t* ii_b, int64_t* jj_b, int64_t* kk_b, float* net_b,
                   float* weight_b, float* target_b, int64_t* ii_i, int64_t* jj_i, int64_t* kk_i,
                   float* weight_i, float* target_i, int DIM, int* counts, int* pos,
                   int max_edges, void* stream);
/* DPVO.keyframe's window removal (dpvo.py:684-693) with thresholds relative to
   the device frame count n = *n_dev: remove ix[kk] < n + thresh_off, except
   (lc_on) edges with jj - ii > 30 and jj > n + lc_off.  Graph-replayable. */
int dpvo_pg_remove_window_dev(const int64_t* ix, const int32_t* n_dev, int64_t thresh_off,
                              int64_t lc_off, int lc_on, int store, int64_t* ii, int64_t* jj,
                              int64_t* kk, float* net, float* weight, float* target,
                              int64_t* ii_b, int64_t* jj_b, int64_t* kk_b, float* net_b,
                              float* weight_b, float* target_b, int64_t* ii_i, int64_t* jj_i,
                              int64_t* kk_i, float* weight_i, float* target_i, int DIM,
                              int* counts, int* pos, int max_edges, void* stream);
/* append_factors with a device count: n = min(*n_dev, n_cap) edges (e.g. the
   output of dpvo_edges_loop, dpvo.py:986-988).  Graph-replayable. */
int dpvo_pg_append_dev(const int64_t* ix, const int64_t* kk_new, const int64_t* jj_new,
                       const int32_t* n_dev, int n_cap, int64_t* ii, int64_t* jj, int64_t* kk,
                       float* net, int DIM, int* counts, int max_edges, void* stream);
/* DPVO.keyframe's frame-drop removal (dpvo.py:633-641): when kf[0] (the
   device decision of dpvo_kf_motion), remove the active edges with ii == kf[1]
   or jj == kf[1], not stored.  Always compacts into the *_b buffers (a copy
   when nothing is dropped), so the caller swaps unconditionally. */
int dpvo_pg_remove_frame_dev(const int32_t* kf, int64_t* ii, int64_t* jj, int64_t* kk,
                             float* net, float* weight, float* target, int64_t* ii_b,
                             int64_t* jj_b, int64_t* kk_b, float* net_b, float* weight_b,
                             float* target_b, int DIM, int* counts, int* pos, int max_edges,
                             void* stream);

/* --------------------------------------------------------- SPD solve (training) */

/* Batched dense SPD factor + solve: the device side of CholeskySolver
   (dpvo/ba.py:13-38, which calls torch.linalg.cholesky_ex(H) and
   cholesky_solve(b, U); block_solve 67-77 passes it the damped pose system).
   batch items of H [n, n] (row-major; the lower triangle is read, as
   cholesky_ex(upper=False)) and B [n, k]; dtype DPVO_F32 / DPVO_F64.
   factor = 1: L = lower Cholesky factor (zeros above; required when
   n x (n + k) elements exceed 160 KB of LDS: it is then the working copy),
   X = H^-1 B, info[b] = first column whose pivot is not positive (1-based,
   0 = success; LAPACK potrf / cholesky_ex semantics), X = 0 for a failed item.
   factor = 0: H holds a lower factor from a factor = 1 call; X = (H H^T)^-1 B,
   L and info must be null.  One 256-thread workgroup per item. */
int dpvo_spd_solve(const void* H, const void* B, void* L, void* X, int32_t* info, int batch, int n,
                   int k, int factor, int dtype, void* stream);

/* ---------------------------------------------------------------- keyframe */

/* DPVO.keyframe's decision (dpvo.py:586-599, 619-624) on the device.  st =
   {n, m} (device frame counters), i = n - keyframe_index - 1,
   j = n - keyframe_index + 1; motionmag over the active edges with
   projective_ops.flow_mag (projective_ops.py:120-130, beta 0.5).  Writes
   kf = {drop, k = n - keyframe_index} and mag = {motionmag(i,j),
   motionmag(j,i)}.  No host synchronisation: kf predicates
   dpvo_pg_remove_frame_dev and dpvo_kf_shift. */
int dpvo_kf_motion(const int64_t* ii, const int64_t* jj, const int64_t* kk, const int32_t* counts,
                   const float* poses, const float* patches, const float* intrinsics, int P,
                   const int32_t* st, int keyframe_index, double keyframe_thresh, int32_t* kf,
                   float* mag, void* stream);
/* The rest of a frame drop (dpvo.py:626-673), predicated on kf[0]: log
   (t1, t0, poses[k] * poses[k-1]^-1) as pg.delta[t1] into delta_log[7 x cap] /
   delta_tstamps[2 x cap] at *delta_count (optional: all three null), shift the
   active edges past k (kk -= M, ii -= 1; jj -= 1), move the per-frame rows
   k+1 .. n-1 of every frame array one row down (ring[a] > 0: row = frame %
   ring[a], the imap/gmap/fmap rings), then n -= 1, m -= M.  A drop whose
   pg.delta record finds the log full ORs 8 into counts[2] (the patch graph's
   error word; the record is not kept). */
int dpvo_kf_shift(const int32_t* kf, int M, int32_t* st, int64_t* ii, int64_t* jj, int64_t* kk,
                  int32_t* counts, int max_edges, void* const* frame_arrays,
                  const int64_t* bytes_per_frame, const int32_t* ring, int narrays,
                  const float* poses, const int64_t* tstamps, float* delta_log,
                  int64_t* delta_tstamps, int32_t* delta_count, int delta_cap, void* stream);
/* PatchGraph.edges_loop (dpvo/patchgraph.py:65-91, reduce_edges
   loop_closure/optim_utils.py:24-60) gated like its caller (dpvo.py:984-988:
   only when n - *last_global_ba >= global_opt_freq; *last_global_ba = n when
   edges are found; last_global_ba may be null = no gate).  n = st[0] on the
   device, n_cap >= n sizes the launch.  Writes kk (i M + arange(M)) and jj of
   the accepted loop edges and their count (edges x M) to out_n, ready for
   dpvo_pg_append_dev.  work: dpvo_edges_loop_work_floats() floats.
   Limits: (global_opt_freq - keyframe_index) x min(n_cap - removal_window,
   max_edge_age) <= 16384, n_cap x (global_opt_freq - keyframe_index) <=
   131072, max_num_edges <= 1024.  A device n above n_cap takes no loop edges
   and ORs 4 into *errors (optional; the patch graph's counts[2]). */
int dpvo_edges_loop(const float* poses, const float* patches, const float* intrinsics,
                    const int64_t* ix, int P, int M, const int32_t* st, int n_cap,
                    int32_t* last_global_ba, int removal_window, int max_edge_age,
                    int global_opt_freq, int keyframe_index, float backend_thresh,
                    int max_num_edges, int nms, float* work, int64_t* out_kk, int64_t* out_jj,
                    int32_t* out_n, int32_t* errors, void* stream);
size_t dpvo_edges_loop_work_floats(void);

#ifdef __cplusplus
}
#endif

#endif /* DPVO_HOT_H */
