"""fastba on MI355X: Schur bundle adjustment (F-BA), reprojection (F-REPROJ)
and edge neighbours (F-NBR), backed by the `cuda_ba` HIP extension.

Reference surface: dpvo/fastba/ba.py:1-8 (cuteboyqq/DPVO) --
`BA(poses, patches, intrinsics, target, weight, lmbda, ii, jj, kk, t0, t1,
M, iterations, eff_impl=False)` updates poses[t0:t1] and the inverse depth
of every patch in kk IN PLACE and returns nothing useful (the extension
returns []); `neighbors(ii, jj)`; `reproject(poses, patches, intrinsics,
ii, jj, kk)` -> [1, E, 2, P, P].
"""
from __future__ import annotations

import torch

from .._native import load_extension

cuda_ba = load_extension("cuda_ba")


def BA(poses, patches, intrinsics, target, weight, lmbda, ii, jj, kk, t0, t1, M, iterations,
       eff_impl=False, plan=None):
    """fastba.BA (dpvo/fastba/ba.py:7-8): note the extension's argument order
    puts patches-per-frame (M) before t0 (ba.cpp:32-45).  ``plan``: a
    workspace from :func:`plan` for the same ii / jj / kk / t0 / t1 (the edge
    grouping then is not redone here)."""
    data = poses.data if hasattr(poses, "data") else poses
    # the fork's MIXED_PRECISION patch graph holds target / weight in fp16
    # (patchgraph.py:46-52 with autocast kwargs); the kernels read fp32, so the
    # global-BA call of dpvo.py:695-715 gets fp32 copies here (with
    # fp16 buffers the fork's own global BA never runs)
    if target.dtype != torch.float32:
        target = target.float()
    if weight.dtype != torch.float32:
        weight = weight.float()
    if plan is not None:
        cuda_ba.forward_planned(plan, data, patches, intrinsics, target, weight, lmbda, ii, jj, kk,
                                t0, t1, iterations)
        return []
    return cuda_ba.forward(data, patches, intrinsics, target, weight, lmbda, ii, jj, kk, M, t0, t1,
                           iterations, eff_impl)


def BA_dev(poses, patches, intrinsics, target, weight, lmbda, ii, jj, kk, t0_dev, N, plan,
           iterations=1):
    """BA on a planned workspace with the window start t0 read from an int32
    device scalar (``t0_dev``) and N = t1 - t0 free poses: graph-replayed
    updates, where t0 moves every frame (same results as BA(plan=...))."""
    data = poses.data if hasattr(poses, "data") else poses
    cuda_ba.forward_planned_dev(plan, data, patches, intrinsics, target.float(), weight.float(),
                                lmbda, ii, jj, kk, t0_dev, int(N), int(iterations))
    return []


def reproject_window_dev(poses, patches, intrinsics, ii, jj, kk, mem, t0_dev, N):
    """reproject(..., mem, plan_window=(t0, t0 + N)) with t0 read from an int32
    device scalar: coords, A-CORR edge order and the BA plan in one launch."""
    return tuple(cuda_ba.reproject_ordered_plan_dev(poses, patches, intrinsics, ii, jj, kk,
                                                    int(mem), t0_dev, int(N)))


def plan(ii, jj, kk, t0, t1, num_patches, num_poses, P=3):
    """Group the edges by patch for a later ``BA(..., plan=ws)`` with the same
    graph.  Reads ii / jj / kk only, so DPVO can issue it on a side stream
    while A-CORR runs (the patch graph is fixed before the update,
    dpvo/dpvo.py:775-824).  Returns None when the window path does not cover
    the shape (then BA() plans internally)."""
    if not cuda_ba.plan_supported(int(ii.numel()), int(t0), int(t1), int(P)):
        return None
    return cuda_ba.plan(ii, jj, kk, int(num_patches), int(num_poses), int(t0), int(t1))


def neighbors(ii, jj):
    """cuda_ba.neighbors (ba.cpp:59-97): previous / next edge of the same ii
    ordered by jj (stable), -1 at the ends."""
    return cuda_ba.neighbors(ii, jj)


def reproject(poses, patches, intrinsics, ii, jj, kk, mem=None, plan_window=None, insert=None):
    """cuda_ba.reproject (ba_cuda.cu:379-429, 585-616).  With ``mem`` (the
    feature ring size the targets jj index), also returns the A-CORR edge
    order (int32 [E], edges grouped by target frame) computed in the same
    launch: ``coords, order = reproject(..., mem=36)``.  With ``mem`` and
    ``plan_window=(t0, t1)`` the same launch also groups the edges for the
    update's BA: ``coords, order, ws = reproject(..., mem=36, plan_window=(t0, t1))``
    and later ``BA(..., plan=ws)`` (identical to :func:`plan`; the window path
    must cover the shape, see :func:`plan`).  With ``insert=(fmap, dst, scales)``
    (and mem, plan_window) the same launch also inserts the update's new frame
    into the channels-last pyramid (``altcorr.insert_frame``'s work; ``dst``
    are the per-level slot views), bit-identical to the separate launches."""
    if insert is not None:
        # insert = (fmap [C, H, W], [channels-last slot view per level], scales):
        # the new frame's pyramid insertion (altcorr.insert_frame) in the same launch
        if mem is None or plan_window is None:
            raise ValueError("reproject: insert needs mem and plan_window")
        fmap, dst, scales = insert
        t0, t1 = plan_window
        return tuple(cuda_ba.reproject_ordered_plan_insert(
            poses, patches, intrinsics, ii, jj, kk, int(mem), int(t0), int(t1), fmap, list(dst),
            [int(s) for s in scales]))
    if mem is None:
        if plan_window is not None:
            raise ValueError("reproject: plan_window needs mem")
        return cuda_ba.reproject(poses, patches, intrinsics, ii, jj, kk)
    if plan_window is not None:
        t0, t1 = plan_window
        return tuple(cuda_ba.reproject_ordered_plan(poses, patches, intrinsics, ii, jj, kk,
                                                    int(mem), int(t0), int(t1)))
    return tuple(cuda_ba.reproject_ordered(poses, patches, intrinsics, ii, jj, kk, int(mem)))


__all__ = ["BA", "BA_dev", "plan", "neighbors", "reproject", "reproject_window_dev", "cuda_ba"]
