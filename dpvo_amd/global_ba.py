"""DPVO's global bundle adjustment driver on the MI355X ops.

Reference: DPVO.__run_global_BA (dpvo/dpvo.py:695-715) and
PatchGraph.normalize (dpvo/patchgraph.py:93-106), triggered from
DPVO.update (dpvo.py:814-816) when an active edge reaches back past the
removal window.  The driver concatenates the inactive store and the active
edges (inactive first), normalises depth and scale, and runs
fastba.BA(..., iterations=2, eff_impl=True) from t0 = min(ii) to n -- on the
large-graph HIP path (ba_large.hip).

The fork's MIXED_PRECISION patch graph holds target / weight in fp16, which
its cuda_ba rejects, so its global BA never runs; here fp16
buffers are widened to fp32 on the device before the call (the values the
kernels see are the fp16 values, exactly).

`pg` is anything with the reference PatchGraph's edge attributes: ii, jj, kk,
target, weight, ii_inac, jj_inac, kk_inac, target_inac, weight_inac,
num_edges, num_edges_inac -- dpvo_amd.patchgraph.DevicePatchGraph or the
reference's own object.  The edge counts are host integers, as in the
reference (one read of the device counts).
"""
from __future__ import annotations

import torch

from . import fastba
from .lietorch import SE3


def needs_global_ba(pg, n, removal_window):
    """dpvo.py:815 condition: an active edge with ii < n - REMOVAL_WINDOW - 1
    (the caller also checks ran_global_ba[n])."""
    E = pg.num_edges
    return bool((pg.ii[:E] < n - removal_window - 1).any())


def normalize(poses, patches, n, M, delta=None, points=None, intrinsics=None, ix=None, m=None):
    """PatchGraph.normalize (patchgraph.py:93-106), in place.

    poses [N, 7] (or [1, N, 7]), patches [N*M, 3, P, P] (or [1, N*M, ...]):
    s = mean inverse depth of frames [0, n); depths /= s, translations *= s,
    every pose re-based on pose 0 (poses * poses[0]^-1).  delta: the device
    pg.delta log [cap, 7] (dP.scale(s) on every record).  points / intrinsics
    / ix / m: the viewer point cloud of the first m patches (optional)."""
    P7 = poses.view(-1, 7)
    P = patches.shape[-1]
    K = patches.view(-1, M, 3, P, P)
    s = K[:n, :, 2].mean()
    K[:n, :, 2] /= s
    P7[:n, :3] *= s
    if delta is not None:
        delta[:, :3] *= s
    P7[:n] = (SE3(P7[:n]) * SE3(P7[[0]]).inv()).data
    if points is not None:
        from . import projective_ops as pops

        X = pops.point_cloud(SE3(P7.view(1, -1, 7)), patches.view(1, -1, 3, P, P)[:, :m],
                             intrinsics.view(1, -1, 4), ix[:m])
        X = (X[..., 1, 1, :3] / X[..., 1, 1, 3:]).reshape(-1, 3)
        points[:len(X)] = X
    return s


def run_global_ba(pg, poses, patches, intrinsics, n, M, lmbda=None, iterations=2, delta=None,
                  points=None, ix=None, m=None):
    """DPVO.__run_global_BA (dpvo.py:695-715): BA over inactive + active
    edges with eff_impl=True, after normalize().  Returns the number of edges
    used (0: nothing to do, the BA is skipped as in the reference)."""
    na, ni = int(pg.num_edges), int(pg.num_edges_inac)
    tot = na + ni

    def cat(a, b, ax):
        return torch.cat((a.narrow(ax, 0, ni), b.narrow(ax, 0, na)), dim=ax)

    target = cat(pg.target_inac, pg.target, 1).float()
    weight = cat(pg.weight_inac, pg.weight, 1).float()
    ii = cat(pg.ii_inac, pg.ii, 0)
    jj = cat(pg.jj_inac, pg.jj, 0)
    kk = cat(pg.kk_inac, pg.kk, 0)
    normalize(poses, patches, n, M, delta=delta, points=points, intrinsics=intrinsics, ix=ix, m=m)
    if lmbda is None:
        lmbda = torch.as_tensor([1e-4], device=poses.device)
    if tot > 0:
        t0 = int(ii.min().item())
        fastba.BA(poses, patches, intrinsics, target, weight, lmbda, ii, jj, kk, t0, n, M,
                  iterations, eff_impl=True)
    return tot


__all__ = ["needs_global_ba", "normalize", "run_global_ba"]
