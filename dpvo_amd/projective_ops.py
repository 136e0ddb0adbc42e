"""Projective geometry of the update loop (P-TRANSFORM), over dpvo_amd.lietorch.

Restates dpvo/projective_ops.py (cuteboyqq/DPVO): iproj 19-29, proj 32-50,
transform 53-113, point_cloud 115-117, flow_mag 120-130, so that DPVO's
caller code (DPVO.reproject, ba.py) runs unchanged on the HIP lietorch ops.
`reproject` is the fused single-kernel form used by the MI355X update loop
(cuda_ba.reproject semantics: intrinsics row 0, no depth clamp).
"""
from __future__ import annotations

import torch

from .fastba import cuda_ba
from .lietorch import SE3, Sim3

MIN_DEPTH = 0.2


def extract_intrinsics(intrinsics):
    return intrinsics[..., None, None, :].unbind(dim=-1)


def coords_grid(ht, wd, **kwargs):
    y, x = torch.meshgrid(torch.arange(ht).to(**kwargs).float(),
                          torch.arange(wd).to(**kwargs).float(), indexing="ij")
    return torch.stack([x, y], dim=-1)


def iproj(patches, intrinsics):
    """(x, y, d) patches -> homogeneous points ((x-cx)/fx, (y-cy)/fy, 1, d)."""
    x, y, d = patches.unbind(dim=2)
    fx, fy, cx, cy = intrinsics[..., None, None].unbind(dim=2)
    return torch.stack([(x - cx) / fx, (y - cy) / fy, torch.ones_like(d), d], dim=-1)


def proj(X, intrinsics, depth=False):
    """Pinhole projection with inverse depth 1 / max(Z, 0.1)."""
    X, Y, Z, W = X.unbind(dim=-1)
    fx, fy, cx, cy = intrinsics[..., None, None].unbind(dim=2)
    d = 1.0 / Z.clamp(min=0.1)
    x = fx * (d * X) + cx
    y = fy * (d * Y) + cy
    if depth:
        return torch.stack([x, y, d], dim=-1)
    return torch.stack([x, y], dim=-1)


def transform(poses, patches, intrinsics, ii, jj, kk, depth=False, valid=False, jacobian=False,
              tonly=False):
    """Reproject patch kk from frame ii into frame jj; optionally the
    Jacobians at the patch centre (projective_ops.py:53-113)."""
    X0 = iproj(patches[:, kk], intrinsics[:, ii])
    Gij = poses[:, jj] * poses[:, ii].inv()
    if tonly:
        Gij[..., 3:] = torch.as_tensor([0, 0, 0, 1], device=Gij.device)
    X1 = Gij[:, :, None, None] * X0
    x1 = proj(X1, intrinsics[:, jj], depth)

    if jacobian:
        p = X1.shape[2]
        X, Y, Z, H = X1[..., p // 2, p // 2, :].unbind(dim=-1)
        o = torch.zeros_like(H)
        fx, fy, cx, cy = intrinsics[:, jj].unbind(dim=-1)
        d = torch.where(Z.abs() > 0.2, 1.0 / Z, torch.zeros_like(Z))
        if isinstance(Gij, SE3):
            Ja = torch.stack([H, o, o, o, Z, -Y,
                              o, H, o, -Z, o, X,
                              o, o, H, Y, -X, o,
                              o, o, o, o, o, o], dim=-1).view(1, len(ii), 4, 6)
        elif isinstance(Gij, Sim3):  # pragma: no cover - Sim3 is not built
            raise NotImplementedError("Sim3 transform")
        Jp = torch.stack([fx * d, o, -fx * X * d * d, o,
                          o, fy * d, -fy * Y * d * d, o], dim=-1).view(1, len(ii), 2, 4)
        Jj = torch.matmul(Jp, Ja)
        Ji = -Gij[:, :, None].adjT(Jj)
        Jz = torch.matmul(Jp, Gij.matrix()[..., :, 3:])
        return x1, (Z > 0.2).float(), (Ji, Jj, Jz)

    if valid:
        return x1, (X1[..., 2] > 0.2).float()
    return x1


def point_cloud(poses, patches, intrinsics, ix):
    return poses[:, ix, None, None].inv() * iproj(patches, intrinsics[:, ix])


def flow_mag(poses, patches, intrinsics, ii, jj, kk, beta=0.3):
    coords0 = transform(poses, patches, intrinsics, ii, ii, kk)
    coords1, val = transform(poses, patches, intrinsics, ii, jj, kk, tonly=False, valid=True)
    coords2 = transform(poses, patches, intrinsics, ii, jj, kk, tonly=True)
    flow1 = (coords1 - coords0).norm(dim=-1)
    flow2 = (coords2 - coords0).norm(dim=-1)
    return beta * flow1 + (1 - beta) * flow2, (val > 0.5)


def reproject(poses, patches, intrinsics, ii, jj, kk):
    """Fused reprojection of every edge's p x p patch: [1, E, 2, P, P]
    (one HIP kernel; cuda_ba.reproject semantics)."""
    data = poses.data if isinstance(poses, SE3) else poses
    return cuda_ba.reproject(data, patches, intrinsics, ii, jj, kk)
