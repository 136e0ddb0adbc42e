"""Dense block solves of dpvo/ba.py for the training path.

CholeskySolver (dpvo/ba.py:13-38): batched SPD solve with autograd; on a
failed factorisation the forward returns zeros and the backward returns no
gradient ("don't crash training").  block_matmul / block_solve (59-77) are the
block-matrix helpers its callers use.  The factorisation runs on the HIP
device through rocSOLVER (torch.linalg); the per-frame inference BA does not
use this module (it runs the fused HIP kernels of fastba).
"""
from __future__ import annotations

import torch


def _require_gpu(t, name):
    if not t.is_cuda:
        raise RuntimeError(f"{name} must be a GPU (HIP) tensor; the MI355X build has no CPU path")


class CholeskySolver(torch.autograd.Function):
    """x = H^-1 b for SPD H [..., n, n], b [..., n, k] (dpvo/ba.py:13-38)."""

    @staticmethod
    def forward(ctx, H, b):
        _require_gpu(H, "H")
        _require_gpu(b, "b")
        U, info = torch.linalg.cholesky_ex(H)
        if torch.any(info):
            ctx.failed = True
            return torch.zeros_like(b)
        xs = torch.cholesky_solve(b, U)
        ctx.save_for_backward(U, xs)
        ctx.failed = False
        return xs

    @staticmethod
    def backward(ctx, grad_x):
        if ctx.failed:
            return None, None
        U, xs = ctx.saved_tensors
        dz = torch.cholesky_solve(grad_x, U)
        dH = -torch.matmul(xs, dz.transpose(-1, -2))
        return dH, dz


def block_matmul(A, B):
    """Block matrix product (dpvo/ba.py:59-65): A [b, n1, m1, p1, q1],
    B [b, n2, m2, p2, q2] -> [b, n1, m2, p1, q2]."""
    b, n1, m1, p1, q1 = A.shape
    b, n2, m2, p2, q2 = B.shape
    A = A.permute(0, 1, 3, 2, 4).reshape(b, n1 * p1, m1 * q1)
    B = B.permute(0, 1, 3, 2, 4).reshape(b, n2 * p2, m2 * q2)
    return torch.matmul(A, B).reshape(b, n1, p1, m2, q2).permute(0, 1, 3, 2, 4)


def block_solve(A, B, ep=1.0, lm=1e-4):
    """Damped block solve (dpvo/ba.py:67-77): (A + (ep + lm A) I) X = B."""
    b, n1, m1, p1, q1 = A.shape
    b, n2, m2, p2, q2 = B.shape
    A = A.permute(0, 1, 3, 2, 4).reshape(b, n1 * p1, m1 * q1)
    B = B.permute(0, 1, 3, 2, 4).reshape(b, n2 * p2, m2 * q2)
    A = A + (ep + lm * A) * torch.eye(n1 * p1, device=A.device, dtype=A.dtype)
    X = CholeskySolver.apply(A, B)
    return X.reshape(b, n1, p1, m2, q2).permute(0, 1, 3, 2, 4)


__all__ = ["CholeskySolver", "block_matmul", "block_solve"]
