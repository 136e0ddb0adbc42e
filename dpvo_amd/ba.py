"""Dense block solves for the training path of dpvo/ba.py.

The reference (dpvo/ba.py:13-38, 59-77) solves its damped pose system with
torch.linalg.cholesky_ex + cholesky_solve inside an autograd Function that
returns zeros (and no gradient) when the factorisation fails.  Here the
factor and both triangular sweeps are this build's batched HIP kernel
(spd_solve.hip, through cuda_ba.spd_solve / spd_solve_factored and the C ABI
dpvo_spd_solve); the gradient reuses the stored factor.

Gradient of x = H^-1 b (H symmetric):  db = H^-1 g,  dH = -x db^T  (the same
expression the reference returns: it treats H as unconstrained, so the caller
symmetrises if it needs to).  The per-frame inference BA does not come here
(it runs the fused fastba kernels).
"""
from __future__ import annotations

import torch

from ._native import load_extension

_cuda_ba = load_extension("cuda_ba")


def _require_gpu(t, name):
    if not t.is_cuda:
        raise RuntimeError(f"{name} must be a GPU (HIP) tensor; the MI355X build has no CPU path")


class CholeskySolver(torch.autograd.Function):
    """x = H^-1 b for SPD H [..., n, n], b [..., n, k] (replaces dpvo/ba.py:13-38).
    A failed factorisation anywhere in the batch gives x = 0 and no gradient,
    the reference's "don't crash training" rule."""

    @staticmethod
    def forward(ctx, H, b):
        _require_gpu(H, "H")
        _require_gpu(b, "b")
        x, L, info = _cuda_ba.spd_solve(H, b)
        ctx.failed = bool(torch.any(info))  # one host sync, as the reference's torch.any
        if ctx.failed:
            return torch.zeros_like(b)
        ctx.save_for_backward(L, x)
        return x

    @staticmethod
    def backward(ctx, grad_x):
        if ctx.failed:
            return None, None
        L, x = ctx.saved_tensors
        db = _cuda_ba.spd_solve_factored(L, grad_x.contiguous())
        dH = -(x @ db.transpose(-1, -2))
        return dH, db


def _blocks_to_dense(A):
    """[b, n, m, p, q] block matrix -> dense [b, n p, m q]."""
    b, n, m, p, q = A.shape
    return A.transpose(2, 3).reshape(b, n * p, m * q)


def _dense_to_blocks(X, n, p, m, q):
    """dense [b, n p, m q] -> [b, n, m, p, q] block matrix."""
    return X.reshape(X.shape[0], n, p, m, q).transpose(2, 3)


def block_matmul(A, B):
    """Block matrix product C_ij = sum_k A_ik B_kj (dpvo/ba.py:59-65):
    A [b, n1, m1, p1, q1], B [b, m1, m2, q1, q2] -> [b, n1, m2, p1, q2]."""
    _, n1, _, p1, _ = A.shape
    _, _, m2, _, q2 = B.shape
    return _dense_to_blocks(_blocks_to_dense(A) @ _blocks_to_dense(B), n1, p1, m2, q2)


def block_solve(A, B, ep=1.0, lm=1e-4):
    """Damped block solve (dpvo/ba.py:67-77): X = (A + diag(ep + lm diag A))^-1 B
    on the dense form, A [b, n, n, p, p], B [b, n, m, p, q] -> [b, n, m, p, q]."""
    _, n1, _, p1, _ = A.shape
    _, _, m2, _, q2 = B.shape
    Ad = _blocks_to_dense(A)
    Ad = Ad + torch.diag_embed(ep + lm * torch.diagonal(Ad, dim1=-2, dim2=-1))
    X = CholeskySolver.apply(Ad, _blocks_to_dense(B))
    return _dense_to_blocks(X, n1, p1, m2, q2)


__all__ = ["CholeskySolver", "block_matmul", "block_solve"]
