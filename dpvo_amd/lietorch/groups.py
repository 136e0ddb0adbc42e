"""Lie group objects and their autograd ops.

Behaviour follows dpvo/lietorch/groups.py:51-322, group_ops.py:7-101 and
broadcasting.py:5-31 (cuteboyqq/DPVO); the arithmetic runs in the HIP kernels
of `lietorch_backends` (dpvo_amd/csrc/lie.hip).

Conventions (reference): SE3 data = (tx, ty, tz, qx, qy, qz, qw); tangent =
(tau, phi); gradients w.r.t. a group element live in the tangent space,
carried in an embedding-sized row whose first K entries are used.
"""
from __future__ import annotations

import numpy as np
import torch

from .._native import load_extension

_backend = load_extension("lietorch_backends")


# --------------------------------------------------------------- autograd ops
def _make_op(name, fwd, bwd):
    """Autograd Function for one backend op: forward(group_id, *tensors)."""

    def forward(ctx, group_id, *inputs):
        ctx.group_id = group_id
        ctx.save_for_backward(*inputs)
        return fwd(group_id, *inputs)

    def backward(ctx, grad):
        if bwd is None:
            raise RuntimeError(f"{name}: no backward (lietorch group_ops.py:60-66)")
        grads = bwd(ctx.group_id, grad.contiguous(), *ctx.saved_tensors)
        return (None,) + tuple(grads)

    return type(name, (torch.autograd.Function,),
                {"forward": staticmethod(forward), "backward": staticmethod(backward)})


Exp = _make_op("Exp", _backend.expm, _backend.expm_backward)
Log = _make_op("Log", _backend.logm, _backend.logm_backward)
Inv = _make_op("Inv", _backend.inv, _backend.inv_backward)
Mul = _make_op("Mul", _backend.mul, _backend.mul_backward)
Adj = _make_op("Adj", _backend.adj, _backend.adj_backward)
AdjT = _make_op("AdjT", _backend.adjT, _backend.adjT_backward)
Act3 = _make_op("Act3", _backend.act, _backend.act_backward)
Act4 = _make_op("Act4", _backend.act4, _backend.act4_backward)
Jinv = _make_op("Jinv", _backend.Jinv, None)
ToMatrix = _make_op("ToMatrix", _backend.as_matrix, None)


class ToVec(torch.autograd.Function):
    """group -> embedding vector; backward maps a tangent gradient through the
    orthogonal projector (group_ops.py:88-101)."""

    @staticmethod
    def forward(ctx, group_id, data):
        ctx.group_id = group_id
        ctx.save_for_backward(data)
        return data

    @staticmethod
    def backward(ctx, grad):
        data, = ctx.saved_tensors
        J = _backend.projector(ctx.group_id, data)
        return None, torch.matmul(grad.unsqueeze(-2), J).squeeze(-2)


class FromVec(torch.autograd.Function):
    """embedding vector -> group (group_ops.py:73-86)."""

    @staticmethod
    def forward(ctx, group_id, data):
        ctx.group_id = group_id
        ctx.save_for_backward(data)
        return data

    @staticmethod
    def backward(ctx, grad):
        data, = ctx.saved_tensors
        J = _backend.projector(ctx.group_id, data)
        return None, torch.matmul(grad.unsqueeze(-2), torch.linalg.pinv(J)).squeeze(-2)


def _broadcast(x, y=None):
    """Flatten operands to [n, dim] contiguous rows, broadcasting the leading
    (batch) dims like broadcasting.py:10-31; returns (rows, out_batch_shape)."""
    if y is None:
        return (x.reshape(-1, x.shape[-1]).contiguous(),), tuple(x.shape[:-1])
    if x.dim() != y.dim():
        raise ValueError("lietorch broadcasting needs operands of equal rank")
    shape = torch.broadcast_shapes(x.shape[:-1], y.shape[:-1])
    xe = x.expand(*shape, x.shape[-1]).reshape(-1, x.shape[-1]).contiguous()
    ye = y.expand(*shape, y.shape[-1]).reshape(-1, y.shape[-1]).contiguous()
    return (xe, ye), tuple(shape)


# --------------------------------------------------------------- group objects
class LieGroup:
    """Batch of group elements stored as an embedding tensor `data[..., N]`."""

    group_name = "LieGroup"
    group_id = 0
    manifold_dim = 0
    embedded_dim = 0
    id_elem = None

    def __init__(self, data):
        self.data = data

    def __repr__(self):
        return f"{self.group_name}: size={self.shape}, device={self.device}, dtype={self.dtype}"

    # ---- tensor-like properties
    @property
    def shape(self):
        return self.data.shape[:-1]

    @property
    def device(self):
        return self.data.device

    @property
    def dtype(self):
        return self.data.dtype

    @property
    def tangent_shape(self):
        return self.data.shape[:-1] + (self.manifold_dim,)

    # ---- construction
    @classmethod
    def _batch_shape(cls, batch_shape):
        if len(batch_shape) == 1 and isinstance(batch_shape[0], (tuple, list, torch.Size)):
            return tuple(batch_shape[0])
        return tuple(batch_shape)

    @classmethod
    def Identity(cls, *batch_shape, **kwargs):
        shape = cls._batch_shape(batch_shape)
        data = cls.id_elem.reshape(1, -1)
        if "device" in kwargs:
            data = data.to(kwargs["device"])
        if "dtype" in kwargs:
            data = data.type(kwargs["dtype"])
        data = data.repeat(int(np.prod(shape)), 1)
        return cls(data).view(shape)

    @classmethod
    def IdentityLike(cls, G):
        return cls.Identity(G.shape, device=G.data.device, dtype=G.data.dtype)

    @classmethod
    def InitFromVec(cls, data):
        return cls(cls.apply_op(FromVec, data))

    @classmethod
    def Random(cls, *batch_shape, sigma=1.0, **kwargs):
        shape = cls._batch_shape(batch_shape)
        xi = torch.randn(shape + (cls.manifold_dim,), **kwargs)
        return cls.exp(sigma * xi)

    @classmethod
    def apply_op(cls, op, x, y=None):
        rows, out_shape = _broadcast(x, y)
        out = op.apply(cls.group_id, *rows)
        return out.view(out_shape + (-1,))

    @classmethod
    def exp(cls, x):
        return cls(cls.apply_op(Exp, x))

    # ---- group operations
    def log(self):
        return self.apply_op(Log, self.data)

    def inv(self):
        return self.__class__(self.apply_op(Inv, self.data))

    def mul(self, other):
        return self.__class__(self.apply_op(Mul, self.data, other.data))

    def retr(self, a):
        """Exp(a) * X (groups.py:153-156)."""
        return self.__class__(self.apply_op(Mul, self.__class__.apply_op(Exp, a), self.data))

    def adj(self, a):
        return self.apply_op(Adj, self.data, a)

    def adjT(self, a):
        return self.apply_op(AdjT, self.data, a)

    def Jinv(self, a):
        return self.apply_op(Jinv, self.data, a)

    def act(self, p):
        if p.shape[-1] == 3:
            return self.apply_op(Act3, self.data, p)
        if p.shape[-1] == 4:
            return self.apply_op(Act4, self.data, p)
        raise ValueError("act expects points of dimension 3 or 4")

    def matrix(self):
        """4x4 matrices by acting on the identity (groups.py:180-184)."""
        eye = torch.eye(4, dtype=self.dtype, device=self.device)
        eye = eye.view([1] * (self.data.dim() - 1) + [4, 4])
        return self.__class__(self.data[..., None, :]).act(eye).transpose(-1, -2)

    def translation(self):
        p = torch.as_tensor([0.0, 0.0, 0.0, 1.0], dtype=self.dtype, device=self.device)
        p = p.view([1] * (self.data.dim() - 1) + [4])
        return self.apply_op(Act4, self.data, p)

    def vec(self):
        return self.apply_op(ToVec, self.data)

    def quaternion(self):
        raise NotImplementedError("quaternion() is not implemented (nor in the reference)")

    # ---- container protocol
    def detach(self):
        return self.__class__(self.data.detach())

    def view(self, dims):
        return self.__class__(self.data.view(tuple(dims) + (self.embedded_dim,)))

    def __mul__(self, other):
        if isinstance(other, LieGroup):
            return self.mul(other)
        if isinstance(other, torch.Tensor):
            return self.act(other)
        return NotImplemented

    def __getitem__(self, index):
        return self.__class__(self.data[index])

    def __setitem__(self, index, item):
        self.data[index] = item.data

    def to(self, *args, **kwargs):
        return self.__class__(self.data.to(*args, **kwargs))

    def cpu(self):
        return self.__class__(self.data.cpu())

    def cuda(self):
        return self.__class__(self.data.cuda())

    def float(self, device=None):
        return self.__class__(self.data.float())

    def double(self, device=None):
        return self.__class__(self.data.double())

    def unbind(self, dim=0):
        return [self.__class__(x) for x in self.data.unbind(dim=dim)]


class LieGroupParameter(torch.Tensor):
    """An optimisation variable on a group: a zero tangent vector (the leaf
    tensor an optimiser sees and steps) anchored at ``group``.  Every group
    operation acts on ``retr()`` = Exp(tangent) * anchor, and ``add_`` folds a
    step into the anchor.  Public name and behaviour of lietorch's class
    (dpvo/lietorch/groups.py:9-48); nothing on the update path uses it."""

    __torch_function__ = torch._C._disabled_torch_function_impl

    def __new__(cls, group, requires_grad=True):
        tangent = group.data.new_zeros(group.tangent_shape).as_subclass(cls)
        tangent.requires_grad_(requires_grad)
        tangent.group = group
        return tangent

    def __init__(self, group, requires_grad=True):  # state set in __new__
        pass

    def retr(self):
        return self.group.retr(self)

    def add_(self, update, alpha):
        self.group = self.group.exp(alpha * update) * self.group
        return self

    def __mul__(self, other):
        rhs = other.retr() if isinstance(other, LieGroupParameter) else other
        return self.retr() * rhs


def _on_retraction(name):
    def method(self, *args):
        return getattr(self.retr(), name)(*args)

    method.__name__ = name
    return method


for _name in ("log", "inv", "adj", "__getitem__"):
    setattr(LieGroupParameter, _name, _on_retraction(_name))


class SO3(LieGroup):
    group_name = "SO3"
    group_id = 1
    manifold_dim = 3
    embedded_dim = 4
    id_elem = torch.as_tensor([0.0, 0.0, 0.0, 1.0])

    def __init__(self, data):
        if isinstance(data, SE3):
            data = data.data[..., 3:7]
        super().__init__(data)


class SE3(LieGroup):
    group_name = "SE3"
    group_id = 3
    manifold_dim = 6
    embedded_dim = 7
    id_elem = torch.as_tensor([0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 1.0])

    def __init__(self, data):
        if isinstance(data, SO3):
            data = torch.cat([torch.zeros_like(data.data[..., :3]), data.data], -1)
        super().__init__(data)

    def scale(self, s):
        t, q = self.data.split([3, 4], -1)
        return SE3(torch.cat([t * s.unsqueeze(-1), q], dim=-1))


class _Unsupported(LieGroup):
    def __init__(self, data):
        raise NotImplementedError(
            f"{self.group_name} (lietorch group id {self.group_id}) is not part of the MI355X "
            "build: DPVO's per-frame hot path uses SE3 only (SURVEY 8a L-SE3)")


class RxSO3(_Unsupported):
    group_name = "RxSO3"
    group_id = 2
    manifold_dim = 4
    embedded_dim = 5
    id_elem = torch.as_tensor([0.0, 0.0, 0.0, 1.0, 1.0])


class Sim3(_Unsupported):
    group_name = "Sim3"
    group_id = 4
    manifold_dim = 7
    embedded_dim = 8
    id_elem = torch.as_tensor([0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 1.0, 1.0])


def cat(group_list, dim):
    return group_list[0].__class__(torch.cat([X.data for X in group_list], dim=dim))


def stack(group_list, dim):
    return group_list[0].__class__(torch.stack([X.data for X in group_list], dim=dim))
