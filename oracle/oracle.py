"""TEST INFRASTRUCTURE ONLY -- numpy/ctypes front end of the C restatement
of the reference (oracle/dpvo_oracle.c).

Only tests/, __graft_entry__.smoke() and bench.py's ``cpu_baseline`` leg may
import this module, and only as the checker.  The product package
(dpvo_amd/) never imports it.

Every function mirrors a reference entry point (file:line in the C source).
Inputs are numpy arrays (any float dtype is converted to float32, indices to
int64); outputs are numpy arrays.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "_build", "liborc.so")
_lib = None


def build():
    subprocess.check_call(["make", "-s", "-C", _HERE])


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH) or (
            os.path.getmtime(_LIB_PATH) < os.path.getmtime(os.path.join(_HERE, "dpvo_oracle.c"))
        ):
            build()
        _lib = ctypes.CDLL(_LIB_PATH)
    return _lib


def _f32(a):
    return np.ascontiguousarray(np.asarray(a, dtype=np.float32))


def _f64(a):
    return np.ascontiguousarray(np.asarray(a, dtype=np.float64))


def _i64(a):
    return np.ascontiguousarray(np.asarray(a, dtype=np.int64))


def _p(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def _check(rc, name):
    if rc < 0:
        raise RuntimeError(f"oracle {name} failed ({rc})")
    return rc


# ---------------------------------------------------------------- altcorr
def corr_fwd(fmap1, fmap2, coords, ii, jj, radius):
    """cuda_corr.forward semantics (correlation_kernel.cu:82-175, 232-272).
    Returns [B, M, 2R+1, 2R+1, H, W] (x-offset, y-offset) float32."""
    fmap1, fmap2, coords = _f32(fmap1), _f32(fmap2), _f32(coords)
    ii, jj = _i64(ii), _i64(jj)
    B, N1, C, H, W = fmap1.shape
    _, N2, _, H2, W2 = fmap2.shape
    M = coords.shape[1]
    Dp = 2 * radius + 1
    out = np.empty((B, M, Dp, Dp, H, W), np.float32)
    _check(lib().orc_corr_fwd(_p(fmap1), _p(fmap2), _p(coords), _p(ii), _p(jj), B, M, C, H, W,
                              N1, N2, H2, W2, radius, _p(out)), "corr_fwd")
    return out


def corr_bwd(fmap1, fmap2, coords, ii, jj, grad, radius):
    """cuda_corr.backward semantics (correlation_kernel.cu:178-229, 275-325)."""
    fmap1, fmap2, coords, grad = _f32(fmap1), _f32(fmap2), _f32(coords), _f32(grad)
    ii, jj = _i64(ii), _i64(jj)
    B, N1, C, H, W = fmap1.shape
    _, N2, _, H2, W2 = fmap2.shape
    M = coords.shape[1]
    g1 = np.empty_like(fmap1)
    g2 = np.empty_like(fmap2)
    _check(lib().orc_corr_bwd(_p(fmap1), _p(fmap2), _p(coords), _p(ii), _p(jj), _p(grad), B, M, C,
                              H, W, N1, N2, H2, W2, radius, _p(g1), _p(g2)), "corr_bwd")
    return g1, g2


def patchify_fwd(net, coords, radius, clamp=False):
    """cuda_corr.patchify_forward (correlation_kernel.cu:16-47, zero fill) or the
    fork's runtime patchify_forward_kernel_python (clamp=True)."""
    net, coords = _f32(net), _f32(coords)
    B, C, H, W = net.shape
    M = coords.shape[1]
    D = 2 * radius + 2
    out = np.empty((B, M, C, D, D), np.float32)
    _check(lib().orc_patchify_fwd(_p(net), _p(coords), B, C, H, W, M, radius, int(clamp), _p(out)),
           "patchify_fwd")
    return out


def patchify_bwd(net_shape, coords, grad, radius, clamp=False):
    coords, grad = _f32(coords), _f32(grad)
    B, C, H, W = net_shape
    M = coords.shape[1]
    out = np.empty((B, C, H, W), np.float32)
    _check(lib().orc_patchify_bwd(_p(grad), _p(coords), B, C, H, W, M, radius, int(clamp), _p(out)),
           "patchify_bwd")
    return out


# ---------------------------------------------------------------- fastba
def reproject(poses, patches, intrinsics, ii, jj, kk):
    """cuda_ba.reproject (ba_cuda.cu:379-429, 585-616) -> [1, E, 2, P, P]."""
    poses = _f32(poses).reshape(-1, 7)
    P = patches.shape[-1]
    patches = _f32(patches).reshape(-1, 3, P, P)
    intr = _f32(intrinsics).reshape(-1, 4)
    ii, jj, kk = _i64(ii), _i64(jj), _i64(kk)
    E = ii.shape[0]
    out = np.empty((E, 2, P, P), np.float32)
    _check(lib().orc_reproject(_p(poses), _p(patches), _p(intr), _p(ii), _p(jj), _p(kk), E, P,
                               _p(out)), "reproject")
    return out.reshape(1, E, 2, P, P)


def neighbors(ii, jj):
    """cuda_ba.neighbors (ba.cpp:59-97)."""
    ii, jj = _i64(ii), _i64(jj)
    E = ii.shape[0]
    ix = np.empty(E, np.int64)
    jx = np.empty(E, np.int64)
    _check(lib().orc_neighbors(_p(ii), _p(jj), E, _p(ix), _p(jx)), "neighbors")
    return ix, jx


def ba(poses, patches, intrinsics, target, weight, lmbda, ii, jj, kk, t0, t1, iterations,
       diagnostics=False):
    """cuda_ba.forward semantics (ba_cuda.cu:433-582).  Returns updated copies
    (poses, patches) and, with diagnostics=True, a dict with the last
    iteration's dX [N,6], dZ [M_u], damped S, y and the Cholesky status."""
    pshape, kshape = np.shape(poses), np.shape(patches)
    P = kshape[-1]
    poses = _f32(poses).reshape(-1, 7).copy()
    patches = _f32(patches).reshape(-1, 3, P, P).copy()
    intr = _f32(intrinsics).reshape(-1, 4)
    target = _f32(target).reshape(-1, 2)
    weight = _f32(weight).reshape(-1, 2)
    ii, jj, kk = _i64(ii), _i64(jj), _i64(kk)
    E = ii.shape[0]
    N = max(t1 - t0, 0)
    Mu = len(np.unique(kk))
    dX = np.zeros(6 * N + 1, np.float64)
    dZ = np.zeros(Mu + 1, np.float64)
    S = np.zeros(36 * N * N + 1, np.float64)
    y = np.zeros(6 * N + 1, np.float64)
    rc = lib().orc_ba(_p(poses), _p(patches), _p(intr), _p(target), _p(weight),
                      ctypes.c_float(float(np.asarray(lmbda).reshape(-1)[0])), _p(ii), _p(jj), _p(kk),
                      E, P, int(t0), int(t1), int(iterations), _p(dX), _p(dZ), _p(S), _p(y))
    _check(rc, "ba")
    out = (poses.reshape(pshape), patches.reshape(kshape))
    if diagnostics:
        return out + ({"dX": dX[:6 * N].reshape(N, 6), "dZ": dZ[:Mu],
                       "S": S[:36 * N * N].reshape(6 * N, 6 * N), "y": y[:6 * N], "status": rc},)
    return out


# ---------------------------------------------------------------- lietorch
OPS = {"exp": 0, "log": 1, "inv": 2, "mul": 3, "adj": 4, "adjT": 5, "act": 6, "act4": 7,
       "matrix": 8, "projector": 9, "Jinv": 10}
GROUP_DIMS = {1: (3, 4), 3: (6, 7)}  # group id -> (manifold K, embedding N)


def lie_fwd(group, op, x, y=None):
    """Forward lietorch op on flattened [n, dim] float64 arrays (so3.h / se3.h)."""
    K, N = GROUP_DIMS[group]
    x = _f64(x)
    n = x.shape[0]
    outdim = {"exp": N, "log": K, "inv": N, "mul": N, "adj": K, "adjT": K, "act": 3, "act4": 4,
              "matrix": 16, "projector": N * N, "Jinv": K}[op]
    out = np.empty((n, outdim), np.float64)
    yy = _f64(y) if y is not None else np.zeros(1)
    _check(lib().orc_lie_fwd(group, OPS[op], n, _p(x), _p(yy), _p(out)), "lie_fwd")
    return out


def lie_bwd(group, op, grad, x, y=None):
    """Backward lietorch op; returns tuple of grads like lietorch_backends.*_backward."""
    K, N = GROUP_DIMS[group]
    grad, x = _f64(grad), _f64(x)
    n = x.shape[0]
    yy = _f64(y) if y is not None else np.zeros(1)
    if op == "exp":
        o0 = np.empty((n, K)); o1 = np.zeros(1)
    elif op in ("log", "inv"):
        o0 = np.empty((n, N)); o1 = np.zeros(1)
    elif op == "mul":
        o0 = np.empty((n, N)); o1 = np.empty((n, N))
    elif op in ("adj", "adjT"):
        o0 = np.empty((n, N)); o1 = np.empty((n, K))
    elif op == "act":
        o0 = np.empty((n, N)); o1 = np.empty((n, 3))
    elif op == "act4":
        o0 = np.empty((n, N)); o1 = np.empty((n, 4))
    else:
        raise ValueError(op)
    _check(lib().orc_lie_bwd(group, OPS[op], n, _p(grad), _p(x), _p(yy), _p(o0), _p(o1)), "lie_bwd")
    if op in ("exp", "log", "inv"):
        return (o0,)
    return (o0, o1)


def ba_shard(phase, poses, patches, intrinsics, target, weight, lmbda, ii, jj, kk, t0, t1, PPF,
             own_lo, own_hi, S=None, y=None):
    """Edge-sharded BA step of the C oracle (ba_core in dpvo_oracle.c), test
    infrastructure for the multi-rank driver.  phase 1: returns this rank's
    undamped (S [6N, 6N], y [6N]) over patches with own_lo <= kk // PPF <
    own_hi.  phase 2: applies one step from the GLOBAL (S, y) in place on the
    given poses / patches (numpy float32 arrays, modified) and returns them."""
    P = np.shape(patches)[-1]
    N = max(t1 - t0, 0)
    ii, jj, kk = _i64(ii), _i64(jj), _i64(kk)
    E = ii.shape[0]
    if phase == 1:
        poses, patches = _f32(poses).reshape(-1, 7), _f32(patches).reshape(-1, 3, P, P)
        S = np.zeros(36 * N * N + 1, np.float64)
        y = np.zeros(6 * N + 1, np.float64)
    else:
        assert poses.dtype == np.float32 and patches.dtype == np.float32
        assert poses.flags.c_contiguous and patches.flags.c_contiguous
        S = np.concatenate([_f64(S).reshape(-1), [0.0]])
        y = np.concatenate([_f64(y).reshape(-1), [0.0]])
    rc = lib().orc_ba_shard(_p(poses), _p(patches), _p(_f32(intrinsics).reshape(-1, 4)),
                            _p(_f32(target).reshape(-1, 2)), _p(_f32(weight).reshape(-1, 2)),
                            ctypes.c_float(float(np.asarray(lmbda).reshape(-1)[0])), _p(ii), _p(jj),
                            _p(kk), E, P, int(t0), int(t1), int(PPF), int(own_lo), int(own_hi),
                            int(phase), _p(S), _p(y))
    _check(rc, "ba_shard")
    if phase == 1:
        return S[:36 * N * N].reshape(6 * N, 6 * N), y[:6 * N]
    return poses, patches


def solve_system(J_Ginv_i, J_Ginv_j, ii, jj, res, ep, lm, freen):
    """cuda_ba.solve_system (dpvo/fastba/ba.cpp:120-180), restated in numpy.

    J [7r, 7n] from the per-edge blocks (ba.cpp:141-158), b = -J^T res and
    A = J^T J in fp64 (160-163), diag(A) += diag(A)*lm, += ep (164-165), with
    ep/lm rounded to fp32 as the pybind signature does; SPD solve of the
    top-left freen*7 block, zero elsewhere (103-118); delta cast to fp32.
    Parity unpinned: the reference needs Eigen (absent here) and its tests
    hold no fixture for this op, so this restatement is the only anchor.
    Poses with no edge get ep on the diagonal here; Eigen's sparse
    ``diagonal()`` has no entry there (reference behaviour undefined)."""
    Ji = np.asarray(J_Ginv_i, np.float32).astype(np.float64)
    Jj = np.asarray(J_Ginv_j, np.float32).astype(np.float64)
    ii = np.asarray(ii, np.int64)
    jj = np.asarray(jj, np.int64)
    v = np.asarray(res, np.float32).reshape(-1).astype(np.float64)
    r = len(ii)
    if np.any(ii == jj):
        raise ValueError("edge with ii == jj (ba.cpp:150-151 exits)")
    n = int(max(ii.max(), jj.max())) + 1
    J = np.zeros((7 * r, 7 * n))
    for x in range(r):
        J[7 * x:7 * x + 7, 7 * ii[x]:7 * ii[x] + 7] = Ji[x]
        J[7 * x:7 * x + 7, 7 * jj[x]:7 * jj[x] + 7] = Jj[x]
    b = -(J.T @ v)
    A = J.T @ J
    d = np.diag(A).copy()
    A[np.diag_indices_from(A)] = (d + d * float(np.float32(lm))) + float(np.float32(ep))
    f = freen * 7
    if f < 0 or f > 7 * n:
        f = 7 * n
    delta = np.zeros(7 * n)
    if f > 0:
        L = np.linalg.cholesky(A[:f, :f])
        y = np.linalg.solve(L, b[:f])
        delta[:f] = np.linalg.solve(L.T, y)
    return delta.astype(np.float32).reshape(n, 7)
