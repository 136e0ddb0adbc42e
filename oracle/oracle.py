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


# ---------------------------------------------------------------- keyframe / edges_loop
def flow_mag(poses, patches, intrinsics, ii, jj, kk, beta=0.5, pixel=None):
    """projective_ops.flow_mag (projective_ops.py:120-130) in fp32 op by op
    (orc_flow_mag).  patches [N, 3, P, P]; pixel=(r, c) selects
    patches[..., r, c] (edges_loop, patchgraph.py:79) -> ([E], [E]) else
    ([E, P, P] flow, valid)."""
    poses = _f32(poses).reshape(-1, 7)
    P = np.shape(patches)[-1]
    patches = _f32(patches).reshape(-1, 3, P, P)
    intr = _f32(intrinsics).reshape(-1, 4)
    ii, jj, kk = _i64(ii), _i64(jj), _i64(kk)
    E = ii.shape[0]
    px0 = -1 if pixel is None else pixel[0] * P + pixel[1]
    npx = P * P if pixel is None else 1
    flow = np.zeros(E * npx, np.float32)
    val = np.zeros(E * npx, np.uint8)
    _check(lib().orc_flow_mag(_p(poses), _p(patches), _p(intr), P, _p(ii), _p(jj), _p(kk), E,
                              px0, ctypes.c_float(beta), _p(flow), _p(val)), "flow_mag")
    if pixel is None:
        return flow.reshape(E, P, P), val.reshape(E, P, P).astype(bool)
    return flow, val.astype(bool)


def _sum_f32(x):
    """fp32 result of a sum accumulated in double in index order."""
    return np.float32(np.sum(np.asarray(x, np.float64)))


def motionmag(st, i, j):
    """DPVO.motionmag (dpvo.py:586-599): mean flow_mag(beta 0.5) over the
    pixels of the active edges i -> j; torch's mean = fp32 sum * (1 / N)."""
    E = st["num_edges"]
    ii, jj, kk = st["ii"][:E], st["jj"][:E], st["kk"][:E]
    sel = (ii == i) & (jj == j)
    if not sel.any():
        return np.float32(0.0)
    fl, _ = flow_mag(st["poses"], st["patches"], st["intrinsics"], ii[sel], jj[sel], kk[sel], 0.5)
    return np.float32(_sum_f32(fl) * (np.float32(1.0) / np.float32(fl.size)))


def keyframe(st, M, keyframe_index=4, keyframe_thresh=12.5, rings=None):
    """DPVO.keyframe's frame drop (dpvo.py:601-673) on a numpy state dict
    (copied): n, m, num_edges, ii/jj/kk/net/weight/target [max_edges, ...],
    poses [N,7], patches [N*M,3,P,P], intrinsics [N,4], tstamps [N], plus any
    per-frame array named in `rings` {name: ring} (ring 0: row = frame).
    Returns (state, {"drop", "k", "mag", "delta"})."""
    st = {k: (v.copy() if isinstance(v, np.ndarray) else v) for k, v in st.items()}
    n = st["n"]
    i, j = n - keyframe_index - 1, n - keyframe_index + 1
    m0, m1 = motionmag(st, i, j), motionmag(st, j, i)
    info = {"drop": False, "k": n - keyframe_index, "mag": (m0, m1), "delta": None}
    if not ((float(m0) + float(m1)) / 2 < keyframe_thresh and i >= 0):
        return st, info
    k = n - keyframe_index
    info["drop"] = True
    info["delta"] = (int(st["tstamps"][k]), int(st["tstamps"][k - 1]),
                     se3_mul_inv(st["poses"][k], st["poses"][k - 1]))
    E = st["num_edges"]
    ii, jj = st["ii"][:E], st["jj"][:E]
    keep = ~((ii == k) | (jj == k))
    ne = int(keep.sum())
    for name in ("ii", "jj", "kk", "net", "weight", "target"):
        if name in st:
            st[name][:ne] = st[name][:E][keep]
    st["num_edges"] = ne
    ii, jj, kk = st["ii"][:ne], st["jj"][:ne], st["kk"][:ne]
    mi, mj = ii > k, jj > k
    kk[mi] -= M
    ii[mi] -= 1
    jj[mj] -= 1
    frames = {"poses": 0, "intrinsics": 0, "tstamps": 0}
    frames.update(rings or {})
    for name, ring in frames.items():
        a = st[name]
        for f in range(k, n - 1):
            src, dst = (f + 1, f) if not ring else ((f + 1) % ring, f % ring)
            a[dst] = a[src]
    pa = st["patches"].reshape(-1, M, *st["patches"].shape[1:])
    for f in range(k, n - 1):
        pa[f] = pa[f + 1]
    st["n"] = n - 1
    st["m"] = st["m"] - M
    return st, info


def se3_mul_inv(a, b):
    """lietorch SE3(a) * SE3(b).inv() in fp32 (se3.h:325-336), 7 floats."""
    out = np.zeros(7, np.float32)
    _check(lib().orc_se3_mul_inv(_p(_f32(a)), _p(_f32(b)), _p(out)), "se3_mul_inv")
    return out


def reduce_edges(flow, ii, jj, max_num_edges=1000, nms=1):
    """loop_closure/optim_utils.py:24-60.  Candidates in ascending flow order
    (ties by index: a stable argsort; numba's argsort is not stable, exact
    fp32 ties between distinct groups are the only case it could differ)."""
    es = []
    if len(ii) == 0:
        return np.zeros((0, 2), np.int64)
    Ni, Nj = int(ii.max()) + 1, int(jj.max()) + 1
    ignore = np.zeros((Ni, Nj), bool)
    for idx in np.argsort(flow, kind="stable"):
        if len(es) + 1 > max_num_edges:
            break
        i, j, mag = int(ii[idx]), int(jj[idx]), flow[idx]
        if j - i < 30 or mag >= 1000 or ignore[i, j]:
            continue
        es.append((i, j))
        for di in range(-nms, nms + 1):
            if 0 <= i + di < Ni:
                ignore[i + di, j] = True
    return np.asarray(es, np.int64).reshape(-1, 2)


def edges_loop(poses, patches, intrinsics, ix, n, M, removal_window=20, max_edge_age=1000,
               global_opt_freq=15, keyframe_index=4, backend_thresh=64.0, max_num_edges=1000,
               nms=1):
    """PatchGraph.edges_loop (patchgraph.py:65-91) -> (kk, jj) int64.
    Group sums accumulate in double in patch order, then fp32 (the
    reference's torch sum is unordered fp32)."""
    l = n - removal_window
    if l <= 0:
        return np.zeros(0, np.int64), np.zeros(0, np.int64)
    jr = np.arange(n - global_opt_freq, n - keyframe_index)
    kr = np.arange(max(l - max_edge_age, 0) * M, l * M)
    jj, kk = np.meshgrid(jr, kr, indexing="ij")
    jj, kk = jj.reshape(-1), kk.reshape(-1)
    ix = np.asarray(ix, np.int64)
    ii = ix[kk]
    if len(kk) == 0:
        return np.zeros(0, np.int64), np.zeros(0, np.int64)
    fl, val = flow_mag(poses, patches, intrinsics, ii, jj, kk, 0.5, pixel=(1, 1))
    G = len(kk) // M
    fl, val = fl.reshape(G, M), val.reshape(G, M)
    s = np.array([_sum_f32(np.where(val[g], fl[g], 0.0)) for g in range(G)], np.float32)
    c = val.sum(1).astype(np.float32)
    fm = np.where(c > M * 0.75, s / np.maximum(c, np.float32(1)), np.float32(np.inf))
    fm = fm.astype(np.float32)
    mask = fm < backend_thresh
    es = reduce_edges(fm[mask], ii[::M][mask], jj[::M][mask], max_num_edges, nms)
    kk = (es[:, 0][:, None] * M + np.arange(M)[None]).reshape(-1)
    jj = np.repeat(es[:, 1], M)
    return kk.astype(np.int64), jj.astype(np.int64)
