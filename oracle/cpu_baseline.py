"""TEST / BASELINE INFRASTRUCTURE ONLY -- a CPU restatement of the reference's
CPU / PyTorch fallback path for one DPVO update iteration, timed by bench.py's
`cpu_baseline` leg (rank 0, N=1) on the GPU box's host cores.

Restated op sequence (cuteboyqq/DPVO):
  * correlation, per pyramid level: corr_torch_forward
    (dpvo/altcorr/correlation_kernel.py:461-548) -- chunks of edges, whole-frame
    gather fmap2[:, jj_chunk], grid_sample of the (2R+2)^2 x p^2 integer
    window positions, channel dot with the gathered gmap patch, then the
    4-tap bilinear + permute;
  * BA: dpvo/ba.py BA (88-297) / python_ba_wrapper (299-415) -- projective
    transform with Jacobians, dense scatter-sum assembly of B, E, C, v, w,
    Schur complement, Cholesky solve, retractions -- per iteration.
The reference Python itself cannot travel to the GPU box, so this is the
"port" baseline; bench.py reports it as kind="port" with the thread count.
"""
from __future__ import annotations

import time

import torch
import torch.nn.functional as F


# ------------------------------------------------------------------ correlation
def corr_grid_sample(fmap1, fmap2, coords, ii, jj, radius, chunk=64):
    B, M, _, H, W = coords.shape
    C = fmap1.size(2)
    H2, W2 = fmap2.size(3), fmap2.size(4)
    D = 2 * radius + 2
    raw = torch.empty(B, M, D, D, H, W, dtype=fmap1.dtype)
    offs = torch.arange(-radius, radius + 2, dtype=fmap1.dtype)
    oy, ox = torch.meshgrid(offs, offs, indexing="ij")
    ox, oy = ox.view(1, 1, D, D, 1, 1), oy.view(1, 1, D, D, 1, 1)
    for m0 in range(0, M, chunk):
        m1 = min(m0 + chunk, M)
        mc = m1 - m0
        f1 = fmap1[:, ii[m0:m1]]
        f2 = fmap2[:, jj[m0:m1]].reshape(B * mc, C, H2, W2)
        gx = coords[:, m0:m1, 0].floor().unsqueeze(2).unsqueeze(2) + ox
        gy = coords[:, m0:m1, 1].floor().unsqueeze(2).unsqueeze(2) + oy
        grid = torch.stack([2 * gx / (W2 - 1) - 1, 2 * gy / (H2 - 1) - 1], -1)
        s = F.grid_sample(f2, grid.view(B * mc, D * D * H * W, 1, 2), mode="bilinear",
                          align_corners=True).view(B, mc, C, D, D, H, W)
        raw[:, m0:m1] = (f1.unsqueeze(3).unsqueeze(3) * s).sum(dim=2)
    dx = (coords[:, :, 0] - coords[:, :, 0].floor()).unsqueeze(2).unsqueeze(2)
    dy = (coords[:, :, 1] - coords[:, :, 1].floor()).unsqueeze(2).unsqueeze(2)
    d = D - 1
    out = ((1 - dx) * (1 - dy) * raw[:, :, :d, :d] + dx * (1 - dy) * raw[:, :, :d, 1:]
           + (1 - dx) * dy * raw[:, :, 1:, :d] + dx * dy * raw[:, :, 1:, 1:])
    return out.permute(0, 1, 3, 2, 4, 5)


# ------------------------------------------------------------------ SE3 (torch)
def _qmul(a, b):
    ax, ay, az, aw = a.unbind(-1)
    bx, by, bz, bw = b.unbind(-1)
    return torch.stack([aw * bx + ax * bw + ay * bz - az * by, aw * by + ay * bw + az * bx - ax * bz,
                        aw * bz + az * bw + ax * by - ay * bx, aw * bw - ax * bx - ay * by - az * bz], -1)


def _qrot(q, p):
    v, w = q[..., :3], q[..., 3:]
    uv = 2 * torch.cross(v.expand_as(p), p, dim=-1)
    return p + w * uv + torch.cross(v.expand_as(uv), uv, dim=-1)


def _inv(P):
    qi = torch.cat([-P[..., 3:6], P[..., 6:]], -1)
    return torch.cat([-_qrot(qi, P[..., :3]), qi], -1)


def _mul(A, B):
    return torch.cat([A[..., :3] + _qrot(A[..., 3:], B[..., :3]), _qmul(A[..., 3:], B[..., 3:])], -1)


def _hat(v):
    o = torch.zeros_like(v[..., 0])
    x, y, z = v.unbind(-1)
    return torch.stack([o, -z, y, z, o, -x, -y, x, o], -1).view(v.shape[:-1] + (3, 3))


def _rotm(q):
    e = torch.eye(3, dtype=q.dtype).expand(q.shape[:-1] + (3, 3))
    return _qrot(q.unsqueeze(-2), e.transpose(-1, -2)).transpose(-1, -2)


def _adjT(G, a):
    R = _rotm(G[..., 3:])
    tR = _hat(G[..., :3]) @ R
    A = torch.zeros(G.shape[:-1] + (6, 6), dtype=G.dtype)
    A[..., :3, :3] = R
    A[..., :3, 3:] = tR
    A[..., 3:, 3:] = R
    return (a.unsqueeze(-2) @ A).squeeze(-2)


def _exp(xi):
    tau, phi = xi[..., :3], xi[..., 3:]
    th = phi.norm(dim=-1, keepdim=True).clamp(min=1e-12)
    K = _hat(phi)
    I = torch.eye(3, dtype=xi.dtype)
    a = ((1 - th.cos()) / th**2).unsqueeze(-1)
    b = ((th - th.sin()) / th**3).unsqueeze(-1)
    V = I + a * K + b * (K @ K)
    q = torch.cat([(0.5 * th).sin() / th * phi, (0.5 * th).cos()], -1)
    return torch.cat([(V @ tau.unsqueeze(-1)).squeeze(-1), q], -1)


# ------------------------------------------------------------------ BA (ba.py)
def ba_step(poses, patches, intr, target, weight, lmbda, ii, jj, kk, t0, ep=100.0, bounds=None):
    """One dpvo/ba.py BA call (88-297), dense Schur, B = 1.  ``bounds``
    (xmin, ymin, xmax, ymax) of the projected patch centre (ba.py:165-171);
    None -> python_ba_wrapper's default [0, 0, W-1, H-1] with W = 2 cx,
    H = 2 cy (ba.py:355-370).  Works in the dtype of the inputs (the pinning
    test runs it in float64 against the reference's own fp64 run)."""
    n = int(max(ii.max(), jj.max())) + 1
    fx, fy, cx, cy = intr.unbind(-1)
    X0 = torch.stack([(patches[kk, 0] - cx) / fx, (patches[kk, 1] - cy) / fy,
                      torch.ones_like(patches[kk, 2]), patches[kk, 2]], -1)  # [E,p,p,4]
    Gij = _mul(poses[jj], _inv(poses[ii]))
    X1 = torch.cat([_qrot(Gij[:, None, None, 3:], X0[..., :3]) + Gij[:, None, None, :3] * X0[..., 3:],
                    X0[..., 3:]], -1)
    d = 1.0 / X1[..., 2].clamp(min=0.1)
    coords = torch.stack([fx * d * X1[..., 0] + cx, fy * d * X1[..., 1] + cy], -1)
    p = coords.shape[1]
    X, Y, Z, Hh = X1[:, p // 2, p // 2].unbind(-1)
    dd = torch.where(Z.abs() > 0.2, 1.0 / Z, torch.zeros_like(Z))
    o = torch.zeros_like(Hh)
    Ja = torch.stack([Hh, o, o, o, Z, -Y, o, Hh, o, -Z, o, X, o, o, Hh, Y, -X, o,
                      o, o, o, o, o, o], -1).view(-1, 4, 6)
    Jp = torch.stack([fx * dd, o, -fx * X * dd * dd, o, o, fy * dd, -fy * Y * dd * dd, o],
                     -1).view(-1, 2, 4)
    Jj = Jp @ Ja
    Ji = -_adjT(Gij[:, None].expand(-1, 2, -1), Jj)
    Gm = torch.cat([Gij[:, :3], torch.ones_like(Gij[:, :1])], -1).unsqueeze(-1)
    Jz = Jp @ Gm
    r = target - coords[:, p // 2, p // 2]
    if bounds is None:
        bounds = (0.0, 0.0, float(2 * cx) - 1.0, float(2 * cy) - 1.0)
    cc = coords[:, p // 2, p // 2]
    inb = (cc[:, 0] > bounds[0]) & (cc[:, 1] > bounds[1]) & (cc[:, 0] < bounds[2]) & \
        (cc[:, 1] < bounds[3])
    v = ((r.norm(dim=-1) < 250) & (Z > 0.2) & inb).to(poses.dtype)
    r = (v[:, None] * r).unsqueeze(-1)
    w = (v[:, None] * weight).unsqueeze(-1)
    wJiT, wJjT, wJzT = (w * Ji).transpose(1, 2), (w * Jj).transpose(1, 2), (w * Jz).transpose(1, 2)
    nf = n - t0
    iif, jjf = ii - t0, jj - t0
    kx, ku = torch.unique(kk, return_inverse=True, sorted=True)
    m = len(kx)
    dt = poses.dtype
    Bm = torch.zeros(nf * nf, 6, 6, dtype=dt)
    Em = torch.zeros(nf * m, 6, dtype=dt)
    vv = torch.zeros(nf, 6, dtype=dt)

    def add_mat(buf, blocks, a, b, nb):
        ok = (a >= 0) & (b >= 0)
        buf.index_add_(0, (a * nb + b)[ok], blocks[ok])

    add_mat(Bm, wJiT @ Ji, iif, iif, nf)
    add_mat(Bm, wJiT @ Jj, iif, jjf, nf)
    add_mat(Bm, wJjT @ Ji, jjf, iif, nf)
    add_mat(Bm, wJjT @ Jj, jjf, jjf, nf)
    add_mat(Em, (wJiT @ Jz).squeeze(-1), iif, ku, m)
    add_mat(Em, (wJjT @ Jz).squeeze(-1), jjf, ku, m)
    C = torch.zeros(m, dtype=dt).index_add_(0, ku, (wJzT @ Jz).view(-1))
    okv = iif >= 0
    vv.index_add_(0, iif[okv], (wJiT @ r).squeeze(-1)[okv])
    okv = jjf >= 0
    vv.index_add_(0, jjf[okv], (wJjT @ r).squeeze(-1)[okv])
    wv = torch.zeros(m, dtype=dt).index_add_(0, ku, (wJzT @ r).view(-1))
    Q = 1.0 / (C + lmbda)
    Bd = Bm.view(nf, nf, 6, 6).permute(0, 2, 1, 3).reshape(6 * nf, 6 * nf)
    Ed = Em.view(nf, m, 6).permute(0, 2, 1).reshape(6 * nf, m)
    S = Bd - (Ed * Q) @ Ed.T
    y = vv.view(-1) - (Ed * Q) @ wv
    S = S + (ep + 1e-4 * S) * torch.eye(6 * nf, dtype=dt)
    L, info = torch.linalg.cholesky_ex(S)
    dX = (torch.cholesky_solve(y.unsqueeze(-1), L).view(nf, 6) if not info.any()
          else torch.zeros(nf, 6, dtype=dt))
    dZ = Q * (wv - Ed.T @ dX.view(-1))
    patches = patches.clone()
    patches[kx, 2] = (patches[kx, 2] + dZ.view(-1, 1, 1)).clamp(1e-3, 10.0)
    poses = poses.clone()
    poses[t0:n] = _mul(_exp(dX), poses[t0:n])
    return poses, patches


def update_iteration(state, levels, iterations=2):
    """reproject (transform) + corr at every level + `iterations` BA calls."""
    G, gmap, pyr = state["G"], state["gmap"], state["pyr"]
    P = G.patches
    fx, fy, cx, cy = G.intrinsics[0].tolist()
    X0 = torch.stack([(P[G.kk, 0] - cx) / fx, (P[G.kk, 1] - cy) / fy, torch.ones_like(P[G.kk, 2]),
                      P[G.kk, 2]], -1)
    Gij = _mul(G.poses[G.jj], _inv(G.poses[G.ii]))
    X1 = _qrot(Gij[:, None, None, 3:], X0[..., :3]) + Gij[:, None, None, :3] * X0[..., 3:]
    d = 1.0 / X1[..., 2].clamp(min=0.1)
    coords = torch.stack([fx * d * X1[..., 0] + cx, fy * d * X1[..., 1] + cy], 1).unsqueeze(0)
    outs = [corr_grid_sample(gmap, f, coords / s, G.kk, G.jj, 3) for f, s in zip(pyr, levels)]
    poses, patches = G.poses, G.patches
    for _ in range(iterations):
        poses, patches = ba_step(poses, patches, G.intrinsics[0], G.target, G.weight, 1e-4, G.ii,
                                 G.jj, G.kk, 1)
    return outs, poses, patches


def measure(G, levels=(1, 2, 4, 8), budget_s=15.0, threads=None, mem=None, C=128, iterations=2):
    """Time update iterations of the CPU port on a bounded sample (>= 1
    iteration, stop once `budget_s` is spent).  Returns (it/s, threads, n).
    ``iterations``: BA iterations per update (2 = fastba default; the fork's
    local call uses 1, dpvo.py:824)."""
    if threads:
        torch.set_num_threads(threads)
    g = torch.Generator().manual_seed(0)
    mem = mem or G.F
    f1 = 0.25 * torch.randn(1, mem, C, 120, 160, generator=g)
    pyr = [f1 if s == 1 else F.avg_pool2d(f1[0], s, s).unsqueeze(0) for s in levels]
    gmap = 0.25 * torch.randn(1, G.F * G.M, C, 3, 3, generator=g)
    state = {"G": G, "gmap": gmap, "pyr": pyr}
    t0 = time.perf_counter()
    n = 0
    while True:
        update_iteration(state, levels, iterations)
        n += 1
        el = time.perf_counter() - t0
        if el >= budget_s or (n >= 1 and el * (n + 1) / n > 2 * budget_s):
            break
    return n / el, torch.get_num_threads(), n
