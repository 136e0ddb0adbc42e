"""Seeded synthetic patch graphs and feature pyramids (SURVEY 8d recipe).

Used by bench.py and the tests; everything is built on the host with a
seeded torch.Generator and then copied, so every rank / run sees the same
graph for the same seed.

cfg1: F=8 frames x M=32 patches, 256 edges.   cfg2: F=12 x 96, 2048 edges.
cfg4: F=1024 x 96, ~131k edges incl. loop blocks (make_graph_large).
Poses Exp(xi_f), xi_f = [0, 0, 0.05 f, 0, 0, 0] + 0.01 N(0, I6); patch centres
U([4,155] x [4,115]) at 1/4 resolution 160x120, inverse depth U(0.2, 1.2);
edges: one per patch plus random extra ones with |j - i| <= 5, sorted by
(kk, jj); target = reprojected centre + N(0, 0.5^2); weight U(0, 1).
"""
from __future__ import annotations

import math
from dataclasses import dataclass

import numpy as np
import torch

CONFIGS = {
    "cfg1": dict(F=8, M=32, E=256),
    "cfg2": dict(F=12, M=96, E=2048),
}


def se3_exp(xi: np.ndarray) -> np.ndarray:
    """Closed-form SE3 exponential, tangent (tau, phi) -> (t, q_xyzw), float64."""
    xi = np.asarray(xi, np.float64).reshape(-1, 6)
    out = np.zeros((xi.shape[0], 7))
    for n, (tau, phi) in enumerate(zip(xi[:, :3], xi[:, 3:])):
        th = float(np.linalg.norm(phi))
        K = np.array([[0, -phi[2], phi[1]], [phi[2], 0, -phi[0]], [-phi[1], phi[0], 0]])
        if th < 1e-8:
            V = np.eye(3) + 0.5 * K
            q = np.array([0.5 * phi[0], 0.5 * phi[1], 0.5 * phi[2], 1.0])
        else:
            V = np.eye(3) + (1 - math.cos(th)) / th**2 * K + (th - math.sin(th)) / th**3 * K @ K
            s = math.sin(0.5 * th) / th
            q = np.array([s * phi[0], s * phi[1], s * phi[2], math.cos(0.5 * th)])
        out[n, :3] = V @ tau
        out[n, 3:] = q / np.linalg.norm(q)
    return out


def _qrot(q, p):
    x, y, z, w = q
    v = np.array([x, y, z])
    uv = 2 * np.cross(v, p)
    return p + w * uv + np.cross(v, uv)


def _qrot_n(q, p):  # batched quaternion rotation, q [n, 4] (x, y, z, w), p [n, 3]
    v, w = q[:, :3], q[:, 3:4]
    uv = 2 * np.cross(v, p)
    return p + w * uv + np.cross(v, uv)


def reproject_centres(poses, patches, intr, ii, jj, kk):
    """Centre-pixel reprojection (fp64, host) used only to place targets:
    G_ij = P_j P_i^-1 applied to the homogeneous centre point (X, d)."""
    fx, fy, cx, cy = intr
    poses = np.asarray(poses, np.float64)
    Pi, Pj = poses[np.asarray(ii)], poses[np.asarray(jj)]
    c = np.asarray(patches, np.float64)[np.asarray(kk), :, 1, 1]
    X = np.stack([(c[:, 0] - cx) / fx, (c[:, 1] - cy) / fy, np.ones(len(c))], -1)
    d = c[:, 2:3]
    qi_inv = np.concatenate([-Pi[:, 3:6], Pi[:, 6:7]], -1)
    Xw = _qrot_n(qi_inv, X - Pi[:, :3] * d)
    Xj = _qrot_n(Pj[:, 3:], Xw) + Pj[:, :3] * d
    return np.stack([fx * Xj[:, 0] / Xj[:, 2] + cx, fy * Xj[:, 1] / Xj[:, 2] + cy], -1)


@dataclass
class Graph:
    poses: torch.Tensor       # [num_poses, 7] f32
    patches: torch.Tensor     # [num_patches, 3, p, p] f32
    intrinsics: torch.Tensor  # [num_poses, 4] f32
    ii: torch.Tensor          # [E] int64 source frame (= kk // M)
    jj: torch.Tensor          # [E] int64 target frame
    kk: torch.Tensor          # [E] int64 patch
    target: torch.Tensor      # [E, 2] f32
    weight: torch.Tensor      # [E, 2] f32
    F: int
    M: int

    def to(self, device):
        kw = {k: getattr(self, k).to(device) for k in
              ("poses", "patches", "intrinsics", "ii", "jj", "kk", "target", "weight")}
        return Graph(F=self.F, M=self.M, **kw)

    @property
    def E(self):
        return int(self.ii.numel())


def make_graph(F, M, E, seed=0, H=120, W=160, p=3, span=5, noise=0.5, lateral=0.0, wmin=0.0,
               num_poses=None, num_patches=None, intr=(80.0, 80.0, 80.0, 60.0)) -> Graph:
    g = torch.Generator().manual_seed(seed)
    xi = torch.zeros(F, 6, dtype=torch.float64)
    xi[:, 2] = 0.05 * torch.arange(F, dtype=torch.float64)
    xi[:, 0] = lateral * torch.arange(F, dtype=torch.float64)
    xi += 0.01 * torch.randn(F, 6, generator=g, dtype=torch.float64)
    xi[0] = 0
    poses_np = se3_exp(xi.numpy())
    cxy = torch.stack([torch.rand(F * M, generator=g) * (W - 9) + 4,
                       torch.rand(F * M, generator=g) * (H - 9) + 4], -1).floor()
    d = torch.rand(F * M, generator=g) + 0.2
    off = torch.arange(p, dtype=torch.float32) - p // 2
    patches = torch.zeros(F * M, 3, p, p)
    patches[:, 0] = cxy[:, 0].view(-1, 1, 1) + off.view(1, 1, p)
    patches[:, 1] = cxy[:, 1].view(-1, 1, 1) + off.view(1, p, 1)
    patches[:, 2] = d.view(-1, 1, 1)

    # candidate edges (k, j) with |j - i| <= span; one per patch + random extras
    k_all = torch.arange(F * M)
    i_all = k_all // M
    lo = (i_all - span).clamp(min=0)
    hi = (i_all + span + 1).clamp(max=F)
    cnt = hi - lo
    first_j = lo + (torch.rand(F * M, generator=g) * cnt).long().clamp(max=cnt - 1)
    cand_k = torch.repeat_interleave(k_all, cnt)
    cand_j = torch.cat([torch.arange(a, b) for a, b in zip(lo.tolist(), hi.tolist())])
    taken = cand_j == first_j[cand_k]
    rest = (~taken).nonzero().view(-1)
    n_extra = max(E - F * M, 0)
    extra = rest[torch.randperm(len(rest), generator=g)[:n_extra]]
    kk = torch.cat([k_all, cand_k[extra]])[:E]
    jj = torch.cat([first_j, cand_j[extra]])[:E]
    order = torch.argsort(kk * (F + 1) + jj)
    kk, jj = kk[order].long(), jj[order].long()
    ii = kk // M

    num_poses = num_poses or F
    num_patches = num_patches or F * M
    poses = torch.zeros(num_poses, 7)
    poses[:, 6] = 1.0
    poses[:F] = torch.from_numpy(poses_np).float()
    P = torch.zeros(num_patches, 3, p, p)
    P[:, 2] = 1.0
    P[: F * M] = patches
    intrinsics = torch.tensor(intr).view(1, 4).repeat(num_poses, 1)
    ctr = reproject_centres(poses[:F].double().numpy(), patches.double().numpy(), intr,
                            ii.numpy(), jj.numpy(), kk.numpy())
    target = torch.from_numpy(ctr).float() + noise * torch.randn(len(ii), 2, generator=g)
    weight = wmin + (1 - wmin) * torch.rand(len(ii), 2, generator=g)
    return Graph(poses, P, intrinsics, ii, jj, kk, target, weight, F, M)


def make_dpvo_window(n=22, M=96, lifetime=13, seed=0, H=120, W=160, p=3, noise=0.5,
                     intr=(80.0, 80.0, 80.0, 60.0)) -> Graph:
    """A local-BA window with DPVO's own edge pattern (dpvo/dpvo.py:838-903):
    when frame f is added its M patches get edges to frames
    [max(f - lifetime + 1, 0), f] (__edges_back) and every patch of frames
    [f - lifetime + 1, f) gets an edge to frame f (__edges_forw), so a patch
    of frame g ends up with edges to frames g-lifetime+1 .. g+lifetime-1
    inside [0, n).  Edges are in creation order (not grouped by patch), as
    DPVO's PatchGraph appends them.  E = 394 M for the defaults (n=22,
    lifetime=13): M = 10 / 18 / 25 -> ~4k / 7k / 10k edges.  Use with
    t0 = n - OPTIMIZATION_WINDOW (10), t1 = n (dpvo.py:818-824)."""
    g = torch.Generator().manual_seed(seed)
    xi = torch.zeros(n, 6, dtype=torch.float64)
    xi[:, 2] = 0.05 * torch.arange(n, dtype=torch.float64)
    xi += 0.01 * torch.randn(n, 6, generator=g, dtype=torch.float64)
    xi[0] = 0
    poses_np = se3_exp(xi.numpy())
    cxy = torch.stack([torch.rand(n * M, generator=g) * (W - 9) + 4,
                       torch.rand(n * M, generator=g) * (H - 9) + 4], -1).floor()
    d = torch.rand(n * M, generator=g) * 0.8 + 0.3
    off = torch.arange(p, dtype=torch.float32) - p // 2
    patches = torch.zeros(n * M, 3, p, p)
    patches[:, 0] = cxy[:, 0].view(-1, 1, 1) + off.view(1, 1, p)
    patches[:, 1] = cxy[:, 1].view(-1, 1, 1) + off.view(1, p, 1)
    patches[:, 2] = d.view(-1, 1, 1)
    kk, jj = [], []
    for f in range(n):  # frame f added: forward edges, then backward edges
        lo = max(f - lifetime + 1, 0)
        if f > 0:
            k = torch.arange(lo * M, f * M)
            kk.append(k)
            jj.append(torch.full_like(k, f))
        k = torch.arange(f * M, (f + 1) * M).repeat_interleave(f + 1 - lo)
        kk.append(k)
        jj.append(torch.arange(lo, f + 1).repeat(M))
    kk = torch.cat(kk).long()
    jj = torch.cat(jj).long()
    ii = kk // M
    poses = torch.from_numpy(poses_np).float()
    intrinsics = torch.tensor(intr).view(1, 4).repeat(n, 1)
    ctr = reproject_centres(poses.double().numpy(), patches.double().numpy(), intr, ii.numpy(),
                            jj.numpy(), kk.numpy())
    target = torch.from_numpy(ctr).float() + noise * torch.randn(len(ii), 2, generator=g)
    weight = torch.rand(len(ii), 2, generator=g)
    return Graph(poses, patches, intrinsics, ii, jj, kk, target, weight, n, M)


LARGE_CONFIGS = {
    # BASELINE cfg4: 1024 frames x 96 patches, ~131k edges
    "cfg4": dict(F=1024, M=96, n_random=32000, n_loops=10),
    # same recipe at oracle-checkable sizes (tests)
    "cfg4s": dict(F=96, M=12, n_random=600, n_loops=3),
    "cfg4m": dict(F=200, M=24, n_random=3000, n_loops=6),
}


def make_graph_large(F, M, n_random, n_loops, seed=0, H=120, W=160, p=3, span=6, period=64,
                     radius=0.25, noise=0.5, intr=(80.0, 80.0, 80.0, 60.0)) -> Graph:
    """SURVEY 8d cfg4 recipe: every patch gets an edge to frame i+1, plus
    ``n_random`` random edges with |j - i| <= span, plus ``n_loops`` loop blocks
    (all M slots of frame i observed from frame i + k*period, k >= 1).  The
    trajectory is periodic (a small loop every ``period`` frames, deviation
    from the reference recipe's straight line) so that loop edges reproject
    in front of the camera.  Edges are left in a shuffled order (the solver
    must group them itself, as after DPVO's append/remove bookkeeping)."""
    g = torch.Generator().manual_seed(seed)
    f = torch.arange(F, dtype=torch.float64)
    ang = 2 * math.pi * f / period
    xi = torch.zeros(F, 6, dtype=torch.float64)
    xi[:, 0] = radius * torch.sin(ang)
    xi[:, 2] = radius * (1 - torch.cos(ang))
    xi[:, 4] = 0.05 * torch.sin(ang)
    xi += 0.005 * torch.randn(F, 6, generator=g, dtype=torch.float64)
    xi[0] = 0
    poses_np = se3_exp(xi.numpy())
    cxy = torch.stack([torch.rand(F * M, generator=g) * (W - 9) + 4,
                       torch.rand(F * M, generator=g) * (H - 9) + 4], -1).floor()
    d = torch.rand(F * M, generator=g) * 0.6 + 0.3
    off = torch.arange(p, dtype=torch.float32) - p // 2
    patches = torch.zeros(F * M, 3, p, p)
    patches[:, 0] = cxy[:, 0].view(-1, 1, 1) + off.view(1, 1, p)
    patches[:, 1] = cxy[:, 1].view(-1, 1, 1) + off.view(1, p, 1)
    patches[:, 2] = d.view(-1, 1, 1)

    k_next = torch.arange((F - 1) * M)
    j_next = k_next // M + 1
    kr = torch.randint(0, F * M, (n_random,), generator=g)
    ir = kr // M
    jr = (ir + torch.randint(-span, span + 1, (n_random,), generator=g)).clamp(0, F - 1)
    kl, jl = [], []
    starts = torch.randperm(max(F - period, 1), generator=g)[:n_loops]
    for i0 in starts.tolist():
        j0 = i0 + period * (1 + (i0 % 2)) if i0 + 2 * period < F else i0 + period
        j0 = min(j0, F - 1)
        kl.append(torch.arange(i0 * M, (i0 + 1) * M))
        jl.append(torch.full((M,), j0, dtype=torch.long))
    kk = torch.cat([k_next, kr] + kl)
    jj = torch.cat([j_next, jr] + jl)
    perm = torch.randperm(len(kk), generator=g)
    kk, jj = kk[perm].long(), jj[perm].long()
    ii = kk // M
    poses = torch.from_numpy(poses_np).float()
    intrinsics = torch.tensor(intr).view(1, 4).repeat(F, 1)
    ctr = reproject_centres(poses.double().numpy(), patches.double().numpy(), intr, ii.numpy(),
                            jj.numpy(), kk.numpy())
    target = torch.from_numpy(ctr).float() + noise * torch.randn(len(ii), 2, generator=g)
    weight = torch.rand(len(ii), 2, generator=g)
    return Graph(poses, patches, intrinsics, ii, jj, kk, target, weight, F, M)


def make_config(name, seed=0, **kw) -> Graph:
    if name in LARGE_CONFIGS:
        c = dict(LARGE_CONFIGS[name])
        c.update(kw)
        return make_graph_large(seed=seed, **c)
    c = dict(CONFIGS[name])
    c.update(kw)
    return make_graph(seed=seed, **c)


def make_features(mem=36, C=128, H=120, W=160, levels=(1, 4), seed=0, device="cuda",
                  dtype=torch.float32):
    """fmap level 1 = 0.25 N(0,1) [1, mem, C, H, W]; level l = avg_pool(level 1, l)."""
    g = torch.Generator(device=device).manual_seed(seed)
    f1 = 0.25 * torch.randn(1, mem, C, H, W, generator=g, device=device, dtype=torch.float32)
    pyr = []
    for s in levels:
        if s == 1:
            pyr.append(f1)
        else:
            pyr.append(torch.nn.functional.avg_pool2d(f1[0], s, s).unsqueeze(0))
    return [p.to(dtype).contiguous() for p in pyr]


def channels_last(level):
    """[B, N, C, H, W] -> the same tensor in channels-last memory
    ([B, N, H, W, C] storage; what cuda_corr.forward_levels' matrix-core path
    reads)."""
    return level.permute(0, 1, 3, 4, 2).contiguous().permute(0, 1, 4, 2, 3)
