"""DPVO.update() data flow on the MI355X ops at real shapes.

Reproduces, per frame, what dpvo/dpvo.py does around the update operator with
the default config (config/default.yaml: PATCHES_PER_FRAME 96,
PATCH_LIFETIME 13, REMOVAL_WINDOW 22, OPTIMIZATION_WINDOW 10; mem = pmem = 36):

  frame insertion   fmap -> channels-last pyramid ring, levels [1, 4]
                    (dpvo.py __call__; one launch: altcorr.insert_frame), gmap of
                    the new patches (altcorr.patchify)
  edges             __edges_forw / __edges_back (dpvo.py:838-903) appended on the
                    device (DevicePatchGraph.append_factors, dpvo.py:480-521)
  update()          reproject (+ A-CORR edge order) -> corr at levels [1, 4] with
                    kk % (M pmem), jj % mem (dpvo.py:456-465) -> [network] ->
                    target = coords[..., 1, 1] + delta (dpvo.py:805-806) ->
                    fastba.BA(t0 = n - OPTIMIZATION_WINDOW, t1 = n) (dpvo.py:818-824,
                    fastba instead of the fork's python_ba_wrapper)
  keyframe removal  edges of patches older than n - REMOVAL_WINDOW moved to the
                    inactive store (dpvo.py:684-693, DevicePatchGraph.remove_by_window)

The update network (net.py) needs trained weights that are absent, so a
synthetic "oracle network" stands in: delta = (true reprojection - coords) +
noise, weight = 0.5 (i.e. a well-trained network on a synthetic scene with a
known trajectory).  Everything else is the real op sequence on HIP kernels.
"""
from __future__ import annotations

import math
import time

import numpy as np
import torch

from . import altcorr, fastba
from .patchgraph import DevicePatchGraph
from .synthetic import channels_last, se3_exp


class UpdateHarness:
    def __init__(self, device="cuda", M=96, lifetime=13, removal_window=22, opt_window=10,
                 mem=36, H=120, W=160, C=128, DIM=384, max_edges=60000, buffer=512,
                 ba_iters=2, seed=0, feat_dtype=torch.float32, pose_noise=0.01, depth_init=0.6):
        self.dev = torch.device(device)
        self.M, self.r, self.rw, self.ow = M, lifetime, removal_window, opt_window
        self.mem = self.pmem = mem
        self.H, self.W, self.C = H, W, C
        self.ba_iters = ba_iters
        self.n = 0
        g = torch.Generator().manual_seed(seed)
        self.g = g
        N = buffer
        # ground-truth trajectory (forward motion + wobble) and scene depths
        xi = torch.zeros(N, 6, dtype=torch.float64)
        t = torch.arange(N, dtype=torch.float64)
        xi[:, 2] = 0.04 * t
        xi[:, 0] = 0.05 * torch.sin(0.1 * t)
        xi[:, 4] = 0.02 * torch.sin(0.07 * t)
        self.gt_poses = torch.from_numpy(se3_exp(xi.numpy())).float().to(self.dev)
        self.poses = self.gt_poses.clone()
        self.poses[:, :3] += pose_noise * torch.randn(N, 3, generator=g).to(self.dev)
        self.poses[0] = self.gt_poses[0]
        P = 3
        self.P = P
        cxy = torch.stack([torch.rand(N * M, generator=g) * (W - 9) + 4,
                           torch.rand(N * M, generator=g) * (H - 9) + 4], -1).floor()
        self.gt_d = (torch.rand(N * M, generator=g) * 0.8 + 0.3).to(self.dev)
        off = torch.arange(P, dtype=torch.float32) - P // 2
        patches = torch.zeros(N * M, 3, P, P)
        patches[:, 0] = cxy[:, 0].view(-1, 1, 1) + off.view(1, 1, P)
        patches[:, 1] = cxy[:, 1].view(-1, 1, 1) + off.view(1, P, 1)
        patches[:, 2] = depth_init  # DPVO initialises new patch depths to a median
        self.patches = patches.to(self.dev)
        self.gt_patches = self.patches.clone()
        self.gt_patches[:, 2] = self.gt_d.view(-1, 1, 1)
        self.intrinsics = torch.tensor([80.0, 80.0, 80.0, 60.0]).view(1, 4).repeat(N, 1).to(self.dev)
        self.ix = torch.arange(N, device=self.dev).repeat_interleave(M)
        # feature rings: channels-last pyramid (levels 1, 4) and gmap
        self.levels = (1, 4)
        self.pyr = [channels_last(torch.zeros(1, mem, C, H // s, W // s, device=self.dev,
                                              dtype=feat_dtype)) for s in self.levels]
        self.gmap = torch.zeros(1, self.pmem * M, C, P, P, device=self.dev, dtype=feat_dtype)
        self.pg = DevicePatchGraph(max_edges=max_edges, DIM=DIM, device=self.dev, net=False)
        self.lmbda = torch.tensor([1e-4], device=self.dev)
        self.feat_dtype = feat_dtype
        self.stats = []

    # -- dpvo.py __call__: features of the new frame ------------------------
    def _insert_frame(self):
        n = self.n
        fmap = 0.25 * torch.randn(self.C, self.H, self.W, device=self.dev,
                                  dtype=torch.float32).to(self.feat_dtype)
        altcorr.insert_frame(fmap, self.pyr, n % self.mem, self.levels)
        ctr = self.patches[n * self.M:(n + 1) * self.M, :2, 1, 1].unsqueeze(0)
        slot = n % self.pmem
        self.gmap[0, slot * self.M:(slot + 1) * self.M] = altcorr.patchify(
            fmap.unsqueeze(0), ctr, 1)[0]

    # -- dpvo.py:838-903 ------------------------------------------------------
    def _edges(self):
        n, M, r = self.n + 1, self.M, self.r  # DPVO adds edges after n += 1
        d = self.dev
        t0, t1 = M * max(n - r, 0), M * max(n - 1, 0)
        kf = torch.arange(t0, t1, device=d)
        jf = torch.full_like(kf, n - 1)
        kb = torch.arange(M * (n - 1), M * n, device=d).repeat_interleave(n - max(n - r, 0))
        jb = torch.arange(max(n - r, 0), n, device=d).repeat(M)
        return torch.cat([kf, kb]), torch.cat([jf, jb])

    # -- the oracle network --------------------------------------------------
    def _network(self, coords, ii, jj, kk):
        true = fastba.reproject(self.gt_poses, self.gt_patches, self.intrinsics, ii, jj, kk)
        c = coords[..., self.P // 2, self.P // 2]
        delta = (true[..., self.P // 2, self.P // 2] - c) + 0.1 * torch.randn(
            c.shape, device=self.dev, generator=None)
        weight = torch.full_like(c, 0.5)
        return delta, weight

    def step(self):
        """One frame: insertion, edges, update (reproject, corr, network, BA),
        removal.  Returns a dict of per-phase wall-clock ms (synchronised)."""
        sync = torch.cuda.synchronize
        t = [time.perf_counter()]
        self._insert_frame()
        kk_new, jj_new = self._edges()
        self.pg.append_factors(self.ix, kk_new, jj_new)
        self.n += 1
        E = self.pg.num_edges  # host count: DPVO keeps it on the host too
        sync()
        t.append(time.perf_counter())
        ii, jj, kk = self.pg.ii[:E], self.pg.jj[:E], self.pg.kk[:E]
        t0 = max(self.n - self.ow, 1)
        ws = None
        if fastba.cuda_ba.plan_supported(E, t0, self.n, self.P):
            # the BA's edge grouping rides in the reprojection launch (the
            # edges stay fixed until the BA below)
            coords, order, ws = fastba.reproject(self.poses, self.patches, self.intrinsics, ii,
                                                 jj, kk, mem=self.mem, plan_window=(t0, self.n))
        else:
            coords, order = fastba.reproject(self.poses, self.patches, self.intrinsics, ii, jj,
                                             kk, mem=self.mem)
        corr = altcorr.corr_levels(self.gmap, self.pyr, coords, kk % (self.M * self.pmem),
                                   jj % self.mem, 3, self.levels, order=order)
        delta, weight = self._network(coords, ii, jj, kk)
        target = coords[..., self.P // 2, self.P // 2] + delta
        self.pg.target[0, :E] = target[0]
        self.pg.weight[0, :E] = weight[0]
        sync()
        t.append(time.perf_counter())
        fastba.BA(self.poses, self.patches, self.intrinsics, self.pg.target[:, :E],
                  self.pg.weight[:, :E], self.lmbda, ii, jj, kk, t0, self.n, M=self.M,
                  iterations=self.ba_iters, plan=ws)
        sync()
        t.append(time.perf_counter())
        self.pg.remove_by_window(self.ix, self.n, self.rw)
        sync()
        t.append(time.perf_counter())
        st = {"frame": self.n, "edges": E, "corr_shape": tuple(corr.shape),
              "insert+edges_ms": 1e3 * (t[1] - t[0]), "reproject+corr+net_ms": 1e3 * (t[2] - t[1]),
              "ba_ms": 1e3 * (t[3] - t[2]), "removal_ms": 1e3 * (t[4] - t[3]),
              "total_ms": 1e3 * (t[4] - t[0])}
        self.stats.append(st)
        return st

    def depth_error(self, lo, hi):
        """Mean |inverse depth - truth| of the patches of frames [lo, hi)."""
        s = slice(lo * self.M, hi * self.M)
        return float((self.patches[s, 2, 1, 1] - self.gt_d[s]).abs().mean())

    def pose_error(self):
        """Mean translation error of the optimised window vs ground truth (m)."""
        n = self.n
        a, b = self.poses[max(n - self.ow, 1):n, :3], self.gt_poses[max(n - self.ow, 1):n, :3]
        return float((a - b).norm(dim=-1).mean())


__all__ = ["UpdateHarness"]
