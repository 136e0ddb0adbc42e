"""DPVO.update() data flow on the MI355X ops at real shapes.

Reproduces, per frame, what dpvo/dpvo.py does around the update operator
(config/default.yaml: PATCH_LIFETIME 13, REMOVAL_WINDOW 22,
OPTIMIZATION_WINDOW 10; mem = pmem = 36; MAX_EDGES 10000, dpvo/config.py:42):

  frame insertion   fmap -> channels-last pyramid ring, levels [1, 4]
                    (dpvo.py __call__; one launch: altcorr.insert_frame_ring), gmap of
                    the new patches (altcorr.patchify)
  edges             __edges_forw / __edges_back (dpvo.py:838-903) appended on the
                    device (DevicePatchGraph.append_factors, dpvo.py:480-521)
  update()          reproject (+ A-CORR edge order + BA plan) -> corr at levels
                    [1, 4] with kk % (M pmem), jj % mem (dpvo.py:456-465) ->
                    [network] -> target = coords[..., 1, 1] + delta (dpvo.py:805-806)
                    -> fastba.BA(t0 = n - OPTIMIZATION_WINDOW, t1 = n, iterations=1)
                    (dpvo.py:818-824: the fork's local call, python_ba_wrapper with
                    iterations=1, here on the HIP fastba)
  keyframe()        (keyframes=True) the frame drop of dpvo.py:601-673 on the device
                    (DevicePatchGraph.keyframe: motion magnitude, decision flag,
                    edge removal + index shift, every per-frame buffer and ring
                    shifted, n -= 1), then the window removal: edges of patches
                    older than n - REMOVAL_WINDOW moved to the inactive store
                    (dpvo.py:684-693)

Every per-frame scalar the kernels need (frame count n, ring slots, the BA
window start t0) lives in a small int32 device tensor (`fs`), so once the
edge count is steady (it is, with the window rule) ONE update is captured as
a hipGraph (`capture()`) and replayed for every later frame (`replay()`): no
host synchronisation and no per-kernel launch from Python inside a frame.
With keyframes=True the edge count depends on which frames were dropped, so
the harness reads n and the edge count back once per frame, as the
reference does (its num_edges / n are host integers): eager only.

Frames are inserted by timestamp t (the synthetic truth, the initial pose and
patches and the features are functions of t) at buffer index n; with frame
drops t and n part, and the truth moves with the frame data.

The update network (net.py) needs trained weights that are absent, so a
deterministic "oracle network" stands in: delta = (true reprojection - coords)
+ a fixed pseudo-random perturbation of amplitude net_noise px (default 0.1),
weight = 0.5.  The frame features
are a fixed random field modulated per frame (deterministic, so an eager run
and a graph replay produce the same bits).

MAX_EDGES: with M patches per frame a steady-state update sees 497 M active
edges (lifetime 13, removal window 22: the patches of the last 23 frames), so
the reference's MAX_EDGES = 10000 admits M <= 20; DPVO's default.yaml M = 96
needs ~47.7k (the reference's append_factors raises RuntimeError beyond
MAX_EDGES, dpvo.py:502-507).
"""
from __future__ import annotations

import time

import torch

from . import altcorr, fastba
from .patchgraph import DevicePatchGraph
from .synthetic import channels_last, se3_exp


class UpdateHarness:
    def __init__(self, device="cuda", M=20, lifetime=13, removal_window=22, opt_window=10,
                 mem=36, H=120, W=160, C=128, DIM=384, max_edges=10000, buffer=512,
                 ba_iters=1, seed=0, feat_dtype=torch.float32, pose_noise=0.01, depth_init=0.6,
                 keyframes=False, keyframe_index=4, keyframe_thresh=12.5, net_noise=0.1):
        self.dev = torch.device(device)
        self.M, self.r, self.rw, self.ow = M, lifetime, removal_window, opt_window
        self.mem = self.pmem = mem
        self.H, self.W, self.C = H, W, C
        self.ba_iters = ba_iters
        self.net_noise = float(net_noise)
        self.keyframes, self.ki, self.kthresh = keyframes, keyframe_index, keyframe_thresh
        self.n = 0
        self.t = 0
        g = torch.Generator().manual_seed(seed)
        N = buffer
        self.buffer = N
        # ground-truth trajectory (forward motion + wobble) and scene depths
        xi = torch.zeros(N, 6, dtype=torch.float64)
        t = torch.arange(N, dtype=torch.float64)
        xi[:, 2] = 0.04 * t
        xi[:, 0] = 0.05 * torch.sin(0.1 * t)
        xi[:, 4] = 0.02 * torch.sin(0.07 * t)
        # by timestamp: truth and initial values (copied to index n on insertion)
        self.gt_poses_t = torch.from_numpy(se3_exp(xi.numpy())).float().to(self.dev)
        self.init_poses_t = self.gt_poses_t.clone()
        self.init_poses_t[:, :3] += pose_noise * torch.randn(N, 3, generator=g).to(self.dev)
        self.init_poses_t[0] = self.gt_poses_t[0]
        self.gt_poses = self.gt_poses_t.clone()
        self.poses = self.init_poses_t.clone()
        P = 3
        self.P = P
        cxy = torch.stack([torch.rand(N * M, generator=g) * (W - 9) + 4,
                           torch.rand(N * M, generator=g) * (H - 9) + 4], -1).floor()
        gt_d = (torch.rand(N * M, generator=g) * 0.8 + 0.3).to(self.dev)
        off = torch.arange(P, dtype=torch.float32) - P // 2
        patches = torch.zeros(N * M, 3, P, P)
        patches[:, 0] = cxy[:, 0].view(-1, 1, 1) + off.view(1, 1, P)
        patches[:, 1] = cxy[:, 1].view(-1, 1, 1) + off.view(1, P, 1)
        patches[:, 2] = depth_init  # DPVO initialises new patch depths to a median
        self.init_patches_t = patches.to(self.dev)
        self.gt_patches_t = self.init_patches_t.clone()
        self.gt_patches_t[:, 2] = gt_d.view(-1, 1, 1)
        self.patches = self.init_patches_t.clone()
        self.gt_patches = self.gt_patches_t.clone()
        self.tstamps = torch.arange(N, dtype=torch.long, device=self.dev)
        self.intrinsics = torch.tensor([80.0, 80.0, 80.0, 60.0]).view(1, 4).repeat(N, 1).to(self.dev)
        self.ix = torch.arange(N, device=self.dev).repeat_interleave(M)
        # feature rings: channels-last pyramid (levels 1, 4) and gmap
        self.levels = (1, 4)
        self.pyr = [channels_last(torch.zeros(1, mem, C, H // s, W // s, device=self.dev,
                                              dtype=feat_dtype)) for s in self.levels]
        self.gmap = torch.zeros(1, self.pmem * M, C, P, P, device=self.dev, dtype=feat_dtype)
        self.field = torch.randn(C, H, W, generator=g).to(self.dev)
        self.pg = DevicePatchGraph(max_edges=max_edges, DIM=DIM, device=self.dev, net=False)
        self.lmbda = torch.tensor([1e-4], device=self.dev)
        self.feat_dtype = feat_dtype
        # device frame state: [0] n (frames before this step), [1] t0 of the BA
        # window, [2] n + 1 (DPVO's n after the increment), [3] DPVO's m
        # ([2:4] is keyframe()'s {n, m}), [4] n % pmem, [5] timestamp t
        self.fs = torch.zeros(8, dtype=torch.int32, device=self.dev)
        if keyframes:
            self._kf = (torch.zeros(2, dtype=torch.int32, device=self.dev),
                        torch.zeros(2, dtype=torch.float32, device=self.dev))
            self.delta = (torch.zeros(N, 7, device=self.dev),
                          torch.zeros(N, 2, dtype=torch.long, device=self.dev),
                          torch.zeros(1, dtype=torch.int32, device=self.dev))
            self.dropped = 0
        self._arM = torch.arange(M, device=self.dev)
        self.graph = None
        self.keep_inputs = False
        self.last = {}
        self.stats = []

    # -- per-frame device scalars -------------------------------------------
    def _frame_scalars(self):
        fs = self.fs
        fs[2:3].copy_(fs[0:1] + 1)
        fs[1:2].copy_(torch.clamp_min(fs[2:3] - self.ow, 1))
        fs[3:4].copy_(fs[2:3] * self.M)
        fs[4:5].copy_(torch.remainder(fs[0:1], self.pmem))

    # -- dpvo.py __call__: features of the new frame ------------------------
    def _insert_frame(self):
        tf = self.fs[5:6].float()
        fmap = (0.25 * torch.sin(self.field + 0.37 * tf)).to(self.feat_dtype)
        altcorr.insert_frame_ring(fmap, self.pyr, self.fs[0:1], self.levels)
        n64, t64 = self.fs[0:1].long(), self.fs[5:6].long()
        # the frame's truth / initial values: timestamp row t -> index row n
        for dst, src in ((self.poses, self.init_poses_t), (self.gt_poses, self.gt_poses_t)):
            dst.index_copy_(0, n64, src.index_select(0, t64))
        tidx = t64 * self.M + self._arM
        idx = n64 * self.M + self._arM
        for dst, src in ((self.patches, self.init_patches_t),
                         (self.gt_patches, self.gt_patches_t)):
            dst.index_copy_(0, idx, src.index_select(0, tidx))
        self.tstamps.index_copy_(0, n64, t64)
        ctr = self.patches.index_select(0, idx)[:, :2, 1, 1].unsqueeze(0)
        rows = self.fs[4:5].long() * self.M + self._arM
        g = altcorr.patchify(fmap.unsqueeze(0), ctr, 1)[0]
        self.gmap[0].index_copy_(0, rows, g)

    # -- dpvo.py:838-903 (counts from the host n, values from the device n) --
    def _edges(self, n):
        M, r = self.M, self.r
        n1 = n + 1  # DPVO adds edges after n += 1
        lo = max(n1 - r, 0)
        cf, cb = M * (n1 - 1 - lo), n1 - lo
        nd = self.fs[2:3].long()
        lod = torch.clamp_min(nd - r, 0)
        kf = lod * M + torch.arange(cf, device=self.dev)
        jf = (nd - 1).expand(cf)
        kb = (nd - 1) * M + self._arM.repeat_interleave(cb)
        jb = lod + torch.arange(cb, device=self.dev).repeat(M)
        return torch.cat([kf, kb]), torch.cat([jf, jb])

    # -- the oracle network --------------------------------------------------
    def _network(self, coords, ii, jj, kk):
        true = fastba.reproject(self.gt_poses, self.gt_patches, self.intrinsics, ii, jj, kk)
        c = coords[..., self.P // 2, self.P // 2]
        h = (kk.float() * 12.9898 + jj.float() * 78.233 + 0.5 * self.fs[0:1].float())
        u = torch.stack([torch.sin(h), torch.cos(1.7 * h)], -1).view(c.shape)
        delta = (true[..., self.P // 2, self.P // 2] - c) + self.net_noise * u
        weight = torch.full_like(c, 0.5)
        return delta, weight

    def _frame_start(self, n):
        self._frame_scalars()
        self._insert_frame()
        kk_new, jj_new = self._edges(n)
        self.pg.append_factors(self.ix, kk_new, jj_new)

    def _update_ops(self, n, E, started=False):
        """Everything of one frame after the host decided the shapes (n, E)."""
        if not started:
            self._frame_start(n)
        ii, jj, kk = self.pg.ii[:E], self.pg.jj[:E], self.pg.kk[:E]
        n1 = n + 1
        N = n1 - max(n1 - self.ow, 1)
        t0d = self.fs[1:2]
        coords, order, ws = fastba.reproject_window_dev(self.poses, self.patches, self.intrinsics,
                                                        ii, jj, kk, self.mem, t0d, N)
        corr = altcorr.corr_levels(self.gmap, self.pyr, coords, kk % (self.M * self.pmem),
                                   jj % self.mem, 3, self.levels, order=order)
        delta, weight = self._network(coords, ii, jj, kk)
        target = coords[..., self.P // 2, self.P // 2] + delta
        self.pg.target[0, :E] = target[0]
        self.pg.weight[0, :E] = weight[0]
        if self.keep_inputs:  # tests: the BA's inputs, before it changes poses / depths
            self.last_inputs = {"poses": self.poses.clone(), "patches": self.patches.clone(),
                                "ii": ii.clone(), "jj": jj.clone(), "kk": kk.clone(),
                                "target": self.pg.target[:, :E].clone(),
                                "weight": self.pg.weight[:, :E].clone(), "N": N,
                                "gmap": self.gmap.clone(), "pyr": [p.clone() for p in self.pyr]}
        fastba.BA_dev(self.poses, self.patches, self.intrinsics, self.pg.target[:, :E],
                      self.pg.weight[:, :E], self.lmbda, ii, jj, kk, t0d, N, ws,
                      iterations=self.ba_iters)
        if self.keyframes:
            self._keyframe()
        self.pg.remove_by_window_dev(self.ix, self.fs[2:3], self.rw)
        self.fs[0:1].copy_(self.fs[2:3])
        self.fs[5:6].add_(1)
        self.last = {"coords": coords, "corr": corr, "ws": ws}

    def _keyframe(self):
        """dpvo.py:601-673 on the device: every per-frame buffer the harness
        keeps moves with the dropped frame (rings: the pyramid levels and the
        gmap by slot; the truth by index)."""
        M = self.M
        frames = [self.gt_poses, self.gt_patches.view(self.buffer, -1)]
        rings = [0, 0]
        for p in self.pyr:  # channels-last storage [1, mem, H, W, C]
            frames.append(p.permute(0, 1, 3, 4, 2).reshape(self.mem, -1))
            rings.append(self.mem)
        frames.append(self.gmap.view(self.pmem, -1))
        rings.append(self.pmem)
        self.pg.keyframe(self.fs[2:4], self.poses, self.patches, self.intrinsics, M,
                         frames=frames, rings=rings, tstamps=self.tstamps,
                         keyframe_index=self.ki, keyframe_thresh=self.kthresh,
                         kf=self._kf[0], mag=self._kf[1], delta=self.delta)

    def _edges_after_append(self, n):
        """Host count of active edges after frame n's append: the window rule
        makes it a function of n alone (no device read)."""
        M, r, rw = self.M, self.r, self.rw
        n1 = n + 1
        # patches of frames g < n1 - 1 - ... : edges live if ix >= (n1 - 1) - rw
        # at the previous removal; count directly from the rule
        keep_lo = max(n1 - 1 - rw, 0)  # the last removal (previous frame) used n = n1 - 1
        tot = 0
        for g in range(keep_lo, n1):
            lo, hi = max(g - r + 1, 0), min(g + r - 1, n1 - 1)
            tot += M * (hi - lo + 1)
        return tot

    def step(self):
        """One frame, eagerly: insertion, edges, update (reproject, corr,
        network, BA), removal.  Returns per-phase host wall-clock ms."""
        if self.t + 1 >= self.buffer:  # t >= n (frames dropped)
            raise RuntimeError("UpdateHarness: frame buffer exhausted")
        n = self.n
        t = time.perf_counter()
        if self.keyframes:  # edge count after the append: read back (host int in DPVO)
            self._frame_start(n)
            E = self.pg.num_edges
            if self.pg.errors & 1:
                raise RuntimeError(f"active edges exceed MAX_EDGES={self.pg.max_edges} "
                                   "(dpvo.py:502-507 raises too)")
            self._update_ops(n, E, started=True)
            self.n = int(self.fs[0].item())
            self.dropped += n + 1 - self.n
        else:
            E = self._edges_after_append(n)
            if E > self.pg.max_edges:
                raise RuntimeError(f"{E} active edges exceed MAX_EDGES={self.pg.max_edges} "
                                   "(dpvo.py:502-507 raises too)")
            self._update_ops(n, E)
            torch.cuda.synchronize()
            self.n += 1
        self.t += 1
        st = {"frame": self.n, "edges": E, "corr_shape": tuple(self.last["corr"].shape),
              "total_ms": 1e3 * (time.perf_counter() - t)}
        self.stats.append(st)
        return st

    def steady(self):
        """True once the edge count no longer changes from frame to frame."""
        return (self.n + 1 >= self.rw + self.r and
                self._edges_after_append(self.n) == self._edges_after_append(self.n - 1))

    def capture(self):
        """Capture one steady-state update as hipGraphs (replayed by replay()).

        The patch-graph removal compacts into the other of two buffer sets
        (ping-pong), so a frame's graph depends on which set is active: two
        graphs are captured, one per parity, and replay() alternates them."""
        if self.keyframes:
            raise RuntimeError("capture(): frame drops make the edge count data-dependent")
        if not self.steady():
            raise RuntimeError("capture() needs the steady state (call step() first)")
        n, E = self.n, self._edges_after_append(self.n)
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        self.graph = []
        pool = None
        for _ in range(2):  # each capture swaps the host's active buffer set once
            g = torch.cuda.CUDAGraph()
            with torch.cuda.stream(s):
                with torch.cuda.graph(g, stream=s, pool=pool):
                    self._update_ops(n, E)
            pool = g.pool()
            self.graph.append(g)
        torch.cuda.current_stream().wait_stream(s)
        # two swaps: the host view is back on the set graph 0 reads; the
        # captures ran no kernel, frame n is still to be processed
        self._parity = 0
        self._graph_E = E

    def replay(self, frames=1):
        """Run `frames` frames through the captured graphs (no host sync)."""
        if not self.graph:
            raise RuntimeError("replay() needs capture()")
        if self.n + frames >= self.buffer:
            raise RuntimeError("UpdateHarness: frame buffer exhausted")
        for _ in range(frames):
            self.graph[self._parity].replay()
            self._parity ^= 1
            self.pg._a, self.pg._b = self.pg._b, self.pg._a  # the set the next frame reads
            self.n += 1
            self.t += 1

    def check(self):
        """Raise on a recorded device-side failure (synchronises): an append
        past MAX_EDGES (error flag 1), an edges_loop frame count past its
        n_cap (4), a full pg.delta log (8) or a fatal BA status.  A full
        inactive store (flag 2) only drops the removed edges, as the
        reference's warning does (dpvo.py:547-549)."""
        if self.pg.errors & (1 | 4 | 8):
            raise RuntimeError(f"patch graph error flags {self.pg.errors}")
        return fastba.cuda_ba.check_status(self.poses)

    def depth_error(self, lo, hi):
        """Mean |inverse depth - truth| of the patches of frames [lo, hi)."""
        s = slice(lo * self.M, hi * self.M)
        return float((self.patches[s, 2, 1, 1] - self.gt_patches[s, 2, 1, 1]).abs().mean())

    def pose_error(self):
        """Mean translation error of the optimised window vs ground truth (m)."""
        n = self.n
        a, b = self.poses[max(n - self.ow, 1):n, :3], self.gt_poses[max(n - self.ow, 1):n, :3]
        return float((a - b).norm(dim=-1).mean())

    def pose_error_scaled(self):
        """pose_error after the best global scale of the trajectory's camera
        centres (monocular BA fixes the scene only up to scale; the error left
        after the scale is the part a scale drift does not explain)."""
        from .lietorch import SE3

        n = self.n
        c = SE3(self.poses[1:n]).inv().data[:, :3].double()
        g = SE3(self.gt_poses[1:n]).inv().data[:, :3].double()
        c0, g0 = c - c.mean(0), g - g.mean(0)
        s = float((c0 * g0).sum() / (c0 * c0).sum())
        lo = max(n - self.ow, 1) - 1
        return float((s * c0[lo:] - g0[lo:]).norm(dim=-1).mean()), s


__all__ = ["UpdateHarness"]
