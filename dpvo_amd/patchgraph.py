"""PatchGraph edge bookkeeping on the device.

Mirrors the edge part of dpvo/patchgraph.py (11-63: static MAX_EDGES buffers
ii / jj / kk, net, weight, target and the *_inac store) and DPVO's
append_factors / remove_factors (dpvo/dpvo.py:480-568), with the edge counts
kept on the device: every call is a fixed sequence of HIP kernel launches and
never synchronises with the host (the reference calls mask.sum().item() and
boolean-mask gathers on every removal).  The window rule of
DPVO.keyframe (dpvo.py:684-693) is a predicate evaluated on the device
(remove_by_window).

Removal is a stable compaction into a second set of buffers that is then
swapped in (ping-pong), so `ii` / `jj` / ... may be different tensor objects
after a removal -- read them from the graph, do not keep references.
"""
from __future__ import annotations

import torch

from ._native import load_extension, require_gpu


class DevicePatchGraph:
    def __init__(self, max_edges=10000, DIM=384, device="cuda", net=True):
        self._ext = load_extension("cuda_ba")
        dev = torch.device(device)
        self.max_edges = int(max_edges)
        self.DIM = int(DIM)

        def bufs(with_net):
            return {
                "ii": torch.zeros(max_edges, dtype=torch.long, device=dev),
                "jj": torch.zeros(max_edges, dtype=torch.long, device=dev),
                "kk": torch.zeros(max_edges, dtype=torch.long, device=dev),
                "net": (torch.zeros(1, max_edges, DIM, device=dev) if with_net
                        else torch.empty(0, device=dev)),
                "weight": torch.zeros(1, max_edges, 2, device=dev),
                "target": torch.zeros(1, max_edges, 2, device=dev),
            }

        self._a = bufs(net)
        self._b = bufs(net)
        inac = bufs(False)
        self.ii_inac, self.jj_inac, self.kk_inac = inac["ii"], inac["jj"], inac["kk"]
        self.weight_inac, self.target_inac = inac["weight"], inac["target"]
        # [0] num_edges [1] num_edges_inac [2] error flags [3..4] scratch
        self.counts = torch.zeros(8, dtype=torch.int32, device=dev)
        self._pos = torch.zeros(max_edges, dtype=torch.int32, device=dev)
        require_gpu(self.counts)

    # active buffers (the objects change after a removal: ping-pong)
    ii = property(lambda self: self._a["ii"])
    jj = property(lambda self: self._a["jj"])
    kk = property(lambda self: self._a["kk"])
    net = property(lambda self: self._a["net"])
    weight = property(lambda self: self._a["weight"])
    target = property(lambda self: self._a["target"])

    @property
    def num_edges(self) -> int:
        """Host copy of the active edge count (synchronises; for callers that
        need the number on the host, e.g. to slice)."""
        return int(self.counts[0].item())

    @property
    def num_edges_inac(self) -> int:
        return int(self.counts[1].item())

    @property
    def errors(self) -> int:
        """1: an append overflowed MAX_EDGES (edges not added); 2: the inactive
        store was full (removed edges not stored); 4: edges_loop saw a frame
        count above its n_cap (no loop edges taken); 8: the keyframe pg.delta
        log was full (a record was not kept).  Synchronises."""
        return int(self.counts[2].item())

    def append_factors(self, ix, kk, jj):
        """dpvo.py:480-521 append_factors(ii=kk, jj): edges at [num, num + n),
        ii = ix[kk], hidden states zeroed."""
        a = self._a
        self._ext.pg_append(ix, kk.contiguous(), jj.contiguous(), a["ii"], a["jj"], a["kk"],
                            a["net"], self.counts)

    def _remove(self, mask, ix, thresh, lc_min, store):
        a, b = self._a, self._b
        keys = ("ii", "jj", "kk", "net", "weight", "target")
        self._ext.pg_remove(mask, ix, int(thresh), int(lc_min), bool(store), [a[k] for k in keys],
                            [b[k] for k in keys],
                            [self.ii_inac, self.jj_inac, self.kk_inac, self.weight_inac,
                             self.target_inac], self.counts, self._pos)
        self._a, self._b = b, a

    def remove_factors(self, mask, store: bool):
        """dpvo.py:523-568 remove_factors(m, store): mask (bool, 1 = remove)
        over the active edges (longer masks are read up to num_edges)."""
        self._remove(mask, None, 0, -1, store)

    def remove_by_window(self, ix, n, removal_window, loop_closure=False, optimization_window=10,
                         store=True):
        """The removal of DPVO.keyframe (dpvo.py:684-693): edges whose patch
        frame ix[kk] < n - REMOVAL_WINDOW, except (LOOP_CLOSURE) edges with
        jj - ii > 30 and jj > n - OPTIMIZATION_WINDOW; removed edges stored."""
        lc_min = n - optimization_window if loop_closure else -1
        self._remove(None, ix, n - removal_window, lc_min, store)

    def remove_by_window_dev(self, ix, n_dev, removal_window, loop_closure=False,
                             optimization_window=10, store=True):
        """remove_by_window with the frame count read on the device (int32
        scalar n_dev): graph-replayable, the thresholds move with the frame."""
        a, b = self._a, self._b
        keys = ("ii", "jj", "kk", "net", "weight", "target")
        self._ext.pg_remove_window_dev(ix, n_dev, -int(removal_window), -int(optimization_window),
                                       bool(loop_closure), bool(store), [a[k] for k in keys],
                                       [b[k] for k in keys],
                                       [self.ii_inac, self.jj_inac, self.kk_inac, self.weight_inac,
                                        self.target_inac], self.counts, self._pos)
        self._a, self._b = b, a

    def append_factors_dev(self, ix, kk, jj, n_dev):
        """append_factors of the first min(n_dev, len(kk)) edges, n_dev an
        int32 device scalar (edges_loop's count, dpvo.py:986-988)."""
        a = self._a
        self._ext.pg_append_dev(ix, kk.contiguous(), jj.contiguous(), n_dev, a["ii"], a["jj"],
                                a["kk"], a["net"], self.counts)

    def keyframe(self, st, poses, patches, intrinsics, M, frames=(), rings=(), tstamps=None,
                 keyframe_index=4, keyframe_thresh=12.5, kf=None, mag=None, delta=None):
        """DPVO.keyframe's frame drop (dpvo.py:586-673) on the device, no host
        sync: the decision (motionmag of frames n-KI-1 <-> n-KI+1 below
        KEYFRAME_THRESH) is a device flag kf = {drop, k} that predicates the
        removal of the edges touching k (not stored), the edge index shift,
        the move of every per-frame array in `frames` (ring[a] > 0: row =
        frame % ring) and n -= 1, m -= M in st = {n, m} (int32 device).
        poses / patches / intrinsics / tstamps are the per-frame buffers
        (patches [N*M,3,P,P]); they are shifted too.  delta = (log [cap,7],
        tstamps [cap,2] (t1, t0), count int32[1]) records pg.delta.
        Returns (kf, mag) device tensors."""
        dev = self.counts.device
        kf = torch.zeros(2, dtype=torch.int32, device=dev) if kf is None else kf
        mag = torch.zeros(2, dtype=torch.float32, device=dev) if mag is None else mag
        a, b = self._a, self._b
        self._ext.kf_motion(a["ii"], a["jj"], a["kk"], self.counts, poses, patches, intrinsics,
                            st, int(keyframe_index), float(keyframe_thresh), kf, mag)
        keys = ("ii", "jj", "kk", "net", "weight", "target")
        self._ext.pg_remove_frame_dev(kf, [a[k] for k in keys], [b[k] for k in keys],
                                      self.counts, self._pos)
        self._a, self._b = b, a
        a = self._a
        # per-frame rows: patches [N*M, 3, P, P] moves M patches per frame
        fr = [poses, patches.view(patches.shape[0] // M, -1), intrinsics] + ([tstamps] if tstamps is not None else []) + list(frames)
        rg = [0, 0, 0] + ([0] if tstamps is not None else []) + [int(r) for r in rings]
        if len(frames) != len(rings):
            raise ValueError("one ring size per frame array")
        dl = dt = dc = None
        if delta is not None:
            if tstamps is None:
                raise ValueError("the delta log needs tstamps")
            dl, dt, dc = delta
        self._ext.kf_shift(kf, int(M), st, a["ii"], a["jj"], a["kk"], self.counts, fr, rg,
                           poses if dl is not None else None, tstamps if dl is not None else None,
                           dl, dt, dc)
        return kf, mag

    def edges_loop(self, poses, patches, intrinsics, ix, st, n_cap, M, last_global_ba=None,
                   removal_window=20, max_edge_age=1000, global_opt_freq=15, keyframe_index=4,
                   backend_thresh=64.0, max_num_edges=1000, nms=1, out=None):
        """PatchGraph.edges_loop (patchgraph.py:65-91) on the device for the
        frame count st[0] (n_cap >= n sizes the launch); with last_global_ba
        (int32 device scalar) gated and updated as dpvo.py:984-988.
        Returns (kk, jj, count) -- count an int32 device scalar (edges x M);
        append them with append_factors_dev(ix, kk, jj, count)."""
        dev = self.counts.device
        if out is None:
            out = (torch.empty(max_num_edges * M, dtype=torch.long, device=dev),
                   torch.empty(max_num_edges * M, dtype=torch.long, device=dev),
                   torch.zeros(1, dtype=torch.int32, device=dev),
                   torch.empty(self._ext.edges_loop_work_floats(), device=dev))
        kk, jj, cnt, work = out
        self._ext.edges_loop(poses, patches, intrinsics, ix, int(M), st, int(n_cap),
                             last_global_ba,
                             int(removal_window), int(max_edge_age), int(global_opt_freq),
                             int(keyframe_index), float(backend_thresh), int(max_num_edges),
                             int(nms), work, kk, jj, cnt, self.counts[2:3])
        return kk, jj, cnt


__all__ = ["DevicePatchGraph"]
