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
        store was full (removed edges not stored).  Synchronises."""
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


__all__ = ["DevicePatchGraph"]
