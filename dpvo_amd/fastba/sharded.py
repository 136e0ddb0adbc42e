"""Edge-sharded global bundle adjustment across ranks.

The reference has no distributed code; its global BA is one
`fastba.BA(..., eff_impl=True)` call on one GPU (dpvo.py:695-715 ->
ba_cuda.cu:433-582 + block_e.cu).  For graphs large enough to shard (BASELINE
cfg4: 1024 frames x 96 patches, ~131k edges, N = 1023 free poses) this driver
runs one process per GPU:

* Edges are partitioned by the SOURCE FRAME of their patch (kk // PPF) into
  contiguous frame ranges with balanced edge counts, so every patch's edges --
  and with them its C, u, Q and E column -- live on one rank.
* Every rank holds the replicated edge list and runs the same setup, so the
  block-sparse pattern of S (and the packed layout [y (6N) | S lower 6x6
  blocks]) is identical everywhere.  Per BA iteration each rank linearises
  only its own patches and writes its partial (S, y) into that layout.
* ONE collective per iteration: all_reduce(SUM) of the packed fp64 buffer
  (torch.distributed, backend "nccl" = RCCL over xGMI).  A ring all-reduce
  delivers identical bits to every rank, so every rank runs the same solve
  and gets the same dX; poses are updated identically everywhere, inverse
  depths only for owned patches.

`backend` abstracts the four native steps (HIP by default); tests plug the C
oracle in to exercise the partitioning + collective on CPU with gloo.
"""
from __future__ import annotations

from typing import List, Optional, Sequence, Tuple

import torch
import torch.distributed as dist

from .._native import load_extension


def frame_partition(kk: torch.Tensor, PPF: int, world: int) -> List[Tuple[int, int]]:
    """Contiguous source-frame ranges [lo, hi) per rank, balanced by edge count.
    The first range starts at -inf and the last ends at +inf so every edge is
    owned by exactly one rank."""
    if world <= 1:
        return [(-(2**31) + 1, 2**31 - 1)]
    frames = torch.div(kk, PPF, rounding_mode="floor").clamp(min=0)
    counts = torch.bincount(frames).cpu()
    cum = torch.cumsum(counts, 0)
    total = int(cum[-1])
    cuts = []
    for r in range(1, world):
        target = total * r / world
        f = int(torch.searchsorted(cum, torch.tensor(target, dtype=cum.dtype), right=False)) + 1
        cuts.append(max(f, cuts[-1] if cuts else 0))
    bounds = [-(2**31) + 1] + cuts + [2**31 - 1]
    return [(bounds[r], bounds[r + 1]) for r in range(world)]


class HipBackend:
    """The large-graph F-BA kernels of ba_large.hip through the cuda_ba module."""

    def __init__(self):
        self.ext = load_extension("cuda_ba")

    def setup(self, ii, jj, kk, num_patches, PPF, t0, t1, own_lo, own_hi):
        ws = self.ext.gba_setup(ii, jj, kk, num_patches, PPF, t0, t1, own_lo, own_hi)
        info = self.ext.gba_info(ws, ii.numel(), t0, t1).cpu().tolist()  # one sync per BA call
        return {"ws": ws, "E": ii.numel(), "t0": t0, "t1": t1, "info": info,
                "packed": self.ext.gba_packed(ws, ii.numel(), t0, t1, info[3])}

    def packed(self, st) -> torch.Tensor:
        return st["packed"]

    def build(self, st, poses, patches, intrinsics, target, weight, lmbda, ii, jj):
        self.ext.gba_build(st["ws"], poses, patches, intrinsics, target, weight, lmbda, ii, jj,
                           st["t0"], st["t1"])

    def solve_update(self, st, poses, patches):
        self.ext.gba_solve_update(st["ws"], poses, patches, st["E"], st["t0"], st["t1"])

    def status(self, st) -> List[int]:
        return self.ext.gba_info(st["ws"], st["E"], st["t0"], st["t1"]).cpu().tolist()


class ShardedBA:
    """fastba.BA for one (large) graph, edge-sharded over the ranks of `group`.

    Construct on every rank with the same replicated edge list, then call like
    fastba.BA (poses / patches updated in place).  With world size 1 it is the
    plain single-GPU large-graph BA."""

    def __init__(self, ii, jj, kk, num_patches: int, PPF: int, t0: int, t1: int,
                 group=None, backend=None, ranges: Optional[Sequence[Tuple[int, int]]] = None):
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_available() and dist.is_initialized() else 1
        self.rank = dist.get_rank(group) if self.world > 1 else 0
        self.backend = backend if backend is not None else HipBackend()
        self.ranges = list(ranges) if ranges is not None else frame_partition(kk, PPF, self.world)
        assert len(self.ranges) == self.world
        self.own = self.ranges[self.rank]
        self.ii, self.jj, self.kk = ii, jj, kk
        self.t0, self.t1 = t0, t1
        self.state = self.backend.setup(ii, jj, kk, num_patches, PPF, t0, t1, *self.own)

    @property
    def allreduce_bytes(self) -> int:
        return self.backend.packed(self.state).numel() * 8

    def owned_patches(self, num_patches: int, PPF: int) -> torch.Tensor:
        f = torch.arange(num_patches) // PPF
        return (f >= self.own[0]) & (f < self.own[1])

    def __call__(self, poses, patches, intrinsics, target, weight, lmbda, iterations: int = 2):
        for _ in range(iterations):
            self.backend.build(self.state, poses, patches, intrinsics, target, weight, lmbda,
                               self.ii, self.jj)
            if self.world > 1 and self.t1 > self.t0:
                dist.all_reduce(self.backend.packed(self.state), op=dist.ReduceOp.SUM,
                                group=self.group)
            self.backend.solve_update(self.state, poses, patches)
        return []
