"""Edge-sharded global BA driver (dpvo_amd/fastba/sharded.py) on
CPU: world size 2 over gloo, with the C oracle's sharded BA phases
(oracle.ba_shard, test infrastructure) standing in for the HIP kernels.  It
checks the partitioning, the ownership rule, the packed all-reduce and the
replicated solve against the single-process oracle."""
import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import REPO

sys.path.insert(0, REPO)


class OracleBackend:
    """ShardedBA backend over oracle.ba_shard; packed = [y (6N) | S lower 6x6
    blocks, dense pattern (N (N+1) / 2 blocks)]."""

    def setup(self, ii, jj, kk, num_patches, PPF, t0, t1, own_lo, own_hi):
        N = t1 - t0
        return {"ii": ii.numpy(), "jj": jj.numpy(), "kk": kk.numpy(), "PPF": PPF, "t0": t0,
                "t1": t1, "own": (own_lo, own_hi), "N": N,
                "packed": torch.zeros(6 * N + 36 * (N * (N + 1) // 2), dtype=torch.float64)}

    def packed(self, st):
        return st["packed"]

    @staticmethod
    def _tri(N):
        return [(a, b) for a in range(N) for b in range(a + 1)]

    def build(self, st, poses, patches, intrinsics, target, weight, lmbda, ii, jj):
        import oracle

        N = st["N"]
        S, y = oracle.ba_shard(1, poses.numpy(), patches.numpy(), intrinsics.numpy(),
                               target.numpy(), weight.numpy(), float(lmbda[0]), st["ii"], st["jj"],
                               st["kk"], st["t0"], st["t1"], st["PPF"], *st["own"])
        blocks = [S[6 * a:6 * a + 6, 6 * b:6 * b + 6].reshape(-1) for a, b in self._tri(N)]
        st["packed"].copy_(torch.from_numpy(np.concatenate([y] + blocks)))
        st["aux"] = (intrinsics.numpy(), target.numpy(), weight.numpy(), float(lmbda[0]))

    def solve_update(self, st, poses, patches):
        import oracle

        N = st["N"]
        p = st["packed"].numpy()
        y = p[:6 * N]
        S = np.zeros((6 * N, 6 * N))
        for q, (a, b) in enumerate(self._tri(N)):
            blk = p[6 * N + 36 * q: 6 * N + 36 * (q + 1)].reshape(6, 6)
            S[6 * a:6 * a + 6, 6 * b:6 * b + 6] = blk
            S[6 * b:6 * b + 6, 6 * a:6 * a + 6] = blk.T
        intr, target, weight, lm = st["aux"]
        oracle.ba_shard(2, poses.numpy(), patches.numpy(), intr, target, weight, lm, st["ii"],
                        st["jj"], st["kk"], st["t0"], st["t1"], st["PPF"], *st["own"], S=S, y=y)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, out):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from dpvo_amd import synthetic
        from dpvo_amd.fastba.sharded import ShardedBA

        G = synthetic.make_config("cfg4s", seed=3)
        poses, patches = G.poses.clone(), G.patches.clone()
        ba = ShardedBA(G.ii, G.jj, G.kk, G.patches.shape[0], G.M, 1, G.F, backend=OracleBackend())
        ba(poses, patches, G.intrinsics, G.target, G.weight, torch.tensor([1e-4]), iterations=2)
        own = ba.owned_patches(G.patches.shape[0], G.M)
        torch.save({"poses": poses, "patches": patches, "own": own, "range": ba.own,
                    "bytes": ba.allreduce_bytes}, os.path.join(out, f"r{rank}.pt"))
    finally:
        dist.destroy_process_group()


def test_frame_partition_is_balanced_and_covering():
    from dpvo_amd.fastba.sharded import frame_partition

    kk = torch.arange(96 * 40) % (96 * 40)
    r = frame_partition(kk, 96, 4)
    assert len(r) == 4 and r[0][0] < 0 and r[-1][1] > 10**9
    assert all(r[i][1] == r[i + 1][0] for i in range(3))
    frames = kk // 96
    counts = [int(((frames >= lo) & (frames < hi)).sum()) for lo, hi in r]
    assert sum(counts) == kk.numel() and max(counts) - min(counts) <= 2 * 96


def test_sharded_world2_matches_single_process(tmp_path):
    import oracle

    from dpvo_amd import synthetic

    world = 2
    mp.spawn(_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    res = [torch.load(os.path.join(tmp_path, f"r{r}.pt"), weights_only=True) for r in range(world)]
    G = synthetic.make_config("cfg4s", seed=3)
    Pr, Kr = oracle.ba(G.poses.numpy(), G.patches.numpy(), G.intrinsics.numpy(),
                       G.target.numpy(), G.weight.numpy(), 1e-4, G.ii.numpy(), G.jj.numpy(),
                       G.kk.numpy(), 1, G.F, 2)
    # the ranges split the frames
    assert res[0]["range"][1] == res[1]["range"][0] and 0 < res[0]["range"][1] < G.F
    own0, own1 = res[0]["own"], res[1]["own"]
    assert bool((own0 ^ own1).all())
    for r in res:  # replicated solve: every rank holds the full pose update
        np.testing.assert_allclose(r["poses"].numpy(), Pr, rtol=0, atol=1e-6)
    # inverse depths: each rank updated exactly its own patches
    depth = np.where(own0.numpy()[:, None, None], res[0]["patches"].numpy()[:, 2],
                     res[1]["patches"].numpy()[:, 2])
    np.testing.assert_allclose(depth, Kr[:, 2], rtol=1e-5, atol=1e-6)
    assert not np.allclose(res[0]["patches"].numpy()[own1.numpy(), 2], Kr[own1.numpy(), 2])
    N = G.F - 1
    assert res[0]["bytes"] == 8 * (6 * N + 36 * N * (N + 1) // 2)
