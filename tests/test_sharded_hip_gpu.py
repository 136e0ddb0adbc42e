"""Edge-sharded global BA (dpvo_amd/fastba/sharded.py) with the HIP backend
under a real collective: two processes share the one GPU of the test box and
all-reduce the packed fp64 (y, S blocks) through gloo (RCCL needs one GPU per
rank; the 8-GPU RCCL run is bench.py --sharded).  Checks the replicated pose
update and the owned inverse depths against the single-process HIP BA, and
the all-reduce byte count the bench reports."""
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
pytestmark = pytest.mark.gpu


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

        dev = torch.device("cuda:0")
        G = synthetic.make_config("cfg4s", seed=3).to(dev)
        poses, patches = G.poses.clone(), G.patches.clone()
        ba = ShardedBA(G.ii, G.jj, G.kk, G.patches.shape[0], G.M, 1, G.F)
        ba(poses, patches, G.intrinsics, G.target, G.weight, torch.tensor([1e-4], device=dev),
           iterations=2)
        st = ba.backend.status(ba.state)[0]
        own = ba.owned_patches(G.patches.shape[0], G.M)
        torch.save({"poses": poses.cpu(), "patches": patches.cpu(), "own": own, "status": st,
                    "bytes": ba.allreduce_bytes}, os.path.join(out, f"r{rank}.pt"))
    finally:
        dist.destroy_process_group()


def test_sharded_hip_world2_matches_single_gpu(gpu, tmp_path):
    from dpvo_amd import fastba, synthetic

    world = 2
    mp.spawn(_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    res = [torch.load(os.path.join(tmp_path, f"r{r}.pt"), weights_only=True) for r in range(world)]
    G = synthetic.make_config("cfg4s", seed=3)
    D = G.to(gpu)
    P, K = D.poses.clone(), D.patches.clone()
    fastba.BA(P, K, D.intrinsics, D.target, D.weight, torch.tensor([1e-4], device=gpu), D.ii,
              D.jj, D.kk, 1, G.F, M=G.M, iterations=2, eff_impl=True)
    P, K = P.cpu().numpy(), K.cpu().numpy()
    assert all(r["status"] == 0 for r in res)
    own0, own1 = res[0]["own"], res[1]["own"]
    assert bool((own0 ^ own1).all())
    for r in res:  # every rank holds the same full pose update
        np.testing.assert_allclose(r["poses"].numpy(), P, rtol=0, atol=2e-6)
    assert torch.equal(res[0]["poses"], res[1]["poses"])  # identical bits after the all-reduce
    depth = np.where(own0.numpy()[:, None, None], res[0]["patches"].numpy()[:, 2],
                     res[1]["patches"].numpy()[:, 2])
    np.testing.assert_allclose(depth, K[:, 2], rtol=1e-5, atol=1e-6)
    assert res[0]["bytes"] == res[1]["bytes"] > 0
