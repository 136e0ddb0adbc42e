"""DPVO's global BA driver (dpvo_amd/global_ba.py):
__run_global_BA (dpvo/dpvo.py:695-715) = inactive + active edges, fp16
target / weight widened to fp32 (the fork's MIXED_PRECISION buffers, which its
own cuda_ba rejects), PatchGraph.normalize (patchgraph.py:93-106), then
fastba.BA(t0 = min ii, t1 = n, iterations 2, eff_impl=True) on the
large-graph HIP path -- against the oracle: normalize restated in numpy
(float64 SE3 via oracle.lie_fwd) and oracle.ba on the same concatenated
edges, on cfg4s (96 frames, loop blocks).

Tolerances: the scale s is a fp32 mean over n*M*P*P depths (torch's order vs
the oracle's double sum: a few ulp), then the BA tolerances of
tests/test_ba_large_gpu.py widened by that input difference."""
import types

import numpy as np
import pytest
import torch

import oracle
from dpvo_amd import synthetic

pytestmark = pytest.mark.gpu


def _pg(G, gpu, split, fp16):
    """a reference-PatchGraph-shaped object: the first `split` edges of G
    (shuffled) inactive, the rest active; target / weight [1, E, 2]."""
    E = G.E
    perm = torch.randperm(E, generator=torch.Generator().manual_seed(5))
    dt = torch.float16 if fp16 else torch.float32
    cols = {k: getattr(G, k)[perm] for k in ("ii", "jj", "kk", "target", "weight")}
    ns = split
    pg = types.SimpleNamespace()
    pad = 64
    for suf, sl in (("_inac", slice(0, ns)), ("", slice(ns, E))):
        for k in ("ii", "jj", "kk"):
            v = torch.zeros(E + pad, dtype=torch.long)
            v[:sl.stop - sl.start] = cols[k][sl]
            setattr(pg, k + suf, v.to(gpu))
        for k in ("target", "weight"):
            v = torch.zeros(1, E + pad, 2, dtype=dt)
            v[0, :sl.stop - sl.start] = cols[k][sl].to(dt)
            setattr(pg, k + suf, v.to(gpu))
    pg.num_edges, pg.num_edges_inac = E - ns, ns
    order = torch.cat([perm[:ns], perm[ns:]])
    return pg, order


def _oracle_normalize(poses, patches, n, M):
    P = patches.shape[-1]
    K = patches.reshape(-1, M, 3, P, P).astype(np.float32).copy()
    s = np.float32(K[:n, :, 2].astype(np.float64).mean())
    K[:n, :, 2] /= s
    X = poses.astype(np.float32).copy()
    X[:n, :3] *= s
    inv0 = oracle.lie_fwd(3, "inv", X[[0]].astype(np.float64))
    X[:n] = oracle.lie_fwd(3, "mul", X[:n].astype(np.float64),
                           np.repeat(inv0, n, 0)).astype(np.float32)
    return X, K.reshape(patches.shape)


@pytest.mark.parametrize("fp16", [True, False])
def test_global_ba_matches_oracle(gpu, fp16):
    from dpvo_amd.global_ba import run_global_ba

    G = synthetic.make_config("cfg4s", seed=3)
    n, M = G.F, G.M
    pg, order = _pg(G, gpu, split=int(0.4 * G.E), fp16=fp16)
    poses, patches = G.poses.clone().to(gpu), G.patches.clone().to(gpu)
    intr = G.intrinsics.to(gpu)
    used = run_global_ba(pg, poses, patches, intr, n, M)
    assert used == G.E
    torch.cuda.synchronize()
    from dpvo_amd import fastba

    assert fastba.cuda_ba.check_status(poses) == 0

    Xn, Kn = _oracle_normalize(G.poses.numpy(), G.patches.numpy(), n, M)
    tg = G.target[order]
    wg = G.weight[order]
    if fp16:
        tg, wg = tg.half().float(), wg.half().float()
    ii, jj, kk = G.ii[order].numpy(), G.jj[order].numpy(), G.kk[order].numpy()
    t0 = int(ii.min())
    Pr, Kr = oracle.ba(Xn, Kn, G.intrinsics.numpy(), tg.numpy(), wg.numpy(), 1e-4, ii, jj, kk,
                       t0, n, 2)
    P, K = poses.cpu().numpy(), patches.cpu().numpy()
    np.testing.assert_allclose(P, Pr, rtol=0, atol=1e-4)
    np.testing.assert_allclose(K[:, 2], Kr[:, 2], rtol=2e-4, atol=2e-5)
    np.testing.assert_array_equal(K[:, :2], Kr[:, :2])


def test_global_ba_trigger_and_empty(gpu):
    """dpvo.py:815: needs_global_ba on an active edge older than
    n - REMOVAL_WINDOW - 1; with no edge at all, normalize only."""
    from dpvo_amd.global_ba import needs_global_ba, run_global_ba

    G = synthetic.make_config("cfg4s", seed=4)
    pg, _ = _pg(G, gpu, split=0, fp16=False)
    n = G.F
    assert needs_global_ba(pg, n, 20) == bool((G.ii < n - 21).any())
    pg.num_edges = 0
    poses, patches = G.poses.clone().to(gpu), G.patches.clone().to(gpu)
    assert run_global_ba(pg, poses, patches, G.intrinsics.to(gpu), n, G.M) == 0
    Xn, Kn = _oracle_normalize(G.poses.numpy(), G.patches.numpy(), n, G.M)
    np.testing.assert_allclose(poses.cpu().numpy(), Xn, rtol=0, atol=2e-6)
    np.testing.assert_allclose(patches.cpu().numpy(), Kn, rtol=2e-6, atol=0)
