"""GPU parity of fastba (F-BA, F-REPROJ, F-NBR) through the cuda_ba extension
(-> C ABI -> HIP kernels) against the oracle (ba_cuda.cu semantics, pinned to
the reference's ba.py in tests/test_oracle.py).

Tolerances: per-edge math is fp32 on both sides (GPU contracts to FMA, the
oracle does not), every reduction and the solve are fp64 on both sides.
Pose deltas dX: relative 2-norm error <= 1e-4 (north_star); poses after the
update: 2e-5 absolute; inverse depths: 1e-4 relative + 1e-5."""
import numpy as np
import pytest
import torch

import oracle
from conftest import REL_TOL, assert_ba_rel, rel_err
from dpvo_amd import synthetic

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def cb(gpu):
    import dpvo_amd

    return dpvo_amd.load_extension("cuda_ba")


@pytest.fixture(params=[0, 2], ids=["window", "multikernel"])
def path(request, cb):
    """F-BA implementation under test: 0 = auto (ba_window.hip: plan kernel +
    one persistent workgroup per share of a block of S, solve in every
    workgroup), 2 = the multi-kernel path (ba.hip, DPVO windows above 4096
    edges)."""
    cb.select_path(request.param)
    yield request.param
    cb.select_path(0)


def _dev(G, gpu):
    return G.to(gpu)


def _run_gpu(cb, G, gpu, t0, t1, iters, eff=False):
    D = G.to(gpu)
    poses, patches = D.poses.clone(), D.patches.clone()
    lm = torch.tensor([1e-4], device=gpu)
    cb.forward(poses, patches, D.intrinsics, D.target, D.weight, lm, D.ii, D.jj, D.kk, G.M, t0,
               t1, iters, eff)
    return poses.cpu().numpy(), patches.cpu().numpy()


def _run_oracle(G, t0, t1, iters, diag=False):
    return oracle.ba(G.poses.numpy(), G.patches.numpy(), G.intrinsics.numpy(), G.target.numpy(),
                     G.weight.numpy(), 1e-4, G.ii.numpy(), G.jj.numpy(), G.kk.numpy(), t0, t1,
                     iters, diagnostics=diag)


def _check(P, K, Pr, Kr, G=None, t0=0, t1=0):
    if G is not None:  # north_star's 1e-4 relative bar on the deltas (conftest.assert_ba_rel)
        P0, K0 = G.poses.numpy(), G.patches.numpy()
        if t1 > t0:
            assert_ba_rel(P, K, Pr, Kr, P0, K0, t0, t1)
        else:
            assert rel_err(K[:, 2] - K0[:, 2], Kr[:, 2] - K0[:, 2]) <= REL_TOL
    np.testing.assert_allclose(P, Pr, rtol=0, atol=2e-5)
    np.testing.assert_allclose(K[:, 2], Kr[:, 2], rtol=1e-4, atol=1e-5)
    np.testing.assert_array_equal(K[:, :2], Kr[:, :2])  # x, y never change


@pytest.mark.parametrize("cfg,iters", [("cfg1", 1), ("cfg1", 2), ("cfg2", 1), ("cfg2", 2)])
def test_ba_matches_oracle(cb, gpu, path, cfg, iters):
    G = synthetic.make_config(cfg, seed=1)
    t1 = G.F
    P, K = _run_gpu(cb, G, gpu, 1, t1, iters)
    Pr, Kr = _run_oracle(G, 1, t1, iters)
    _check(P, K, Pr, Kr, G, 1, t1)


def test_pose_deltas_relative(cb, gpu):
    # dX through the split entry points vs the oracle's dX: ||d - d_ref|| / ||d_ref|| <= 1e-4
    G = synthetic.make_config("cfg2", seed=2)
    D = G.to(gpu)
    t0, t1 = 1, G.F
    poses, patches = D.poses.clone(), D.patches.clone()
    lm = torch.tensor([1e-4], device=gpu)
    ws = cb.setup(D.ii, D.jj, D.kk, patches.shape[0], t0, t1)
    S, y = cb.build_schur(ws, poses, patches, D.intrinsics, D.target, D.weight, lm, D.ii, D.jj,
                          D.kk, t0, t1)
    dX = cb.solve_update(ws, poses, patches, S, y, G.E, t0, t1).cpu().numpy()
    _, _, d = _run_oracle(G, t0, t1, 1, diag=True)
    rel = np.linalg.norm(dX - d["dX"]) / np.linalg.norm(d["dX"])
    assert rel <= 1e-4, rel
    # the damped lower blocks of S match the oracle's damped dense S
    N = t1 - t0
    Sd = np.zeros((6 * N, 6 * N))
    Sl = S.cpu().numpy()
    t = 0
    for a in range(N):
        for b in range(a + 1):
            Sd[6 * a:6 * a + 6, 6 * b:6 * b + 6] = Sl[t]
            t += 1
    Sd[np.diag_indices(6 * N)] += 1e-4 * Sd[np.diag_indices(6 * N)] + 1.0
    low = np.tril_indices(6 * N)
    np.testing.assert_allclose(Sd[low], d["S"][low], rtol=1e-6, atol=1e-6 * np.abs(d["S"]).max())
    np.testing.assert_allclose(y.cpu().numpy(), d["y"], rtol=1e-6, atol=1e-6 * np.abs(d["y"]).max())


def test_ba_is_deterministic(cb, gpu):
    # the multi-kernel path reduces in a fixed order: bit-identical reruns
    cb.select_path(2)
    try:
        G = synthetic.make_config("cfg2", seed=3)
        a = _run_gpu(cb, G, gpu, 1, G.F, 2)
        b = _run_gpu(cb, G, gpu, 1, G.F, 2)
    finally:
        cb.select_path(0)
    assert np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1])


def test_window_path_is_deterministic(cb, gpu):
    # per-block workgroups reduce in a fixed order, every workgroup sums the
    # partials in the same order: bit-identical reruns
    G = synthetic.make_config("cfg2", seed=3)
    a = _run_gpu(cb, G, gpu, 1, G.F, 2)
    b = _run_gpu(cb, G, gpu, 1, G.F, 2)
    assert np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1])


def test_removed_paths_rejected(cb, gpu):
    # the round-1 single-workgroup (1) and per-block (3) kernels were removed
    for mode in (1, 3):
        with pytest.raises(RuntimeError):
            cb.select_path(mode)
    cb.select_path(0)


def test_eff_impl_flag_is_same_algorithm(cb, gpu, path):
    G = synthetic.make_config("cfg1", seed=4)
    a = _run_gpu(cb, G, gpu, 1, G.F, 2, eff=False)
    b = _run_gpu(cb, G, gpu, 1, G.F, 2, eff=True)
    np.testing.assert_allclose(a[0], b[0], rtol=0, atol=1e-6)
    np.testing.assert_allclose(a[1], b[1], rtol=1e-6, atol=1e-7)


def test_structure_only(cb, gpu, path):
    # t1 == t0: dZ = Q u, poses untouched (ba_cuda.cu:521-531)
    G = synthetic.make_config("cfg1", seed=5)
    P, K = _run_gpu(cb, G, gpu, 3, 3, 2)
    Pr, Kr = _run_oracle(G, 3, 3, 2)
    _check(P, K, Pr, Kr, G, 3, 3)
    np.testing.assert_array_equal(P, G.poses.numpy())


def test_window_with_fixed_poses_and_buffers(cb, gpu, path):
    # optimisation window t0=4 (poses < t0 fixed) inside larger pose/patch buffers
    G = synthetic.make_config("cfg2", seed=6, num_poses=64, num_patches=12 * 96 + 500)
    P, K = _run_gpu(cb, G, gpu, 4, 12, 2)
    Pr, Kr = _run_oracle(G, 4, 12, 2)
    _check(P, K, Pr, Kr, G, 4, 12)
    np.testing.assert_array_equal(P[:4], G.poses.numpy()[:4])
    np.testing.assert_array_equal(P[12:], G.poses.numpy()[12:])


def test_unsorted_edges_and_shuffled_kk(cb, gpu, path):
    G = synthetic.make_config("cfg1", seed=7)
    perm = torch.randperm(G.E, generator=torch.Generator().manual_seed(0))
    for k in ("ii", "jj", "kk", "target", "weight"):
        setattr(G, k, getattr(G, k)[perm].contiguous())
    P, K = _run_gpu(cb, G, gpu, 1, G.F, 2)
    Pr, Kr = _run_oracle(G, 1, G.F, 2)
    _check(P, K, Pr, Kr, G, 1, G.F)


def test_failed_factorisation_gives_zero_step(cb, gpu):
    G = synthetic.make_config("cfg1", seed=8)
    G.weight[:] = float("nan")  # NaN Hessian: Cholesky must fail, dX = 0
    D = G.to(gpu)
    poses = D.poses.clone()
    patches = D.patches.clone()
    lm = torch.tensor([1e-4], device=gpu)
    ws = cb.setup(D.ii, D.jj, D.kk, patches.shape[0], 1, G.F)
    S, y = cb.build_schur(ws, poses, patches, D.intrinsics, D.target, D.weight, lm, D.ii, D.jj,
                          D.kk, 1, G.F)
    dX = cb.solve_update(ws, poses, patches, S, y, G.E, 1, G.F)
    assert int(cb.last_status(ws, G.E, 1, G.F).item()) & 1
    assert torch.count_nonzero(dX) == 0
    assert torch.equal(poses, D.poses)


def test_rejects_fp16_target_like_reference(cb, gpu):
    # ba_cuda.cu:498-500 packed_accessor32<float> rejects fp16 target/weight
    G = synthetic.make_config("cfg1", seed=9).to(gpu)
    lm = torch.tensor([1e-4], device=gpu)
    with pytest.raises(RuntimeError, match="float32"):
        cb.forward(G.poses, G.patches, G.intrinsics, G.target.half(), G.weight, lm, G.ii, G.jj,
                   G.kk, G.M, 1, G.F, 1, False)


def test_empty_graph_is_noop(cb, gpu):
    G = synthetic.make_config("cfg1", seed=10).to(gpu)
    poses = G.poses.clone()
    e = G.ii[:0]
    assert cb.forward(poses, G.patches, G.intrinsics, G.target, G.weight,
                      torch.tensor([1e-4], device=gpu), e, e, e, G.M, 1, G.F, 2, False) == []
    assert torch.equal(poses, G.poses)


@pytest.mark.parametrize("cfg", ["cfg1", "cfg2"])
def test_reproject_matches_oracle(cb, gpu, cfg):
    G = synthetic.make_config(cfg, seed=11)
    D = G.to(gpu)
    c = cb.reproject(D.poses, D.patches, D.intrinsics, D.ii, D.jj, D.kk).cpu().numpy()
    r = oracle.reproject(G.poses.numpy(), G.patches.numpy(), G.intrinsics.numpy(), G.ii.numpy(),
                         G.jj.numpy(), G.kk.numpy())
    assert c.shape == r.shape == (1, G.E, 2, 3, 3)
    np.testing.assert_allclose(c, r, rtol=0, atol=2e-4)


@pytest.mark.parametrize("E", [1, 7, 300, 2048, 5000])
def test_neighbors_matches_oracle(cb, gpu, E):
    r = np.random.default_rng(E)
    ii = r.integers(0, max(2, E // 5), E)
    jj = r.integers(0, 12, E)
    ix, jx = cb.neighbors(torch.from_numpy(ii).to(gpu), torch.from_numpy(jj).to(gpu))
    rx, ry = oracle.neighbors(ii, jj)
    np.testing.assert_array_equal(ix.cpu().numpy(), rx)
    np.testing.assert_array_equal(jx.cpu().numpy(), ry)


def test_fastba_python_surface(gpu):
    # dpvo_amd.fastba.BA mirrors dpvo/fastba/ba.py:7-8 (argument order included)
    from dpvo_amd import fastba

    G = synthetic.make_config("cfg1", seed=12)
    D = G.to(gpu)
    poses, patches = D.poses.clone(), D.patches.clone()
    fastba.BA(poses, patches, D.intrinsics, D.target, D.weight, torch.tensor([1e-4], device=gpu),
              D.ii, D.jj, D.kk, 1, G.F, M=G.M, iterations=2, eff_impl=False)
    Pr, Kr = _run_oracle(G, 1, G.F, 2)
    _check(poses.cpu().numpy(), patches.cpu().numpy(), Pr, Kr, G, 1, G.F)


@pytest.mark.parametrize("seed", [20, 21])
def test_fused_general_graph_structure(cb, gpu, path, seed):
    """Edges whose source pose differs inside one patch, duplicate (kk, jj)
    edges, self edges (ii == jj) and edges touching fixed poses on both sides:
    every E-entry branch of the fused Schur assembly (prim merge, non-prim
    source entries, cross terms) against the oracle."""
    G = synthetic.make_config("cfg1", seed=seed)
    r = np.random.default_rng(seed)
    ii, jj, kk = G.ii.numpy().copy(), G.jj.numpy().copy(), G.kk.numpy().copy()
    E = len(ii)
    sel = r.choice(E, E // 8, replace=False)
    ii[sel] = r.integers(0, G.F, len(sel))          # mixed source poses per patch
    dup = r.choice(E, E // 16, replace=False)
    ii = np.concatenate([ii, ii[dup]]); jj = np.concatenate([jj, jj[dup]])  # duplicates
    kk = np.concatenate([kk, kk[dup]])
    tg = torch.cat([G.target, G.target[dup] + 0.3]); wt = torch.cat([G.weight, G.weight[dup]])
    G.ii, G.jj, G.kk = (torch.from_numpy(x).long() for x in (ii, jj, kk))
    G.target, G.weight = tg.contiguous(), wt.contiguous()
    P, K = _run_gpu(cb, G, gpu, 2, G.F - 1, 2)
    Pr, Kr = _run_oracle(G, 2, G.F - 1, 2)
    _check(P, K, Pr, Kr, G, 2, G.F - 1)


def test_window_solve_precision(cb, gpu):
    """The window kernel's dense solve (fp32 blocked Cholesky + one fp64
    refinement step, ba_solve.hpp) stays at fp64-solve accuracy against the
    fp64 oracle on cfg2 (condition numbers ~2e5)."""
    for seed in (0, 4):
        G = synthetic.make_config("cfg2", seed=seed)
        P, K = _run_gpu(cb, G, gpu, 1, G.F, 2)
        Pr, Kr = _run_oracle(G, 1, G.F, 2)
        _check(P, K, Pr, Kr, G, 1, G.F)
        np.testing.assert_allclose(P, Pr, rtol=0, atol=2e-6)
