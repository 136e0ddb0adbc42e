"""F-BA on DPVO-realistic local-BA windows and BA status surfacing.

Windows: synthetic.make_dpvo_window builds DPVO's own edge pattern
(dpvo/dpvo.py:838-903: __edges_forw / __edges_back, creation order) over 22
frames with PATCH_LIFETIME 13; M = 10 / 18 / 25 patches per frame give
E = 3940 / 7092 / 9850 edges (MAX_EDGES = 10000, dpvo/config.py:42).  The BA
runs as DPVO's local call does: t0 = n - OPTIMIZATION_WINDOW (10), t1 = n
(dpvo.py:818-824), so edges into the 12 fixed poses take part.
Tolerances: north_star's 1e-4 relative bar on the pose delta, the
inverse-depth delta and the last iteration's pose step dX
(conftest.assert_ba_rel), plus poses 2e-5 abs, inverse depths 1e-4 rel."""
import numpy as np
import pytest
import torch

import oracle
from conftest import assert_ba_rel
from dpvo_amd import synthetic

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def cb(gpu):
    import dpvo_amd

    m = dpvo_amd.load_extension("cuda_ba")
    m.check_status(torch.zeros(1, device=gpu))  # clean slate
    return m


def _run(cb, G, gpu, t0, t1, iters, lm=1e-4, dx=False):
    D = G.to(gpu)
    poses, patches = D.poses.clone(), D.patches.clone()
    fn = cb.forward_dx if dx else cb.forward
    d = fn(poses, patches, D.intrinsics, D.target, D.weight, torch.tensor([lm], device=gpu),
           D.ii, D.jj, D.kk, G.M, t0, t1, iters, False)
    return (poses, patches, d) if dx else (poses, patches)


@pytest.mark.parametrize("M", [10, 18, 25])
@pytest.mark.parametrize("iters", [1, 2])
def test_dpvo_window_matches_oracle(cb, gpu, M, iters):
    G = synthetic.make_dpvo_window(M=M, seed=M)
    n = G.F
    t0, t1 = n - 10, n
    P, K, dX = _run(cb, G, gpu, t0, t1, iters, dx=True)
    assert cb.check_status(P) == 0
    Pr, Kr, d = oracle.ba(G.poses.numpy(), G.patches.numpy(), G.intrinsics.numpy(),
                          G.target.numpy(), G.weight.numpy(), 1e-4, G.ii.numpy(), G.jj.numpy(),
                          G.kk.numpy(), t0, t1, iters, diagnostics=True)
    P, K = P.cpu().numpy(), K.cpu().numpy()
    assert_ba_rel(P, K, Pr, Kr, G.poses.numpy(), G.patches.numpy(), t0, t1, dX.cpu().numpy(),
                  d["dX"])
    np.testing.assert_allclose(P, Pr, rtol=0, atol=2e-5)
    np.testing.assert_allclose(K[:, 2], Kr[:, 2], rtol=1e-4, atol=1e-5)
    np.testing.assert_array_equal(P[:t0], G.poses.numpy()[:t0])  # fixed poses untouched
    # the window moved: the step is not trivially zero
    assert np.abs(P[t0:] - G.poses.numpy()[t0:]).max() > 1e-5


def test_dpvo_window_four_iterations_hbm_entries(cb, gpu):
    """E = 9850 keeps the per-edge E entries in the shared HBM buffer
    (double-buffered by iteration parity): four iterations reuse each parity
    slot twice, against the oracle at the 1e-4 relative bar."""
    G = synthetic.make_dpvo_window(M=25, seed=25)
    t0, t1 = G.F - 10, G.F
    P, K = _run(cb, G, gpu, t0, t1, 4)
    assert cb.check_status(P) == 0
    Pr, Kr = oracle.ba(G.poses.numpy(), G.patches.numpy(), G.intrinsics.numpy(), G.target.numpy(),
                       G.weight.numpy(), 1e-4, G.ii.numpy(), G.jj.numpy(), G.kk.numpy(), t0, t1, 4)
    assert_ba_rel(P.cpu().numpy(), K.cpu().numpy(), Pr, Kr, G.poses.numpy(), G.patches.numpy(),
                  t0, t1)


@pytest.mark.parametrize("iters", [1, 2])
@pytest.mark.parametrize("features", [torch.float32, torch.float16])
def test_bench_call_matches_oracle_rel(cb, gpu, iters, features):
    """The exact call sequence bench.py times on cfg2: the fused frame
    insertion + reprojection + A-CORR edge order + BA plan launch, then
    BA(plan=ws), against the oracle at north_star's 1e-4 relative bar (pose
    delta, inverse-depth delta, last-iteration dX)."""
    from dpvo_amd import altcorr, fastba

    G = synthetic.make_config("cfg2", seed=0)
    D = G.to(gpu)
    t0, t1, mem, levels = 1, G.F, 36, (1, 2, 4, 8)
    pyr_nchw = synthetic.make_features(mem=mem, C=128, levels=levels, seed=0, device=gpu,
                                       dtype=features)
    pyr = [synthetic.channels_last(p) for p in pyr_nchw]
    poses, patches = D.poses.clone(), D.patches.clone()
    lm = torch.tensor([1e-4], device=gpu)
    assert fastba.cuda_ba.plan_supported(G.E, t0, t1, 3)
    coords, order, ws = fastba.reproject(
        poses, patches, D.intrinsics, D.ii, D.jj, D.kk, mem=mem, plan_window=(t0, t1),
        insert=(pyr_nchw[0][0, 3], [p[0, 3] for p in pyr], levels))
    altcorr.corr_levels(torch.zeros(1, mem * G.M, 128, 3, 3, device=gpu, dtype=features), pyr,
                        coords, D.kk % (G.M * mem), D.jj % mem, 3, [float(s) for s in levels],
                        order=order)
    fastba.BA(poses, patches, D.intrinsics, D.target, D.weight, lm, D.ii, D.jj, D.kk, t0, t1,
              M=G.M, iterations=iters, plan=ws)
    dX = cb.last_dx(ws, G.E, t0, t1).cpu().numpy()
    assert cb.check_status(poses) == 0
    Pr, Kr, d = oracle.ba(G.poses.numpy(), G.patches.numpy(), G.intrinsics.numpy(),
                          G.target.numpy(), G.weight.numpy(), 1e-4, G.ii.numpy(), G.jj.numpy(),
                          G.kk.numpy(), t0, t1, iters, diagnostics=True)
    e = assert_ba_rel(poses.cpu().numpy(), patches.cpu().numpy(), Pr, Kr, G.poses.numpy(),
                      G.patches.numpy(), t0, t1, dX, d["dX"])
    assert e["dP"] < 1e-5  # measured: 0 (1 iteration) / 4.2e-6 (2 iterations)


@pytest.mark.parametrize("cfg", ["cfg1", "cfg2"])
def test_planned_forward_is_bit_identical(cb, gpu, cfg):
    """fastba.plan on a side stream + BA(plan=) == BA() (dpvo_ba_plan /
    dpvo_ba_forward_planned vs dpvo_ba_forward)."""
    from dpvo_amd import fastba

    G = synthetic.make_config(cfg, seed=7)
    D = G.to(gpu)
    lm = torch.tensor([1e-4], device=gpu)
    P0, K0 = _run(cb, G, gpu, 1, G.F, 2)
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        ws = fastba.plan(D.ii, D.jj, D.kk, 1, G.F, D.patches.shape[0], D.poses.shape[0])
    assert ws is not None
    torch.cuda.current_stream().wait_stream(side)
    poses, patches = D.poses.clone(), D.patches.clone()
    fastba.BA(poses, patches, D.intrinsics, D.target, D.weight, lm, D.ii, D.jj, D.kk, 1, G.F,
              M=G.M, iterations=2, plan=ws)
    assert torch.equal(poses, P0) and torch.equal(patches, K0)
    assert cb.check_status(poses) == 0


@pytest.mark.parametrize("cfg", ["cfg1", "cfg2", "dpvo10", "dpvo25"])
def test_reproject_plan_fused_is_bit_identical(cb, gpu, cfg):
    """reproject(mem=, plan_window=) (dpvo_reproject_ordered_plan: reprojection,
    A-CORR edge order and BA plan in one launch) == reproject_ordered + plan:
    same coords bits, a valid grouping by target frame, and BA(plan=ws) ==
    BA() bit for bit."""
    from dpvo_amd import fastba

    if cfg.startswith("dpvo"):  # DPVO's edge pattern: E = 3940 (M = 10) / 9850 (M = 25)
        m = int(cfg[4:])
        G = synthetic.make_dpvo_window(M=m, seed=m)
        t0, t1 = G.F - 10, G.F
    else:
        G = synthetic.make_config(cfg, seed=11)
        t0, t1 = 1, G.F
    D = G.to(gpu)
    lm = torch.tensor([1e-4], device=gpu)
    mem = int(D.jj.max().item()) + 1
    c_ref, o_ref = fastba.reproject(D.poses, D.patches, D.intrinsics, D.ii, D.jj, D.kk, mem=mem)
    c, o, ws = fastba.reproject(D.poses, D.patches, D.intrinsics, D.ii, D.jj, D.kk, mem=mem,
                                plan_window=(t0, t1))
    assert torch.equal(c, c_ref)
    # order: a permutation of the edges, grouped by ascending target frame
    assert torch.equal(torch.sort(o.long())[0], torch.arange(D.ii.numel(), device=gpu))
    assert bool((torch.diff(D.jj[o.long()]) >= 0).all())
    assert torch.equal(torch.sort(D.jj[o.long()])[0], torch.sort(D.jj[o_ref.long()])[0])
    P0, K0 = _run(cb, G, gpu, t0, t1, 2)
    poses, patches = D.poses.clone(), D.patches.clone()
    fastba.BA(poses, patches, D.intrinsics, D.target, D.weight, lm, D.ii, D.jj, D.kk, t0, t1,
              M=G.M, iterations=2, plan=ws)
    assert torch.equal(poses, P0) and torch.equal(patches, K0)
    assert cb.check_status(poses) == 0


def test_window_path_covers_dpvo_max_edges(gpu):
    """The window path takes every DPVO local-BA window up to MAX_EDGES =
    10000 (dpvo/config.py:42) with N <= 16 free poses."""
    from dpvo_amd import fastba

    for E in (3940, 7092, 9850, 10000):
        assert fastba.cuda_ba.plan_supported(E, 12, 22, 3)
    assert fastba.cuda_ba.plan_supported(10000, 0, 16, 3)
    assert not fastba.cuda_ba.plan_supported(10241, 12, 22, 3)
    assert not fastba.cuda_ba.plan_supported(4000, 0, 17, 3)


def test_reproject_plan_fused_unsupported_window_raises(gpu):
    """Outside the window path (E > 10240) the fused launch reports
    unsupported (as fastba.plan returns None there) and writes nothing."""
    from dpvo_amd import fastba

    G = synthetic.make_dpvo_window(M=27, seed=27)  # E > 10240
    D = G.to(gpu)
    assert D.ii.numel() > 10240
    assert not fastba.cuda_ba.plan_supported(int(D.ii.numel()), G.F - 10, G.F, 3)
    with pytest.raises(RuntimeError, match="unsupported"):
        fastba.reproject(D.poses, D.patches, D.intrinsics, D.ii, D.jj, D.kk, mem=G.F,
                         plan_window=(G.F - 10, G.F))


def test_bad_patch_index_raises(cb, gpu):
    G = synthetic.make_config("cfg1", seed=3)
    G.kk = G.kk.clone()
    G.kk[5] = G.patches.shape[0] + 7  # outside [0, num_patches): clamped on the device
    _run(cb, G, gpu, 1, G.F, 1)
    with pytest.raises(RuntimeError, match="status"):
        cb.check_status(G.poses.to(gpu))
    # the accumulator was reset by the raise: a clean call reports 0
    _run(cb, synthetic.make_config("cfg1", seed=4), gpu, 1, 8, 1)
    assert cb.check_status(G.poses.to(gpu)) == 0


def test_deferred_status_raises_on_next_forward(cb, gpu):
    G = synthetic.make_config("cfg1", seed=5)
    bad = synthetic.make_config("cfg1", seed=5)
    bad.kk = bad.kk.clone()
    bad.kk[0] = -3
    _run(cb, bad, gpu, 1, bad.F, 1)
    torch.cuda.synchronize()  # the status copy has landed
    with pytest.raises(RuntimeError, match="kk outside"):
        _run(cb, G, gpu, 1, G.F, 1)
    assert cb.check_status(G.poses.to(gpu)) == 0


def test_failed_factorisation_is_reported_not_raised(cb, gpu):
    G = synthetic.make_config("cfg1", seed=6)
    G.weight[:] = float("nan")
    P, _ = _run(cb, G, gpu, 1, G.F, 1)
    assert cb.check_status(P) & 1
    assert torch.equal(P.cpu(), G.poses)  # zero step (dpvo/ba.py:17-21)


def test_large_graph_structure_limit_raises(cb, gpu):
    # global BA (N > 16 free poses -> large-graph solver): one patch observed
    # from 40 free frames exceeds the per-patch free-pose set it handles
    G = synthetic.make_config("cfg4s", seed=1)
    k0 = int(G.kk[0])
    extra_j = torch.arange(2, 42)
    G.kk = torch.cat([G.kk, torch.full_like(extra_j, k0)])
    G.ii = G.kk // G.M
    G.jj = torch.cat([G.jj, extra_j])
    G.target = torch.cat([G.target, G.target[:1].repeat(len(extra_j), 1)])
    G.weight = torch.cat([G.weight, G.weight[:1].repeat(len(extra_j), 1)])
    _run(cb, G, gpu, 1, G.F, 1)
    with pytest.raises(RuntimeError, match="status"):
        cb.check_status(G.poses.to(gpu))


def _host_grouping(ii, jj, kk, t0, t1):
    """numpy restatement of the plan: patches in ascending kk, edges of a
    patch in ascending edge index, free-pose bits of t0 <= ii/jj < t1."""
    order = np.lexsort((np.arange(kk.size), kk))
    uk, first = np.unique(kk[order], return_index=True)
    poff = np.append(first, kk.size)
    N = t1 - t0
    bits = np.zeros(kk.size, np.uint32)
    for x in (ii, jj):
        free = (x >= t0) & (x < t1)
        bits |= np.where(free, np.left_shift(1, np.clip(x - t0, 0, 31)), 0).astype(np.uint32)
    pmask = np.array([np.bitwise_or.reduce(bits[order[poff[u]:poff[u + 1]]])
                      for u in range(uk.size)], np.uint32)
    assert N <= 16
    return order.astype(np.int32), poff.astype(np.int32), pmask, uk.astype(np.int32)


def _check_block_work(meta, ref, N):
    """The sharded plan's block work (meta[64 + lblk(a, b) * 16 + s], shards
    s < meta[3]): edges of the patches whose free-pose mask holds a and b."""
    nsh = int(meta[3])
    if nsh == 0:  # single-workgroup plan: no partials (the kernel splits evenly)
        return
    got = meta[64:64 + 16 * 136].reshape(136, 16)[:, :nsh].sum(1)
    want = np.zeros(136, np.int64)
    poff, pmask = ref[1], ref[2]
    for u in range(pmask.size):
        c, m = int(poff[u + 1] - poff[u]), int(pmask[u])
        bits = [x for x in range(N) if (m >> x) & 1]
        for x in bits:
            for y in bits:
                if y <= x:
                    want[x * (x + 1) // 2 + y] += c
    np.testing.assert_array_equal(got[:N * (N + 1) // 2], want[:N * (N + 1) // 2])


def _plan_arrays(cb, ws, E, t0, t1):
    off = cb.plan_offsets(E, t0, t1)
    b = ws.cpu().numpy()

    def arr(k, n, dt):
        return np.frombuffer(b[off[k]:off[k] + 4 * n].tobytes(), dt)

    meta = arr(4, 64 + 16 * 136, np.int32)  # kMetaWork + kPlanShardMax * kWMaxNB
    nuniq = int(meta[0])
    return (arr(0, E, np.int32), arr(1, nuniq + 1, np.int32), arr(2, nuniq, np.uint32),
            arr(3, nuniq, np.int32), nuniq, meta)


@pytest.mark.parametrize("E,nk,M,seed", [(96, 40, 1024, 0), (700, 650, 1024, 1),
                                         (3000, 2500, 1024, 2), (4096, 300, 1024, 3),
                                         (4000, 3900, 1024, 4), (2048, 1500, 2048, 5),
                                         (10000, 9000, 1024, 6), (10240, 550, 1024, 7),
                                         (6000, 5000, 4096, 8), (9850, 9000, 4096, 9)])
def test_plan_grouping_matches_host(cb, gpu, E, nk, M, seed):
    """Regression for the plan's counting sort (the head flags of every
    bucket are read before any wave bumps a bucket counter): many small
    buckets and E > 64, through fastba.plan and the fused reprojection launch,
    the grouping is exactly the host one, on repeated calls; E > 512 runs the
    sharded plan (one workgroup per kk range) when the kk range fits the
    counting sort.  M = 2048 / 4096
    put the kk range past the counting sort's (bitonic path: 64-bit keys up
    to E = 8192, packed 32-bit keys above)."""
    from dpvo_amd import fastba

    rng = np.random.default_rng(seed)
    F = 12
    t0, t1 = 1, F
    base = np.sort(rng.choice(F * M, nk, replace=False))
    kk = np.concatenate([base, base[rng.integers(0, nk, E - nk)]])
    kk = rng.permutation(kk).astype(np.int64)
    ii = kk // M
    jj = rng.integers(0, F, E).astype(np.int64)
    ref = _host_grouping(ii, jj, kk, t0, t1)
    both = np.concatenate([ii, jj])
    fixed = both[(both < t0) | (both >= t1)]
    fmin = int(np.clip(fixed.min(), 0, F - 1)) if fixed.size else 2 ** 31 - 1
    D = [torch.from_numpy(x).to(gpu) for x in (ii, jj, kk)]
    for rep in range(3):
        ws = fastba.plan(*D, t0, t1, F * M, F)
        assert ws is not None
        epos, poff, pmask, pkk, nuniq, meta = _plan_arrays(cb, ws, E, t0, t1)
        assert nuniq == ref[3].size
        assert int(meta[1]) == fmin and int(meta[2]) == 0  # smallest fixed pose, no clamp
        _check_block_work(meta, ref, t1 - t0)
        np.testing.assert_array_equal(pkk, ref[3])
        np.testing.assert_array_equal(poff, ref[1])
        np.testing.assert_array_equal(epos, ref[0])
        np.testing.assert_array_equal(pmask, ref[2])
    # the same grouping from workgroup 0 of the fused reprojection launch
    poses = torch.zeros(F, 7, device=gpu)
    poses[:, 6] = 1
    patches = torch.ones(F * M, 3, 3, 3, device=gpu)
    intr = torch.tensor([[80.0, 80.0, 80.0, 60.0]], device=gpu).repeat(F, 1)
    _, _, ws = fastba.reproject(poses, patches, intr, *D, mem=F, plan_window=(t0, t1))
    epos, poff, pmask, pkk, nuniq, meta = _plan_arrays(cb, ws, E, t0, t1)
    assert nuniq == ref[3].size and int(meta[1]) == fmin
    np.testing.assert_array_equal(poff, ref[1])
    np.testing.assert_array_equal(epos, ref[0])
    np.testing.assert_array_equal(pkk, ref[3])
    np.testing.assert_array_equal(pmask, ref[2])


@pytest.mark.parametrize("cfg,dtype", [("cfg2", torch.float32), ("cfg2", torch.float16),
                                       ("dpvo25", torch.float32)])
def test_reproject_plan_insert_fused_is_bit_identical(cb, gpu, cfg, dtype):
    """reproject(mem=, plan_window=, insert=) (dpvo_reproject_ordered_plan_insert:
    the new frame's pyramid insertion in the reprojection + plan launch) ==
    reproject(mem=, plan_window=) + altcorr.insert_frame: coords, the order's
    grouping, the plan (BA(plan=ws) bits) and every written pyramid slot."""
    from dpvo_amd import altcorr, fastba

    if cfg == "dpvo25":  # E = 9850: the plan sized for E near MAX_EDGES
        G = synthetic.make_dpvo_window(M=25, seed=25)
        t0, t1 = G.F - 10, G.F
    else:
        G = synthetic.make_config(cfg, seed=12)
        t0, t1 = 1, G.F
    D = G.to(gpu)
    mem, levels = G.F + 2, (1, 2, 4, 8)
    pyr_nchw = synthetic.make_features(mem=mem, C=128, levels=levels, seed=3, device=gpu,
                                       dtype=dtype)
    pa = [synthetic.channels_last(p).clone() for p in pyr_nchw]
    pb = [synthetic.channels_last(p).clone() for p in pyr_nchw]
    src = torch.randn(128, pyr_nchw[0].shape[3], pyr_nchw[0].shape[4], device=gpu).to(dtype)
    slot = 5
    c_ref, o_ref, ws_ref = fastba.reproject(D.poses, D.patches, D.intrinsics, D.ii, D.jj, D.kk,
                                            mem=mem, plan_window=(t0, t1))
    altcorr.insert_frame(src, pa, slot, levels)
    c, o, ws = fastba.reproject(D.poses, D.patches, D.intrinsics, D.ii, D.jj, D.kk, mem=mem,
                                plan_window=(t0, t1),
                                insert=(src, [p[0, slot] for p in pb], levels))
    torch.cuda.synchronize()
    assert torch.equal(c, c_ref)
    # order: a grouping by target frame (the order inside a group is not fixed)
    assert torch.equal(torch.sort(o.long())[0], torch.arange(D.ii.numel(), device=gpu))
    assert torch.equal(D.jj[o.long()] % mem, D.jj[o_ref.long()] % mem)
    for a, b in zip(pa, pb):
        assert torch.equal(a, b)
    lm = torch.tensor([1e-4], device=gpu)
    outs = []
    for w in (ws_ref, ws):
        poses, patches = D.poses.clone(), D.patches.clone()
        fastba.BA(poses, patches, D.intrinsics, D.target, D.weight, lm, D.ii, D.jj, D.kk, t0, t1,
                  M=G.M, iterations=2, plan=w)
        outs.append((poses, patches))
    assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1])
    assert cb.check_status(D.poses) == 0
