"""DPVO.update() data flow on the HIP ops (dpvo_amd/update.py), SURVEY 8(f1):
insertion, device patch-graph bookkeeping, reproject (+ order + BA plan),
corr levels [1, 4], the deterministic oracle network, fastba.BA on the
optimisation window (iterations=1, the fork's local call dpvo.py:824) and
keyframe-window removal, with MAX_EDGES = 10000 (dpvo/config.py:42).

* the eager loop converges and keeps DPVO's steady-state edge count;
* one frame's corr and BA match the oracle (oracle.corr_fwd, oracle.ba) on
  the harness's own inputs (tolerances of tests/test_corr_gpu.py and
  tests/test_ba_gpu.py);
* the captured update graphs replayed frame after frame give the same bits
  as the eager loop (device frame scalars, no host sync inside a frame)."""
import numpy as np
import pytest
import torch

import oracle
from conftest import assert_ba_rel

pytestmark = pytest.mark.gpu


def _expect_edges(n, M, r=13, rw=22):
    """active edges after the removal of frame n (DPVO's n, dpvo.py:684-693)."""
    tot = 0
    for g in range(max(n - rw, 0), n):
        lo, hi = max(g - r + 1, 0), min(g + r - 1, n - 1)
        tot += M * (hi - lo + 1)
    return tot


def test_update_loop_runs_and_converges(gpu):
    from dpvo_amd.update import UpdateHarness

    M = 8
    h = UpdateHarness(device=gpu, M=M, buffer=128, pose_noise=0.0, depth_init=0.6)
    for f in range(40):
        st = h.step()
    n = h.n
    assert h.pg.num_edges == _expect_edges(n, M)
    assert h.check() == 0
    assert st["corr_shape"] == (1, st["edges"], 7 * 7 * 9 * 2)
    # depths of patches observed in many windows: far closer to the truth than
    # the 0.6 initialisation (whose mean error is ~0.2)
    init = float((h.gt_patches[:n * M, 2, 1, 1] - 0.6).abs().mean())
    assert h.depth_error(n - 20, n - 12) < 0.25 * init, (h.depth_error(n - 20, n - 12), init)
    assert h.pose_error() < 0.05


def test_max_edges_is_the_reference_cap(gpu):
    """M = 20 fits MAX_EDGES = 10000 (497 M = 9940 active edges at the BA);
    M = 21 does not and raises before touching the graph, as the reference's
    append_factors does (dpvo.py:502-507)."""
    from dpvo_amd.update import UpdateHarness

    h = UpdateHarness(device=gpu, M=20, buffer=64)
    for _ in range(40):
        st = h.step()
    assert st["edges"] == 9940 and h.pg.max_edges == 10000
    assert h.check() == 0
    h = UpdateHarness(device=gpu, M=21, buffer=64)
    with pytest.raises(RuntimeError, match="MAX_EDGES"):
        for _ in range(40):
            h.step()


def test_harness_frame_matches_oracle(gpu):
    """One steady-state frame: corr at both levels vs oracle.corr_fwd on the
    frame's own coords, and the BA vs oracle.ba on the frame's own inputs."""
    from dpvo_amd.update import UpdateHarness

    M = 10
    h = UpdateHarness(device=gpu, M=M, buffer=64)
    for _ in range(25):
        h.step()
    h.keep_inputs = True
    n = h.n
    h.step()
    I = h.last_inputs
    E = I["ii"].numel()
    coords = h.last["coords"].cpu().numpy()
    corr = h.last["corr"].view(1, E, 7, 7, 3, 3, 2).cpu().numpy()
    kk, jj = I["kk"].cpu().numpy(), I["jj"].cpu().numpy()
    gm = I["gmap"].cpu().numpy()
    for lvl, s in enumerate(h.levels):
        ref = oracle.corr_fwd(gm, I["pyr"][lvl].cpu().numpy(), coords / s, kk % (M * h.pmem),
                              jj % h.mem, 3)
        got = corr[..., lvl]
        assert np.abs(got - ref).max() <= 1e-5 * max(1.0, np.abs(ref).max())
    t1 = n + 1
    t0 = t1 - I["N"]
    Pr, Kr = oracle.ba(I["poses"].cpu().numpy(), I["patches"].cpu().numpy(),
                       h.intrinsics.cpu().numpy(), I["target"].cpu().numpy(),
                       I["weight"].cpu().numpy(), 1e-4, I["ii"].cpu().numpy(), jj, kk, t0, t1,
                       h.ba_iters)
    P, K = h.poses.cpu().numpy(), h.patches.cpu().numpy()
    # north_star's 1e-4 relative bar on the frame's pose / depth deltas
    assert_ba_rel(P, K, Pr, Kr, I["poses"].cpu().numpy(), I["patches"].cpu().numpy(), t0, t1)
    np.testing.assert_allclose(P, Pr, rtol=0, atol=2e-5)
    np.testing.assert_allclose(K[:, 2], Kr[:, 2], rtol=1e-4, atol=1e-5)
    assert h.check() == 0


def _oracle_ba_dev(poses, patches, intrinsics, target, weight, lmbda, ii, jj, kk, t0_dev, N, plan,
                   iterations=1):
    """fastba.BA_dev with the C oracle (ba_cuda.cu:433-582 restated) doing the
    BA on the host: the reference's BA driving the same harness."""
    t0 = int(t0_dev.item())
    P, K = oracle.ba(poses.cpu().numpy(), patches.cpu().numpy(), intrinsics.cpu().numpy(),
                     target.float().cpu().numpy(), weight.float().cpu().numpy(),
                     float(lmbda.reshape(-1)[0]), ii.cpu().numpy(), jj.cpu().numpy(),
                     kk.cpu().numpy(), t0, t0 + int(N), int(iterations))
    poses.copy_(torch.from_numpy(P))
    patches.copy_(torch.from_numpy(K))
    return []


def _run_harness(gpu, M, frames, ba_iters=1, check_from=None):
    """frames eager steps; from frame check_from on, every frame's BA is also
    compared with oracle.ba on that frame's own inputs (1e-4 relative)."""
    from dpvo_amd.update import UpdateHarness

    h = UpdateHarness(device=gpu, M=M, buffer=frames + 8, ba_iters=ba_iters)
    worst = 0.0
    for f in range(frames):
        h.keep_inputs = check_from is not None and f >= check_from
        n = h.n
        h.step()
        if h.keep_inputs:
            I = h.last_inputs
            t1 = n + 1
            t0 = t1 - I["N"]
            Pr, Kr = oracle.ba(I["poses"].cpu().numpy(), I["patches"].cpu().numpy(),
                               h.intrinsics.cpu().numpy(), I["target"].cpu().numpy(),
                               I["weight"].cpu().numpy(), 1e-4, I["ii"].cpu().numpy(),
                               I["jj"].cpu().numpy(), I["kk"].cpu().numpy(), t0, t1, ba_iters)
            e = assert_ba_rel(h.poses.cpu().numpy(), h.patches.cpu().numpy(), Pr, Kr,
                              I["poses"].cpu().numpy(), I["patches"].cpu().numpy(), t0, t1)
            worst = max(worst, *e.values())
    assert h.check() == 0
    return h, worst


def test_harness_pose_error_bounded_at_m20(gpu, monkeypatch):
    """the scaled window pose error at M = 20 (E = 9440,
    80 frames).  With one BA iteration per frame (the fork's call) the error
    leaves the M <= 15 band (~0.011 m) late in the run; two iterations bring
    it back (~0.010 m).  The growth is the reference algorithm's: every
    frame's BA of the last 20 matches oracle.ba on its own inputs at the
    1e-4 bar, and the whole run with oracle.ba doing every BA ends at the
    same error level."""
    import dpvo_amd.update as upd

    h2, _ = _run_harness(gpu, 20, 80, ba_iters=2)
    e2 = h2.pose_error_scaled()[0]
    del h2
    h1, worst = _run_harness(gpu, 20, 80, ba_iters=1, check_from=60)
    e1 = h1.pose_error_scaled()[0]
    del h1
    monkeypatch.setattr(upd.fastba, "BA_dev", _oracle_ba_dev)
    ho, _ = _run_harness(gpu, 20, 80, ba_iters=1)
    eo = ho.pose_error_scaled()[0]
    print(f"M=20 scaled pose error: 2 iterations {e2:.4f}, 1 iteration {e1:.4f} "
          f"(oracle BA {eo:.4f}); per-frame worst rel {worst:.2e}")
    assert e2 <= 0.015
    assert e1 <= 0.045
    assert abs(e1 - eo) <= 0.25 * eo


def test_graph_replay_matches_eager(gpu):
    """The update captured as hipGraphs (one per ping-pong parity of the
    patch-graph buffers) and replayed for 12 frames gives the same bits as 12
    eager frames: poses, inverse depths, the active edge list and counts."""
    from dpvo_amd.update import UpdateHarness

    M, warm, frames = 10, 36, 12
    a = UpdateHarness(device=gpu, M=M, buffer=64)
    b = UpdateHarness(device=gpu, M=M, buffer=64)
    for _ in range(warm + frames):
        a.step()
    for _ in range(warm):
        b.step()
    assert b.steady()
    b.capture()
    b.replay(frames)
    torch.cuda.synchronize()
    assert a.n == b.n
    assert torch.equal(a.poses, b.poses)
    assert torch.equal(a.patches, b.patches)
    assert torch.equal(a.fs, b.fs)
    E = a.pg.num_edges
    assert E == b.pg.num_edges == _expect_edges(a.n, M)
    for k in ("ii", "jj", "kk"):
        assert torch.equal(getattr(a.pg, k)[:E], getattr(b.pg, k)[:E]), k
    assert a.check() == 0 and b.check() == 0


def test_update_loop_with_device_keyframes(gpu):
    """DPVO's update + keyframe() (dpvo.py:1013-1015) with the frame drop on
    the device: frames are dropped, and every per-frame buffer moved with the
    surviving frames -- the truth, the initial patches' pixel positions and the
    feature rings at index i all belong to timestamp tstamps[i] -- and the BA
    still converges."""
    from dpvo_amd.update import UpdateHarness

    M = 8
    h = UpdateHarness(device=gpu, M=M, buffer=160, pose_noise=0.0, depth_init=0.6,
                      keyframes=True)
    for _ in range(70):
        h.step()
    n = h.n
    assert h.dropped > 0 and n + h.dropped == h.t
    assert int(h.delta[2].item()) == h.dropped
    ts = h.tstamps[:n].cpu()
    assert bool((ts[1:] > ts[:-1]).all()) and int(ts[-1]) == h.t - 1
    tsd = ts.to(gpu)
    assert torch.equal(h.gt_poses[:n], h.gt_poses_t[tsd])
    rows = (tsd.view(-1, 1) * M + torch.arange(M, device=gpu)).view(-1)
    assert torch.equal(h.gt_patches[:n * M], h.gt_patches_t[rows])
    assert torch.equal(h.patches[:n * M, :2], h.init_patches_t[rows, :2])  # BA moves depth only
    # the level-1 ring slot of the last frames holds that frame's features
    for i in range(n - 5, n):
        f = (0.25 * torch.sin(h.field + 0.37 * float(ts[i]))).to(h.feat_dtype)
        assert torch.equal(h.pyr[0][0, i % h.mem], f), i
    # a delta record: (t1, t0) of a dropped frame and its predecessor
    t1, t0 = h.delta[1][0].tolist()
    assert t1 > t0 and int((ts == t1).sum()) == 0
    assert h.check() == 0
    assert h.pose_error_scaled()[0] < 0.05
