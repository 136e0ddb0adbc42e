"""DPVO.update() data flow on the HIP ops (dpvo_amd/update.py): runs frames
through insertion, device patch-graph bookkeeping, reproject, corr, the
synthetic oracle network, fastba.BA on the optimisation window and keyframe
removal.  Checks the steady-state edge count against DPVO's edge rule, the
BA status, and that the sliding-window BA recovers the scene: inverse depths
initialised to 0.6 converge to the truth once observed, poses stay within
odometry drift of the known trajectory."""
import pytest

pytestmark = pytest.mark.gpu


def test_update_loop_runs_and_converges(gpu):
    from dpvo_amd import fastba
    from dpvo_amd.update import UpdateHarness

    M, r, rw = 8, 13, 22
    h = UpdateHarness(device=gpu, M=M, lifetime=r, removal_window=rw, max_edges=8000,
                      buffer=128, pose_noise=0.0, depth_init=0.6)
    for f in range(40):
        st = h.step()
    # steady state: patches of frames >= n - rw keep their edges; each patch of
    # frame g has edges to frames g-r+1 .. min(g+r-1, n-1) (dpvo.py:838-903)
    n = h.n
    expect = 0
    for g in range(max(n - rw, 0), n):
        lo, hi = max(g - r + 1, 0), min(g + r - 1, n - 1)
        expect += M * (hi - lo + 1)
    assert h.pg.num_edges == expect
    assert fastba.cuda_ba.check_status(h.poses) == 0
    assert st["corr_shape"] == (1, st["edges"], 7 * 7 * 9 * 2)
    # depths of patches observed in many windows: far closer to the truth than
    # the 0.6 initialisation (whose mean error is ~0.2)
    init = float((h.gt_d[:n * M] - 0.6).abs().mean())
    assert h.depth_error(n - 20, n - 12) < 0.25 * init, (h.depth_error(n - 20, n - 12), init)
    assert h.pose_error() < 0.05
