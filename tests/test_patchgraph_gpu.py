"""PatchGraph edge bookkeeping on the device (dpvo_amd/patchgraph.py,
csrc/pg.hip) vs a numpy restatement of the reference's append_factors /
remove_factors (dpvo/dpvo.py:480-568) and of the keyframe window rule
(:684-693): bit-identical index arrays, hidden states, weights, targets and
inactive store after a random sequence of operations, including an append
overflow and a full inactive store."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


class RefPG:
    """dpvo.py:480-568 on numpy arrays (the reference's semantics)."""

    def __init__(self, max_edges, DIM):
        self.max = max_edges
        z = lambda *s, dt=np.float32: np.zeros(s, dt)  # noqa: E731
        self.ii, self.jj, self.kk = (z(max_edges, dt=np.int64) for _ in range(3))
        self.net, self.weight, self.target = z(max_edges, DIM), z(max_edges, 2), z(max_edges, 2)
        self.ii_i, self.jj_i, self.kk_i = (z(max_edges, dt=np.int64) for _ in range(3))
        self.weight_i, self.target_i = z(max_edges, 2), z(max_edges, 2)
        self.n = 0
        self.ni = 0
        self.err = 0

    def append(self, ix, kk, jj):
        k = len(kk)
        if self.n + k > self.max:  # the reference raises; the device flags and skips
            self.err |= 1
            return
        s, e = self.n, self.n + k
        self.jj[s:e], self.kk[s:e], self.ii[s:e] = jj, kk, ix[kk]
        self.net[s:e] = 0
        self.n = e

    def remove(self, m, store):
        m = m[: self.n]
        if store:
            ns = int(m.sum())
            if ns > 0:
                if self.ni + ns > self.max:
                    self.err |= 2
                else:
                    s, e = self.ni, self.ni + ns
                    self.ii_i[s:e], self.jj_i[s:e], self.kk_i[s:e] = (self.ii[:self.n][m],
                                                                      self.jj[:self.n][m],
                                                                      self.kk[:self.n][m])
                    self.weight_i[s:e], self.target_i[s:e] = (self.weight[:self.n][m],
                                                              self.target[:self.n][m])
                    self.ni = e
        keep = ~m
        nk = int(keep.sum())
        if 0 < nk < self.n:
            for a in (self.ii, self.jj, self.kk, self.net, self.weight, self.target):
                a[:nk] = a[:self.n][keep]
        self.n = nk


def _check(dev_pg, ref):
    n, ni = dev_pg.num_edges, dev_pg.num_edges_inac
    assert (n, ni, dev_pg.errors) == (ref.n, ref.ni, ref.err)
    for name, r in (("ii", ref.ii), ("jj", ref.jj), ("kk", ref.kk)):
        np.testing.assert_array_equal(getattr(dev_pg, name)[:n].cpu().numpy(), r[:n], err_msg=name)
    np.testing.assert_array_equal(dev_pg.net[0, :n].cpu().numpy(), ref.net[:n])
    np.testing.assert_array_equal(dev_pg.weight[0, :n].cpu().numpy(), ref.weight[:n])
    np.testing.assert_array_equal(dev_pg.target[0, :n].cpu().numpy(), ref.target[:n])
    for name, r in (("ii_inac", ref.ii_i), ("jj_inac", ref.jj_i), ("kk_inac", ref.kk_i)):
        np.testing.assert_array_equal(getattr(dev_pg, name)[:ni].cpu().numpy(), r[:ni], err_msg=name)
    np.testing.assert_array_equal(dev_pg.weight_inac[0, :ni].cpu().numpy(), ref.weight_i[:ni])


def test_append_remove_sequence_matches_reference(gpu):
    from dpvo_amd.patchgraph import DevicePatchGraph

    rng = np.random.default_rng(0)
    M, DIM, max_edges = 16, 32, 3000
    pg = DevicePatchGraph(max_edges=max_edges, DIM=DIM, device=gpu)
    ref = RefPG(max_edges, DIM)
    ix = np.repeat(np.arange(400), M).astype(np.int64)  # patch -> frame
    ixd = torch.from_numpy(ix).to(gpu)
    for step in range(40):
        n = 10 + step
        if rng.random() < 0.6 or ref.n == 0:  # DPVO-style forward + backward edges of frame n
            r = 5
            kf = np.arange(M * max(n - r, 0), M * n)
            kb = np.arange(M * n, M * (n + 1)).repeat(r)
            jb = np.tile(np.arange(n - r, n), M)
            kk = np.concatenate([kf, kb]).astype(np.int64)
            jj = np.concatenate([np.full(len(kf), n), jb]).astype(np.int64)
            pg.append_factors(ixd, torch.from_numpy(kk).to(gpu), torch.from_numpy(jj).to(gpu))
            ref.append(ix, kk, jj)
            # the update writes weight / target / net of the active edges
            w = rng.standard_normal((max_edges, 2)).astype(np.float32)
            tg = rng.standard_normal((max_edges, 2)).astype(np.float32)
            h = rng.standard_normal((max_edges, DIM)).astype(np.float32)
            pg.weight[0].copy_(torch.from_numpy(w))
            pg.target[0].copy_(torch.from_numpy(tg))
            pg.net[0].copy_(torch.from_numpy(h))
            ref.weight[:], ref.target[:], ref.net[:] = w, tg, h
        elif rng.random() < 0.5:
            m = rng.random(max_edges) < 0.2
            store = bool(rng.random() < 0.7)
            pg.remove_factors(torch.from_numpy(m).to(gpu), store)
            ref.remove(m, store)
        else:  # the keyframe window rule on the device (dpvo.py:684)
            thresh_n, window = n, 8
            m = np.zeros(max_edges, bool)
            m[: ref.n] = ix[ref.kk[: ref.n]] < thresh_n - window
            pg.remove_by_window(ixd, thresh_n, window, store=True)
            ref.remove(m, True)
        _check(pg, ref)
    # overflow: append more than fits -> flagged, nothing added
    big = np.arange(max_edges).astype(np.int64)
    pg.append_factors(ixd, torch.from_numpy(big).to(gpu), torch.from_numpy(big % 7).to(gpu))
    ref.append(ix, big, big % 7)
    _check(pg, ref)


def test_window_rule_spares_loop_closure_edges(gpu):
    from dpvo_amd.patchgraph import DevicePatchGraph

    M = 4
    pg = DevicePatchGraph(max_edges=64, DIM=8, device=gpu, net=False)
    ix = torch.arange(100, device=gpu).repeat_interleave(M)
    kk = torch.tensor([0, 1, 40, 41, 8, 9], device=gpu)  # frames 0, 0, 10, 10, 2, 2
    jj = torch.tensor([45, 3, 12, 46, 50, 4], device=gpu)
    pg.append_factors(ix, kk, jj)
    pg.remove_by_window(ix, n=48, removal_window=22, loop_closure=True, optimization_window=10)
    # ix[kk] < 26 for all; loop-closure spared: jj - ii > 30 and jj > 38
    kept = pg.kk[: pg.num_edges].tolist()
    assert kept == [0, 41, 8] and pg.num_edges_inac == 3
