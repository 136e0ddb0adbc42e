"""GPU parity of lietorch (L-SE3) through lietorch_backends (-> C ABI -> HIP)
against the oracle's so3.h / se3.h restatement, plus the reference's own
property and gradient tests (dpvo/lietorch/run_tests.py) on the dpvo_amd
groups API."""
import numpy as np
import pytest
import torch

import oracle

pytestmark = pytest.mark.gpu

FWD = [("exp", "expm"), ("log", "logm"), ("inv", "inv"), ("mul", "mul"), ("adj", "adj"),
       ("adjT", "adjT"), ("act", "act"), ("act4", "act4"), ("matrix", "as_matrix"),
       ("projector", "projector"), ("Jinv", "Jinv")]
BWD = [("exp", "expm_backward"), ("log", "logm_backward"), ("inv", "inv_backward"),
       ("mul", "mul_backward"), ("adj", "adj_backward"), ("adjT", "adjT_backward"),
       ("act", "act_backward"), ("act4", "act4_backward")]


@pytest.fixture(scope="module")
def lb(gpu):
    import dpvo_amd

    return dpvo_amd.load_extension("lietorch_backends")


def _inputs(group, op, n=257, seed=0):
    K, N = oracle.GROUP_DIMS[group]
    r = np.random.default_rng(seed)
    if op == "exp":
        x = 0.8 * r.standard_normal((n, K))
        x[:5] *= 1e-9  # small-angle branches
    else:
        x = oracle.lie_fwd(group, "exp", 0.8 * r.standard_normal((n, K)))
        x[:, K - 3 if group == 3 else 0:] *= 1.3  # unnormalised quaternions: normalised on load
        if group == 3:
            x[:, :3] = r.standard_normal((n, 3))
    y = None
    if op == "mul":
        y = oracle.lie_fwd(group, "exp", r.standard_normal((n, K)))
    elif op in ("adj", "adjT", "Jinv"):
        y = r.standard_normal((n, K))
    elif op == "act":
        y = r.standard_normal((n, 3))
    elif op == "act4":
        y = r.standard_normal((n, 4))
    return x, y


@pytest.mark.parametrize("group", [1, 3])
@pytest.mark.parametrize("op,name", FWD)
@pytest.mark.parametrize("dtype", [torch.float64, torch.float32])
def test_forward_matches_oracle(lb, gpu, group, op, name, dtype):
    x, y = _inputs(group, op)
    ref = oracle.lie_fwd(group, op, x, y)
    args = [torch.from_numpy(x).to(gpu, dtype)]
    if y is not None:
        args.append(torch.from_numpy(y).to(gpu, dtype))
    out = getattr(lb, name)(group, *args).reshape(len(x), -1).double().cpu().numpy()
    tol = 1e-10 if dtype == torch.float64 else 2e-4
    np.testing.assert_allclose(out, ref, rtol=tol, atol=tol)


@pytest.mark.parametrize("group", [1, 3])
@pytest.mark.parametrize("op,name", BWD)
def test_backward_matches_oracle(lb, gpu, group, op, name):
    K, N = oracle.GROUP_DIMS[group]
    x, y = _inputs(group, op, seed=1)
    gdim = {"exp": N, "log": K, "inv": N, "mul": N, "adj": K, "adjT": K, "act": 3, "act4": 4}[op]
    g = np.random.default_rng(2).standard_normal((len(x), gdim))
    refs = oracle.lie_bwd(group, op, g, x, y)
    args = [torch.from_numpy(g).to(gpu), torch.from_numpy(x).to(gpu)]
    if y is not None:
        args.append(torch.from_numpy(y).to(gpu))
    outs = getattr(lb, name)(group, *args)
    assert len(outs) == len(refs)
    for o, r in zip(outs, refs):
        np.testing.assert_allclose(o.cpu().numpy(), r, rtol=1e-10, atol=1e-10)


# ---- dpvo/lietorch/run_tests.py on the dpvo_amd groups API (double, GPU) ----
def _groups():
    from dpvo_amd.lietorch import SE3, SO3

    return [SO3, SE3]


@pytest.mark.parametrize("gi", [0, 1])
def test_run_tests_forward_properties(gpu, gi):
    Group = _groups()[gi]
    a = 0.2 * torch.randn(2, 3, 4, 5, Group.manifold_dim, device=gpu).double()
    assert torch.allclose(Group.exp(a).log(), a, atol=1e-8)                      # run_tests.py:16-21
    X = Group.exp(0.1 * torch.randn(2, 3, 4, 5, Group.manifold_dim, device=gpu).double())
    assert torch.allclose((X * X.inv()).log(), torch.zeros_like(a), atol=1e-8)  # :23-28
    X = Group.exp(torch.randn(2, 3, 4, 5, Group.manifold_dim, device=gpu).double())
    b = torch.randn(2, 3, 4, 5, Group.manifold_dim, device=gpu).double()
    c = (Group.exp(X.adj(b)) * X).inv() * (X * Group.exp(b))                      # :30-41
    assert torch.allclose(c.log(), torch.zeros_like(b), atol=1e-8)
    X = Group.exp(torch.randn(1, Group.manifold_dim, device=gpu).double())        # :44-52
    p = torch.randn(1, 3, device=gpu).double()
    p1 = X.act(p)
    p2 = torch.matmul(X.matrix()[0], torch.cat([p[0], torch.ones_like(p[0, :1])]))
    assert torch.allclose(p1[0], p2[:3], atol=1e-8)


@pytest.mark.parametrize("gi", [0, 1])
def test_run_tests_gradients(gpu, gi):
    Group = _groups()[gi]
    D = Group.manifold_dim
    X = Group.exp(0.5 * torch.randn(1, D, device=gpu).double())

    def chk(fn, *inp):
        assert torch.autograd.gradcheck(fn, inp, eps=1e-6, atol=1e-6)

    z = lambda: torch.zeros(1, D, device=gpu, dtype=torch.float64, requires_grad=True)  # noqa
    b = torch.randn(1, D, device=gpu, dtype=torch.float64, requires_grad=True)
    chk(lambda a: Group.exp(a).log(), (0.2 * torch.randn(1, D, device=gpu).double()).requires_grad_())
    chk(lambda a: (Group.exp(a) * X).inv().log(), z())                            # :78-94
    chk(lambda a, bb: (Group.exp(a) * X).adj(bb), z(), b)                         # :97-111
    chk(lambda a, bb: (Group.exp(a) * X).adjT(bb), z(), b)                        # :114-129
    pt = torch.randn(1, 3, device=gpu, dtype=torch.float64, requires_grad=True)
    chk(lambda a, p: (X * Group.exp(a)).act(p), z(), pt)                          # :132-147
    chk(lambda a: (Group.exp(a) * X).matrix(), z())                               # :150-161
    chk(lambda a: (Group.exp(a) * X).translation(), z())                          # :164-178


def test_se3_retr_matches_fastba_retraction(gpu):
    # SE3.retr (Exp(a) * X, groups.py:153-156) == the pose update of cuda_ba
    from dpvo_amd.lietorch import SE3

    X = SE3.exp(torch.randn(16, 6, device=gpu).double())
    a = 0.1 * torch.randn(16, 6, device=gpu).double()
    Y = X.retr(a)
    Z = SE3.exp(a) * X
    assert torch.allclose(Y.data, Z.data, atol=1e-12)


def test_lie_group_parameter(gpu):
    """LieGroupParameter: zero tangent leaf anchored at the group; retr() is
    the anchor, gradients reach the tangent, add_ moves the anchor."""
    from dpvo_amd.lietorch import SE3, LieGroupParameter

    torch.manual_seed(0)
    g = SE3.exp(0.3 * torch.randn(5, 6, device=gpu, dtype=torch.float64))
    p = LieGroupParameter(g)
    assert p.shape == (5, 6) and p.requires_grad and p.is_leaf
    assert torch.allclose(p.retr().data, g.data, atol=1e-12)
    assert torch.allclose(p.log(), g.log(), atol=1e-12)
    assert torch.allclose(p.inv().data, g.inv().data, atol=1e-12)
    (p.retr().log() ** 2).sum().backward()
    assert p.grad is not None and torch.isfinite(p.grad).all() and p.grad.abs().sum() > 0
    step = 0.1 * torch.randn(5, 6, device=gpu, dtype=torch.float64)
    p.add_(step, 0.5)
    assert torch.allclose(p.group.data, (SE3.exp(0.5 * step) * g).data, atol=1e-12)
    q = LieGroupParameter(g)
    assert torch.allclose((p * q).data, (p.group * g).data, atol=1e-12)
