"""CholeskySolver (dpvo/ba.py:13-38) on the HIP device: forward vs a direct
fp64 solve, backward vs torch.autograd.gradcheck (fp64), the failure path
(zeros forward, no gradient), and the CPU-tensor refusal."""
import pytest
import torch

from dpvo_amd.ba import CholeskySolver, block_solve


def _spd(n, k, dev, dtype=torch.float64, seed=0):
    g = torch.Generator().manual_seed(seed)
    A = torch.randn(2, n, n, generator=g, dtype=dtype)
    H = A @ A.transpose(-1, -2) + n * torch.eye(n, dtype=dtype)
    b = torch.randn(2, n, k, generator=g, dtype=dtype)
    return H.to(dev), b.to(dev)


@pytest.mark.gpu
def test_forward_matches_direct_solve(gpu):
    H, b = _spd(30, 2, gpu)
    x = CholeskySolver.apply(H, b)
    torch.testing.assert_close(x, torch.linalg.solve(H, b), rtol=1e-10, atol=1e-10)


@pytest.mark.gpu
def test_backward_gradcheck(gpu):
    H, b = _spd(8, 1, gpu)
    H.requires_grad_()
    b.requires_grad_()
    # the reference's backward treats H as a free (not symmetric-constrained)
    # matrix: dH = -x dz^T; gradcheck on the symmetric part fed through
    assert torch.autograd.gradcheck(lambda h, v: CholeskySolver.apply(0.5 * (h + h.transpose(-1, -2)), v),
                                    (H, b), eps=1e-6, atol=1e-5)


@pytest.mark.gpu
def test_failure_returns_zeros_and_no_grad(gpu):
    H, b = _spd(6, 1, gpu)
    H = -H  # not positive definite
    H.requires_grad_()
    x = CholeskySolver.apply(H, b)
    assert torch.count_nonzero(x) == 0
    x.sum().backward()
    assert H.grad is None


@pytest.mark.gpu
def test_block_solve_shapes(gpu):
    A = torch.randn(1, 3, 3, 6, 6, device=gpu, dtype=torch.float64)
    A = A + A.permute(0, 2, 1, 4, 3)
    A = A + 50 * torch.eye(6, device=gpu, dtype=torch.float64).view(1, 1, 1, 6, 6) * \
        torch.eye(3, device=gpu, dtype=torch.float64).view(1, 3, 3, 1, 1)
    B = torch.randn(1, 3, 1, 6, 1, device=gpu, dtype=torch.float64)
    X = block_solve(A, B)
    assert X.shape == (1, 3, 1, 6, 1)


def test_cpu_tensors_are_refused():
    H, b = _spd(4, 1, "cpu")
    with pytest.raises(RuntimeError, match="GPU"):
        CholeskySolver.apply(H, b)
